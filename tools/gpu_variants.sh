# Per-round profile of kernel variants (A/B): default build first with the GPU parity suite.
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/round_profile.py c4 1 > gpurun_out/rounds_c4.json 2> gpurun_out/rounds_c4.err || { tail -20 gpurun_out/rounds_c4.err; exit 1; }
for v in "$@"; do
  P2PG_LIB=python-p2p-network_amd/csrc/variants/$v/libp2pgpu.so timeout -k 10 300 python tools/round_profile.py c4 1 > gpurun_out/rounds_c4_$v.json 2> gpurun_out/rounds_c4_$v.err || { tail -20 gpurun_out/rounds_c4_$v.err; exit 1; }
done
echo done
