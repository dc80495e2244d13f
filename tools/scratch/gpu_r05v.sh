# round 5: sparse launches up to 8192 blocks (default) vs 2048 (variants/sg2048); parity first
set -o pipefail
mkdir -p gpurun_out/r05v
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_run_modes.py "tests/test_gpu_fullsize.py::test_gossip_full_width_1m_matches_c_oracle" "tests/test_gpu_fullsize.py::test_gossip_wide_rows_hubs_churn_match_c_oracle" tests/test_gpu_parity.py > gpurun_out/r05v/tests.log 2>&1 || { tail -30 gpurun_out/r05v/tests.log; exit 1; }
tail -3 gpurun_out/r05v/tests.log
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05v 4096 3 default sg2048 > gpurun_out/r05v/ab.txt 2>&1 || { cat gpurun_out/r05v/ab.txt; exit 1; }
cat gpurun_out/r05v/ab.txt
for m in 2048 512; do
  timeout -k 10 200 python bench.py --steps 8 --warmup 2 --msgs $m --no-cpu-baseline > gpurun_out/r05v/bench_c4_m$m.json 2> gpurun_out/r05v/bench_c4_m$m.err || { tail -20 gpurun_out/r05v/bench_c4_m$m.err; exit 1; }
  P2PG_LIB=python-p2p-network_amd/csrc/variants/sg2048/libp2pgpu.so timeout -k 10 200 python bench.py --steps 8 --warmup 2 --msgs $m --no-cpu-baseline > gpurun_out/r05v/bench_c4_m${m}_sg2048.json 2> gpurun_out/r05v/bench_c4_m${m}_sg2048.err || { tail -20 gpurun_out/r05v/bench_c4_m${m}_sg2048.err; exit 1; }
  python3 -c "import json,sys; [print(f, round(json.load(open(f))['ms_per_step'],1), {k: round(v,1) for k, v in json.load(open(f))['kernel_ms_per_step'].items() if v}) for f in sys.argv[1:]]" gpurun_out/r05v/bench_c4_m$m.json gpurun_out/r05v/bench_c4_m${m}_sg2048.json
done
