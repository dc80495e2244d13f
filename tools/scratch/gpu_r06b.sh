# round 6: RCCL exchange through TorchTransport, received counter, gossip restore + update at W = 16/64
set -o pipefail
mkdir -p gpurun_out/r06b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_dynamic.py tests/test_gpu_parity.py tests/test_gpu_partition.py -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread -p no:cacheprovider -k "not config4 and not config3" > gpurun_out/r06b/pytest.log 2>&1 || { tail -40 gpurun_out/r06b/pytest.log; exit 1; }
tail -22 gpurun_out/r06b/pytest.log
