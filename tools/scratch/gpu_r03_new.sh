# Round-3 additions on the GPU: bench --gpus spawn, stream-ordered partition exchange,
# quiescent-run deliveries, config-3 full-size oracle check.
#   bash tools/gpu_r03_new.sh <tag>
set -o pipefail
tag=${1:-r03a}
mkdir -p gpurun_out/$tag
timeout -k 10 1000 python -u -m pytest -x -v --timeout 700 --timeout-method thread -m gpu \
  tests/test_bench_launch.py tests/test_gpu_partition.py tests/test_gpu_fullsize.py \
  -k "bench or partition or quiescent or config3 or run_chunks" > gpurun_out/$tag/pytest_new.log 2>&1 \
  || { tail -60 gpurun_out/$tag/pytest_new.log; exit 1; }
tail -3 gpurun_out/$tag/pytest_new.log
