# round 4: schedule changes (blind sparse pushes, decay-aware last dense round, batched tail)
set -o pipefail
mkdir -p gpurun_out/r04f
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_run_modes.py tests/test_gpu_fullsize.py tests/test_gpu_split.py tests/test_gpu_parity.py > gpurun_out/r04f/pt.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r04f/pt.log | head -20; tail -5 gpurun_out/r04f/pt.log; exit 1; }
tail -1 gpurun_out/r04f/pt.log
AB_STEPS=8 bash tools/gpu_bench_ab.sh r04f 4096 3 default env:P2PG_RUN_BATCH=1
