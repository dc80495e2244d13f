# round 5: double-buffered seen plane (default) vs P2PG_SEEN_SPARE=0; reset-heavy parity tests first
set -o pipefail
mkdir -p gpurun_out/r05m
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_run_modes.py tests/test_gpu_parity.py > gpurun_out/r05m/tests.log 2>&1 || { tail -30 gpurun_out/r05m/tests.log; exit 1; }
tail -3 gpurun_out/r05m/tests.log
AB_STEPS=10 bash tools/gpu_bench_ab.sh r05m 4096 3 default env:P2PG_SEEN_SPARE=0 > gpurun_out/r05m/ab.txt 2>&1 || { cat gpurun_out/r05m/ab.txt; exit 1; }
cat gpurun_out/r05m/ab.txt
