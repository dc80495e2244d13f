# round 5: round-0 counters cached per sources (no host sort while the GPU waits, no round-0
# read-back before the push) + numpy conversion of p2pg_run's rounds; vs variants/head (c477e33)
set -o pipefail
mkdir -p gpurun_out/r05p
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_run_modes.py tests/test_gpu_parity.py tests/test_gpu_dynamic.py > gpurun_out/r05p/tests.log 2>&1 || { tail -30 gpurun_out/r05p/tests.log; exit 1; }
tail -3 gpurun_out/r05p/tests.log
AB_STEPS=10 bash tools/gpu_bench_ab.sh r05p 4096 3 default head > gpurun_out/r05p/ab.txt 2>&1 || { cat gpurun_out/r05p/ab.txt; exit 1; }
cat gpurun_out/r05p/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/r05p/trace -o c4 -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r05p/trace_bench.json 2> gpurun_out/r05p/trace.err || { tail -20 gpurun_out/r05p/trace.err; exit 1; }
echo trace ok
