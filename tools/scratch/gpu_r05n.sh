# round 5: coalesced chunk scan (default) vs the thread-major one (variants/scan0); parity first
set -o pipefail
mkdir -p gpurun_out/r05n
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_run_modes.py tests/test_gpu_parity.py > gpurun_out/r05n/tests.log 2>&1 || { tail -30 gpurun_out/r05n/tests.log; exit 1; }
tail -3 gpurun_out/r05n/tests.log
AB_STEPS=10 bash tools/gpu_bench_ab.sh r05n 4096 3 default scan0 > gpurun_out/r05n/ab.txt 2>&1 || { cat gpurun_out/r05n/ab.txt; exit 1; }
cat gpurun_out/r05n/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05n/trace -o c4 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05n/trace_bench.json 2> gpurun_out/r05n/trace.err || { tail -20 gpurun_out/r05n/trace.err; exit 1; }
echo trace ok
