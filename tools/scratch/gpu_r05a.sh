# round 5, first call: baseline bench line on this build + a kernel trace of 3 bench steps
# (host gaps between kernels of a step)
set -o pipefail
mkdir -p gpurun_out/r05a
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05a/bench_c4.json 2> gpurun_out/r05a/bench_c4.err || { tail -20 gpurun_out/r05a/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05a/bench_c4.json')); print(round(d['ms_per_step'],2), {k: round(v,2) for k, v in d['kernel_ms_per_step'].items() if v})"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05a/trace -o c4 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05a/trace_bench.json 2> gpurun_out/r05a/trace.err || { tail -20 gpurun_out/r05a/trace.err; exit 1; }
echo trace ok
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -s > gpurun_out/r05a/rccl.log 2>&1 || { tail -40 gpurun_out/r05a/rccl.log; exit 1; }
tail -3 gpurun_out/r05a/rccl.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_run_modes.py -x -v --timeout 380 --timeout-method thread -p no:cacheprovider --durations 5 > gpurun_out/r05a/run_modes.log 2>&1 || { tail -40 gpurun_out/r05a/run_modes.log; exit 1; }
tail -3 gpurun_out/r05a/run_modes.log
