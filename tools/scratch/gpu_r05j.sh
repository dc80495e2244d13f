# round 5: kernel trace + stats of the current build (bench c4, 3 timed steps)
set -o pipefail
mkdir -p gpurun_out/r05j
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05j/trace -o c4 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05j/trace_bench.json 2> gpurun_out/r05j/trace.err || { tail -20 gpurun_out/r05j/trace.err; exit 1; }
echo trace ok
