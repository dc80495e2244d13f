# round 5: HIP API trace next to the kernel trace (where the ~30 us host gaps between rounds go)
set -o pipefail
mkdir -p gpurun_out/r05o
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/r05o/trace -o c4 -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r05o/trace_bench.json 2> gpurun_out/r05o/trace.err || { tail -20 gpurun_out/r05o/trace.err; exit 1; }
ls -la gpurun_out/r05o/trace/*/ 2>/dev/null || find gpurun_out/r05o/trace -type f | head
