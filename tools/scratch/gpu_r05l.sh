# round 5: 64 stats shards + batched fused rounds (default) vs 8 shards (variants/sh8), no dense
# batches (P2PG_DENSE_BATCH=0) and the 9bb415f build (variants/base); then a kernel trace
set -o pipefail
mkdir -p gpurun_out/r05l
export TMPDIR=/tmp
AB_STEPS=10 bash tools/gpu_bench_ab.sh r05l 4096 3 default sh8 env:P2PG_DENSE_BATCH=0 base > gpurun_out/r05l/ab.txt 2>&1 || { cat gpurun_out/r05l/ab.txt; exit 1; }
cat gpurun_out/r05l/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05l/trace -o c4 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05l/trace_bench.json 2> gpurun_out/r05l/trace.err || { tail -20 gpurun_out/r05l/trace.err; exit 1; }
echo trace ok
