# round 5: fused gathers in flight FG = 6 (variants/fg6) vs 8 under the 3-wave launch bound
set -o pipefail
mkdir -p gpurun_out/r05ad
export TMPDIR=/tmp
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05ad 4096 3 default fg6 > gpurun_out/r05ad/ab.txt 2>&1 || { cat gpurun_out/r05ad/ab.txt; exit 1; }
cat gpurun_out/r05ad/ab.txt
