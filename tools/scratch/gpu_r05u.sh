# round 5: GRID_MAX 4096 / 8192 vs the default 2048 (sparse push and the other grid-stride kernels)

set -o pipefail
mkdir -p gpurun_out/r05u
export TMPDIR=/tmp
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05u 4096 3 default env:P2PG_GRID_MAX=4096 env:P2PG_GRID_MAX=8192 > gpurun_out/r05u/ab.txt 2>&1 || { cat gpurun_out/r05u/ab.txt; exit 1; }
cat gpurun_out/r05u/ab.txt
