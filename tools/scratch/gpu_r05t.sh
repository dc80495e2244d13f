# round 5: grid re-sweep on the current build: update blocks 2048 (default 1024), GRID_MAX 4096
# (default 2048: the sparse push, list passes and other grid-stride kernels)
set -o pipefail
mkdir -p gpurun_out/r05t
export TMPDIR=/tmp
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05t 4096 3 default env:P2PG_UPDATE_GRID=2048 env:P2PG_GRID_MAX=4096 > gpurun_out/r05t/ab.txt 2>&1 || { cat gpurun_out/r05t/ab.txt; exit 1; }
cat gpurun_out/r05t/ab.txt
