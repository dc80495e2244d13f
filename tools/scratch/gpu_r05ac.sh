# round 5: fused-kernel grid multiplier re-swept on the final build (P2PG_FUSED_GRID 24 / 48 vs 32)
set -o pipefail
mkdir -p gpurun_out/r05ac
export TMPDIR=/tmp
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05ac 4096 3 default env:P2PG_FUSED_GRID=24 env:P2PG_FUSED_GRID=48 > gpurun_out/r05ac/ab.txt 2>&1 || { cat gpurun_out/r05ac/ab.txt; exit 1; }
cat gpurun_out/r05ac/ab.txt
