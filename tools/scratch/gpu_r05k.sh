# round 5: grid knobs re-swept on the current build (c4, interleaved)
set -o pipefail
mkdir -p gpurun_out/r05k
export TMPDIR=/tmp
AB_STEPS=10 bash tools/gpu_bench_ab.sh r05k 4096 2 default env:P2PG_UPDATE_GRID=2048 env:P2PG_UPDATE_GRID=4096 env:P2PG_UPDATE_GRID=512 env:P2PG_FUSED_GRID=16 env:P2PG_FUSED_GRID=64 > gpurun_out/r05k/ab.txt 2>&1 || { cat gpurun_out/r05k/ab.txt; exit 1; }
cat gpurun_out/r05k/ab.txt
