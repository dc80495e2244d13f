# round 5: dense-entry / exit thresholds re-swept on the current build (c4, interleaved)
set -o pipefail
mkdir -p gpurun_out/r05i
export TMPDIR=/tmp
AB_STEPS=10 bash tools/gpu_bench_ab.sh r05i 4096 2 default env:P2PG_E_THRESH=0.05 env:P2PG_E_THRESH=0.07 env:P2PG_E_THRESH=0.08 env:P2PG_V_THRESH=0.5 env:P2PG_DECAY_PRED=0 > gpurun_out/r05i/ab.txt 2>&1 || { cat gpurun_out/r05i/ab.txt; exit 1; }
cat gpurun_out/r05i/ab.txt
