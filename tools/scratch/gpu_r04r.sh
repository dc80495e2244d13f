# round 4: dense-entry peer threshold v re-swept at the split shares W = 32 / 16 (default 0.95)
set -o pipefail
AB_STEPS=5 bash tools/gpu_bench_ab.sh r04r 2048 2 default env:P2PG_V_THRESH=0.5 env:P2PG_V_THRESH=0.8 || exit 1
AB_STEPS=5 bash tools/gpu_bench_ab.sh r04r 1024 2 default env:P2PG_V_THRESH=0.5 env:P2PG_V_THRESH=0.8 || exit 1
