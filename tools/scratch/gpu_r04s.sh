# round 4: gathers in flight per target in the fused kernel (P2PG_FG, default 8) -- interleaved A/B
set -o pipefail
AB_STEPS=6 bash tools/gpu_bench_ab.sh r04s 4096 3 default fg6 fg12 || exit 1
AB_STEPS=6 bash tools/gpu_bench_ab.sh r04s 2048 2 default fg6 fg12 || exit 1
