# round 4: fused kernel waves per SIMD (P2PG_FUSED_WAVES 4 default / 3 / 2) on c4 and the W = 32 / 16 shares
set -o pipefail
AB_STEPS=6 bash tools/gpu_bench_ab.sh r04x 4096 2 default w3 w2 || exit 1
AB_STEPS=6 bash tools/gpu_bench_ab.sh r04x 2048 2 default w3 w2 || exit 1
AB_STEPS=6 bash tools/gpu_bench_ab.sh r04x 1024 2 default w3 || exit 1
