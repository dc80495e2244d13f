# round 4: fused kernel at 3 waves per SIMD (P2PG_FUSED_WAVES=3: ~170 VGPRs, no spills) vs 4 -- A/B
set -o pipefail
AB_STEPS=6 bash tools/gpu_bench_ab.sh r04w 4096 3 default w3 || exit 1
