# round 4: grouped fused kernel (W <= 16 shares) launch bounds 4 (default) vs 3 waves per SIMD
set -o pipefail
AB_STEPS=6 bash tools/gpu_bench_ab.sh r04y 512 3 default g3 || exit 1
AB_STEPS=6 bash tools/gpu_bench_ab.sh r04y 1024 3 default g3 || exit 1
