# round 4: gathers in flight (P2PG_FG 8 default / 10 / 12) under the 3-wave launch bound -- c4 A/B
set -o pipefail
AB_STEPS=6 bash tools/gpu_bench_ab.sh r04aa 4096 3 default fg10 fg12 || exit 1
