# round 4: push-time dedup in every sparse round (P2PG_PUSH_DEDUP=1) vs the decay-phase-only default,
# c4 and its message-split shares -- interleaved A/B
set -o pipefail
for m in 512 1024 2048 4096; do
  AB_STEPS=6 bash tools/gpu_bench_ab.sh r04n $m 2 default env:P2PG_PUSH_DEDUP=1 || exit 1
done
