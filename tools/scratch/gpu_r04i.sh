# round 4: decay-aware last dense round on / off per share width (interleaved)
set -o pipefail
for m in 512 1024 2048 4096; do
  AB_STEPS=6 bash tools/gpu_bench_ab.sh r04i $m 2 default env:P2PG_DECAY_PRED=0 || exit 1
done
