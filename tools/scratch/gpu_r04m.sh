# round 4: dense-entry word threshold at W = 64 (e_thresh 0.06 default) -- interleaved c4 A/B
set -o pipefail
AB_STEPS=8 bash tools/gpu_bench_ab.sh r04m 4096 3 default env:P2PG_E_THRESH=0.045 env:P2PG_E_THRESH=0.08
