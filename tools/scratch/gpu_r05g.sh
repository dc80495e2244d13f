# round 5: single-tile chunk scan + bounded blind rising rounds (default) vs the previous build
# (variants/r05e), and the spin-wait for the round counters (P2PG_SPIN=1)
set -o pipefail
mkdir -p gpurun_out/r05g
export TMPDIR=/tmp
AB_STEPS=10 bash tools/gpu_bench_ab.sh r05g 4096 3 default r05e env:P2PG_SPIN=1 > gpurun_out/r05g/ab.txt 2>&1 || { cat gpurun_out/r05g/ab.txt; exit 1; }
cat gpurun_out/r05g/ab.txt
