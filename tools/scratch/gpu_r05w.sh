# round 5: sparse launch cap 8192 (default) vs 16384 / 32768 blocks, c4 and the W = 8 share
set -o pipefail
mkdir -p gpurun_out/r05w
export TMPDIR=/tmp
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05w 4096 2 default sg16384 sg32768 > gpurun_out/r05w/ab.txt 2>&1 || { cat gpurun_out/r05w/ab.txt; exit 1; }
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05w 512 2 default sg16384 sg32768 >> gpurun_out/r05w/ab.txt 2>&1 || { cat gpurun_out/r05w/ab.txt; exit 1; }
cat gpurun_out/r05w/ab.txt
