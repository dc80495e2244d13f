# round 5: LLVM AMDGPU scheduler strategies for the whole library (variants/s_*) vs the default
set -o pipefail
mkdir -p gpurun_out/r05r
export TMPDIR=/tmp
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05r 4096 2 default s_max-ilp s_iterative-ilp s_max-memory-clause > gpurun_out/r05r/ab.txt 2>&1 || { cat gpurun_out/r05r/ab.txt; exit 1; }
cat gpurun_out/r05r/ab.txt
