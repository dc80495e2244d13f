# The whole GPU suite, then interleaved bench A/B of library builds / runtime knobs:
#   bash tools/gpu_suite_ab.sh <tag> "<msgs list>" <reps> variant...   (variants as in gpu_bench_ab.sh)
set -o pipefail
tag=$1; msgs=$2; reps=$3; shift 3
mkdir -p gpurun_out/$tag
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 700 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$tag/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$tag/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$tag/pytest_gpu.log
for m in $msgs; do
  bash tools/gpu_bench_ab.sh $tag $m $reps "$@" || exit 1
done
