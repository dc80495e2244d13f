# Gossip GPU parity subset, then interleaved bench A/B of runtime knobs on the in-tree build:
#   bash tools/gpu_ab_env.sh <tag> "<msgs list>" <reps> variant...   (variants as in gpu_bench_ab.sh)
set -o pipefail
tag=$1; msgs=$2; reps=$3; shift 3
mkdir -p gpurun_out/$tag
if [ -z "$AB_SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_split.py tests/test_gpu_dynamic.py \
    -k "${AB_TESTS:-gossip or split or fused or run_chunks or quiescent or golden}" \
    > gpurun_out/$tag/pytest.log 2>&1 || { tail -40 gpurun_out/$tag/pytest.log; exit 1; }
  tail -1 gpurun_out/$tag/pytest.log
fi
for m in $msgs; do
  bash tools/gpu_bench_ab.sh $tag $m $reps "$@" || exit 1
done
