# Config-4 message-split shares on one GPU (per-rank work at N = 8 / 4 / 2 / 1) under the
# in-tree build, after a gossip parity subset:  bash tools/gpu_shares.sh <tag> [reps]
set -o pipefail
tag=${1:-shares}; reps=${2:-1}; shift 2
mkdir -p gpurun_out/$tag
if [ -z "$AB_SKIP_TESTS" ]; then
  timeout -k 10 1100 python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_split.py tests/test_gpu_dynamic.py \
    -k "${AB_TESTS:-gossip or split or fused or run_chunks or quiescent or golden}" \
    > gpurun_out/$tag/pytest.log 2>&1 || { tail -40 gpurun_out/$tag/pytest.log; exit 1; }
  tail -1 gpurun_out/$tag/pytest.log
fi
for m in 512 1024 2048 4096; do
  bash tools/gpu_bench_ab.sh $tag $m $reps default "$@" || exit 1
done
