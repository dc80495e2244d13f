# GPU parity suite, then per-round c4 A/B of the default build against kernel variants,
# interleaved (default, v1, v2, ..., default, v1, v2, ...) so box drift shows.
#   bash tools/gpu_ab_variants.sh <tag> variant1 variant2 ...   (python-p2p-network_amd/csrc/variants/<v>/)
#   AB_TESTS="tests/test_gpu_parity.py ..." narrows the parity run (default: the whole GPU suite)
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest ${AB_TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$tag/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$tag/pytest_gpu.log
args=()
for rep in 1 2; do
  args+=("P2PG_DUMMY=$rep")
  for v in "$@"; do args+=("P2PG_LIB=python-p2p-network_amd/csrc/variants/$v/libp2pgpu.so"); done
done
bash tools/gpu_env_variants.sh ${tag}_ab "${args[@]}"
