# Parity subset + c4 bench + per-launch kernel trace of one c4 broadcast (sparse-round kernels).
#   bash tools/gpu_sparse_trace.sh <tag> "<test files>"
set -o pipefail
tag=${1:-sp}
export TMPDIR=/tmp
bash tools/gpu_check_files.sh $tag "${2:-tests/test_gpu_parity.py}" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$tag/trace -o t -- python3 tools/round_profile.py c4 1 > gpurun_out/$tag/rp.json 2> gpurun_out/$tag/rp.err || { tail -5 gpurun_out/$tag/rp.err; exit 1; }
echo trace ok
