# round 6 final evidence, part 1: the whole GPU suite on the final tree (durations)
set -o pipefail
mkdir -p gpurun_out/r06i
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --durations=40 --timeout 700 --timeout-method thread -p no:cacheprovider > gpurun_out/r06i/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r06i/pytest_gpu.log; exit 1; }
tail -45 gpurun_out/r06i/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06i/smoke.log 2>&1 && cat gpurun_out/r06i/smoke.log
