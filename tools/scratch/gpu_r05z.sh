# round 5: the whole GPU suite with per-test durations on the final build (split-test fixture,
# round-0 recount test), then smoke()
set -o pipefail
mkdir -p gpurun_out/r05z
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --durations=40 --timeout 700 --timeout-method thread -p no:cacheprovider > gpurun_out/r05z/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05z/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05z/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z/smoke.log 2>&1 || { tail -20 gpurun_out/r05z/smoke.log; exit 1; }
tail -3 gpurun_out/r05z/smoke.log
