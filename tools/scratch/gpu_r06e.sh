# round 6: the whole GPU suite on the current build (durations), then the atomics microbench
set -o pipefail
mkdir -p gpurun_out/r06e
export TMPDIR=/tmp
timeout -k 10 1050 python -u -m pytest tests -m gpu -v --durations=40 --timeout 700 --timeout-method thread -p no:cacheprovider > gpurun_out/r06e/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r06e/pytest_gpu.log; exit 1; }
tail -45 gpurun_out/r06e/pytest_gpu.log
timeout -k 10 60 ./tools/microbench/atomics > gpurun_out/r06e/microbench_atomics.txt 2>&1 && cat gpurun_out/r06e/microbench_atomics.txt
