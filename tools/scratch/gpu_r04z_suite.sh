# round 4 final build: the whole GPU suite in two halves (each under one gpurun limit)
#   bash tools/scratch/gpu_r04z_suite.sh <half: 1|2>
set -o pipefail
mkdir -p gpurun_out/r04z
if [ "$1" = 1 ]; then FILES="tests/test_gpu_fullsize.py tests/test_gpu_parity.py"
else FILES=$(ls tests/test_*.py | grep -v -e test_gpu_fullsize.py -e test_gpu_parity.py | tr '\n' ' '); fi
timeout -k 10 1120 python -u -m pytest $FILES -m gpu -v --timeout 700 --timeout-method thread -p no:cacheprovider --durations=25 > gpurun_out/r04z/pytest_gpu_$1.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r04z/pytest_gpu_$1.log | head; tail -5 gpurun_out/r04z/pytest_gpu_$1.log; exit 1; }
tail -1 gpurun_out/r04z/pytest_gpu_$1.log
