# round 6: first GPU check of the sends stream / relay withdrawal / received counter
set -o pipefail
mkdir -p gpurun_out/r06a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_abi.py tests/test_compat.py tests/test_gpu_dynamic.py tests/test_gpu_parity.py -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread -p no:cacheprovider -k "not config4 and not config3" > gpurun_out/r06a/pytest.log 2>&1 || { tail -40 gpurun_out/r06a/pytest.log; exit 1; }
tail -20 gpurun_out/r06a/pytest.log
