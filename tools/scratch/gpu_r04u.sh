# round 4: config 4 message split at full size, 2 / 4 / 8 ranks (W = 32 / 16 / 8 shares)
set -o pipefail
mkdir -p gpurun_out/r04u
timeout -k 10 1100 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu --durations=5 \
  "tests/test_gpu_split.py::test_message_split_config4_full_size" > gpurun_out/r04u/pt.log 2>&1 || { tail -15 gpurun_out/r04u/pt.log; exit 1; }
tail -8 gpurun_out/r04u/pt.log
