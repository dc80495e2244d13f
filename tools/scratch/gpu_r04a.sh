# round 4: the new partition / snapshot / bench-launch / config-4 parity tests
set -o pipefail
mkdir -p gpurun_out/r04a
timeout -k 10 1100 python -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_partition.py tests/test_gpu_dynamic.py tests/test_bench_launch.py \
  "tests/test_gpu_parity.py::test_config4_full_size_reset_identical" \
  "tests/test_gpu_parity.py::test_config4_full_size_counters_are_the_sum_of_its_words" \
  "tests/test_gpu_parity.py::test_config4_full_size_word_matches_c_oracle" > gpurun_out/r04a/pt.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r04a/pt.log | tail -60
exit $rc
