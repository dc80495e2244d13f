# round 4: partitioned gossip's dense rounds (PART kernels) + folded Philox -- partition suite,
# gossip parity subset, then c4 A/B fold vs the generic Philox
set -o pipefail
mkdir -p gpurun_out/r04l
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu --durations=15 \
  tests/test_gpu_partition.py tests/test_gpu_run_modes.py "tests/test_bench_launch.py::test_bench_c4_vertex_split_4_ranks_gloo" \
  "tests/test_gpu_fullsize.py::test_gossip_wide_rows_hubs_churn_match_c_oracle" \
  "tests/test_gpu_parity.py::test_gpu_gossip_push_forms_match_golden" "tests/test_gpu_parity.py::test_device_philox_kat" > gpurun_out/r04l/pt.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r04l/pt.log | head; tail -5 gpurun_out/r04l/pt.log; exit 1; }
tail -1 gpurun_out/r04l/pt.log
AB_STEPS=8 bash tools/gpu_bench_ab.sh r04l 4096 3 default nofold
