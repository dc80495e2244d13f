# round 4: LDS-staged hub pull -- parity on the hub tests with it on, then c4 A/B
set -o pipefail
mkdir -p gpurun_out/r04j
P2PG_HUB_LDS=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_gpu_fullsize.py::test_gossip_wide_rows_hubs_churn_match_c_oracle" "tests/test_gpu_fullsize.py::test_gossip_full_width_1m_matches_c_oracle" \
  tests/test_gpu_run_modes.py "tests/test_gpu_partition.py::test_partitioned_engines_match_single_gpu" > gpurun_out/r04j/pt.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r04j/pt.log | head; tail -3 gpurun_out/r04j/pt.log; exit 1; }
tail -1 gpurun_out/r04j/pt.log
AB_STEPS=8 bash tools/gpu_bench_ab.sh r04j 4096 3 default env:P2PG_HUB_LDS=1
