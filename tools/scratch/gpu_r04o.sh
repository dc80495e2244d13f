# round 4: Floyd draws through an opaque v_mul_hi_u32 (32-bit dedup compares) -- gossip parity subset,
# then interleaved A/B vs -DP2PG_PICK_ASM=0 on c4 and its shares
set -o pipefail
mkdir -p gpurun_out/r04o
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_split.py tests/test_gpu_run_modes.py "tests/test_gpu_partition.py::test_partitioned_gossip_dense_rounds" \
  "tests/test_gpu_fullsize.py::test_gossip_wide_rows_hubs_churn_match_c_oracle" "tests/test_gpu_fullsize.py::test_gossip_full_width_1m_matches_c_oracle" \
  "tests/test_gpu_parity.py::test_gpu_gossip_push_forms_match_golden" "tests/test_gpu_parity.py::test_device_philox_kat" > gpurun_out/r04o/pt.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r04o/pt.log | head; tail -5 gpurun_out/r04o/pt.log; exit 1; }
tail -1 gpurun_out/r04o/pt.log
for m in 4096 512 2048; do
  AB_STEPS=6 bash tools/gpu_bench_ab.sh r04o $m 3 default noasm || exit 1
done
