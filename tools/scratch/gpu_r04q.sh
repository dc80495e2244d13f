# round 4: wider update grid for rounds with few row pushes -- run-mode parity, then interleaved
# A/B (P2PG_UPDATE_TINY=-1 = the single 1024-block cap) on c4 and the W = 8 share, plus grid sweeps
set -o pipefail
mkdir -p gpurun_out/r04q
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_run_modes.py "tests/test_gpu_fullsize.py::test_gossip_wide_rows_hubs_churn_match_c_oracle" \
  "tests/test_gpu_parity.py::test_gpu_gossip_push_forms_match_golden" > gpurun_out/r04q/pt.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r04q/pt.log | head; tail -5 gpurun_out/r04q/pt.log; exit 1; }
tail -1 gpurun_out/r04q/pt.log
AB_STEPS=6 bash tools/gpu_bench_ab.sh r04q 4096 3 default env:P2PG_UPDATE_TINY=-1 env:P2PG_UPDATE_GRID_TINY=16384 || exit 1
AB_STEPS=6 bash tools/gpu_bench_ab.sh r04q 512 2 default env:P2PG_UPDATE_TINY=-1 || exit 1
