# round 4: folded Philox rounds in the dense pushes -- gossip parity subset, then c4 A/B vs the generic
set -o pipefail
mkdir -p gpurun_out/r04k
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_run_modes.py "tests/test_gpu_fullsize.py::test_gossip_wide_rows_hubs_churn_match_c_oracle" \
  "tests/test_gpu_parity.py::test_gpu_gossip_push_forms_match_golden" "tests/test_gpu_parity.py::test_device_philox_kat" > gpurun_out/r04k/pt.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r04k/pt.log | head; tail -3 gpurun_out/r04k/pt.log; exit 1; }
tail -1 gpurun_out/r04k/pt.log
AB_STEPS=8 bash tools/gpu_bench_ab.sh r04k 4096 3 default nofold
