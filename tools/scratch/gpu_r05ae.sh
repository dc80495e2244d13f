# round 5: hub pushes of fused rounds split into (hub, 8 words) items (default) vs one wave per hub
# (variants/head); parity of the hub cases first
set -o pipefail
mkdir -p gpurun_out/r05ae
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_gossip_full_width_1m_matches_c_oracle" "tests/test_gpu_fullsize.py::test_gossip_wide_rows_hubs_churn_match_c_oracle" tests/test_gpu_run_modes.py > gpurun_out/r05ae/tests.log 2>&1 || { tail -30 gpurun_out/r05ae/tests.log; exit 1; }
tail -3 gpurun_out/r05ae/tests.log
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05ae 4096 3 default head > gpurun_out/r05ae/ab.txt 2>&1 || { cat gpurun_out/r05ae/ab.txt; exit 1; }
cat gpurun_out/r05ae/ab.txt
