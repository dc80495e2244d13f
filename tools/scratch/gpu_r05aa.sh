# round 5: four touched peers per update stage (P2PG_UPDATE_QUAD=1) vs two (default): parity of
# the QUAD kernel first (schedule tests + full-width gossip vs the C oracle), then the c4 A/B
set -o pipefail
mkdir -p gpurun_out/r05aa
export TMPDIR=/tmp
P2PG_UPDATE_QUAD=1 timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_run_modes.py "tests/test_gpu_fullsize.py::test_gossip_full_width_1m_matches_c_oracle" "tests/test_gpu_fullsize.py::test_gossip_wide_rows_hubs_churn_match_c_oracle" > gpurun_out/r05aa/tests.log 2>&1 || { tail -30 gpurun_out/r05aa/tests.log; exit 1; }
tail -3 gpurun_out/r05aa/tests.log
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05aa 4096 3 default env:P2PG_UPDATE_QUAD=1 > gpurun_out/r05aa/ab.txt 2>&1 || { cat gpurun_out/r05aa/ab.txt; exit 1; }
cat gpurun_out/r05aa/ab.txt
