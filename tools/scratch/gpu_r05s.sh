# round 5: line-masked push-row reads in the update and the update+push round (default) vs P2PG_TLINE=0 (whole rows, same
# touched layout) vs variants/head (4b08efe: one touched byte per peer); gossip parity first
set -o pipefail
mkdir -p gpurun_out/r05s
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_run_modes.py tests/test_gpu_dynamic.py "tests/test_gpu_fullsize.py::test_gossip_full_width_1m_matches_c_oracle" "tests/test_gpu_fullsize.py::test_gossip_wide_rows_hubs_churn_match_c_oracle" "tests/test_gpu_fullsize.py::test_run_chunks_keep_the_last_frontier" tests/test_gpu_split.py > gpurun_out/r05s/tests.log 2>&1 || { tail -30 gpurun_out/r05s/tests.log; exit 1; }
tail -3 gpurun_out/r05s/tests.log
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05s 4096 3 default env:P2PG_TLINE=0 head > gpurun_out/r05s/ab.txt 2>&1 || { cat gpurun_out/r05s/ab.txt; exit 1; }
cat gpurun_out/r05s/ab.txt
