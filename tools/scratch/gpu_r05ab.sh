# round 5: rising-phase batches (rounds sparse by a bound run without per-round host syncs) and
# no update+push on a provably sparse round (default) vs variants/head; schedule parity first
set -o pipefail
mkdir -p gpurun_out/r05ab
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_run_modes.py tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_gossip_full_width_1m_matches_c_oracle" "tests/test_gpu_fullsize.py::test_run_chunks_keep_the_last_frontier" > gpurun_out/r05ab/tests.log 2>&1 || { tail -30 gpurun_out/r05ab/tests.log; exit 1; }
tail -3 gpurun_out/r05ab/tests.log
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05ab 4096 3 default head > gpurun_out/r05ab/ab.txt 2>&1 || { cat gpurun_out/r05ab/ab.txt; exit 1; }
cat gpurun_out/r05ab/ab.txt
