# round 5: partial frontier rows (P2PG_PARTIAL_F) and per-launch events (P2PG_BENCH_TIMING) A/B,
# interleaved bench lines on one box; then the parity tests that cover the changed kernels
set -o pipefail
mkdir -p gpurun_out/r05d
export TMPDIR=/tmp
AB_STEPS=10 bash tools/gpu_bench_ab.sh r05d 4096 3 default env:P2PG_PARTIAL_F=0 env:P2PG_BENCH_TIMING=0 > gpurun_out/r05d/ab.txt 2>&1 || { cat gpurun_out/r05d/ab.txt; exit 1; }
cat gpurun_out/r05d/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_run_modes.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "run_modes or push_forms or config4_full_size_word_matches_c_oracle and 63" > gpurun_out/r05d/pt.log 2>&1 || { tail -40 gpurun_out/r05d/pt.log; exit 1; }
tail -3 gpurun_out/r05d/pt.log
