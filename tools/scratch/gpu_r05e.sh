# round 5: two touched peers per stage of the update (P2PG_UPDATE_DUAL) A/B, then the gossip
# parity tests that cover the update / partial-frontier / counter changes
set -o pipefail
mkdir -p gpurun_out/r05e
export TMPDIR=/tmp
AB_STEPS=10 bash tools/gpu_bench_ab.sh r05e 4096 3 default env:P2PG_UPDATE_DUAL=0 > gpurun_out/r05e/ab.txt 2>&1 || { cat gpurun_out/r05e/ab.txt; exit 1; }
cat gpurun_out/r05e/ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_run_modes.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_dynamic.py tests/test_gpu_split.py tests/test_compat.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -k "not config5 and not config4_full_size_counters and not message_split_config4_full_size" --durations 15 > gpurun_out/r05e/pt.log 2>&1 || { tail -60 gpurun_out/r05e/pt.log; exit 1; }
tail -20 gpurun_out/r05e/pt.log
