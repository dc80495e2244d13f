# round 5: the hub chain on a side stream (P2PG_HUB_SIDE) and the update's task table, A/B against
# the ea3a7e1 build (variants/r05e); then the gossip parity tests (hubs, churn, every push form)
set -o pipefail
mkdir -p gpurun_out/r05h
export TMPDIR=/tmp
AB_STEPS=10 bash tools/gpu_bench_ab.sh r05h 4096 3 default r05e > gpurun_out/r05h/ab.txt 2>&1 || { cat gpurun_out/r05h/ab.txt; exit 1; }
cat gpurun_out/r05h/ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_run_modes.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_partition.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -k "not config5 and not config4_full_size and not message_split_config4_full_size" --durations 5 > gpurun_out/r05h/pt.log 2>&1 || { tail -60 gpurun_out/r05h/pt.log; exit 1; }
tail -9 gpurun_out/r05h/pt.log
