# round 5: config 5 bench on one GPU (100M WS, churn 0.05, 4096 floods) on the current build;
set -o pipefail
mkdir -p gpurun_out/r05y
export TMPDIR=/tmp
timeout -k 10 900 python bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/r05y/bench_c5.json 2> gpurun_out/r05y/bench_c5.err || { tail -20 gpurun_out/r05y/bench_c5.err; exit 1; }
tail -c 400 gpurun_out/r05y/bench_c5.json
# and the W = 8 share's dense-round entry (v_thresh 0.95 for W <= 32) re-swept after the sparse grid change
AB_STEPS=8 bash tools/gpu_bench_ab.sh r05y 512 2 default env:P2PG_V_THRESH=0.9 env:P2PG_V_THRESH=0.85 > gpurun_out/r05y/ab_m512.txt 2>&1 || { cat gpurun_out/r05y/ab_m512.txt; exit 1; }
cat gpurun_out/r05y/ab_m512.txt
