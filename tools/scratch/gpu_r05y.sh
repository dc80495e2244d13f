# round 5: config 5 bench on one GPU (100M WS, churn 0.05, 4096 floods) on the current build
set -o pipefail
mkdir -p gpurun_out/r05y
export TMPDIR=/tmp
timeout -k 10 900 python bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/r05y/bench_c5.json 2> gpurun_out/r05y/bench_c5.err || { tail -20 gpurun_out/r05y/bench_c5.err; exit 1; }
tail -c 400 gpurun_out/r05y/bench_c5.json
