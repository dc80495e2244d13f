# round 5: per-rank kernel time of the multi-GPU forms of config 4, each rank alone on the GPU
set -o pipefail
mkdir -p gpurun_out/r05c
for form in "8 4096" "4 2048" "4 4096" "2 4096" "2 2048"; do
  set -- $form
  timeout -k 10 400 python -u tools/rank_times.py $1 $2 2 > gpurun_out/r05c/ranks_v$1_m$2.json 2> gpurun_out/r05c/ranks_v$1_m$2.err || { tail -30 gpurun_out/r05c/ranks_v$1_m$2.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['runs'][-1]; print(sys.argv[1], 'W', d['W'], 'fused_all', d['fused_every_rank'], 'ok', r['relays_equal_one_engine'], 'kern', round(r['slowest_rank_kernel_ms'],1), 'xch', round(r['exchange_ms_at_xgmi'],1), 'proj', round(r['projected_step_ms'],1), 'ranks', [round(x,1) for x in r['rank_kernel_ms_total']])" gpurun_out/r05c/ranks_v$1_m$2.json
done
for m in 2048 1024 512; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --msgs $m --no-cpu-baseline > gpurun_out/r05c/bench_c4_m$m.json 2> gpurun_out/r05c/bench_c4_m$m.err || { tail -20 gpurun_out/r05c/bench_c4_m$m.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],1), 'ms', {k: round(v,1) for k, v in d['kernel_ms_per_step'].items() if v})" gpurun_out/r05c/bench_c4_m$m.json
done
