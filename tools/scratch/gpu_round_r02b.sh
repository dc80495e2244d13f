# Round evidence + message-split shares in one GPU session:
#   bash tools/gpu_round_r02b.sh <tag>
set -o pipefail
tag=${1:-r02}
bash tools/gpu_round_r02.sh $tag || exit 1
for m in 2048 1024 512; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --msgs $m --no-cpu-baseline > gpurun_out/$tag/bench_c4_m$m.json 2> gpurun_out/$tag/bench_c4_m$m.err || { tail -20 gpurun_out/$tag/bench_c4_m$m.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value'],1), 'GTEPS', round(d['ms_per_step'],1), 'ms', {k: round(v,2) for k, v in d['kernel_ms_per_step'].items() if v})" gpurun_out/$tag/bench_c4_m$m.json
done
