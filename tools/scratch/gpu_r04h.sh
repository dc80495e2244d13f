# round 4: message-split shares on the current build + per-round profiles of the W = 8 share
set -o pipefail
mkdir -p gpurun_out/r04h
for m in 2048 1024 512; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --msgs $m --no-cpu-baseline > gpurun_out/r04h/bench_c4_m$m.json 2> gpurun_out/r04h/bench_c4_m$m.err || { tail -20 gpurun_out/r04h/bench_c4_m$m.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],1), 'ms', {k: round(v,1) for k, v in d['kernel_ms_per_step'].items() if v})" gpurun_out/r04h/bench_c4_m$m.json
done
timeout -k 10 300 python -u tools/round_profile.py c4 1 512 > gpurun_out/r04h/rounds_c4_m512.json 2> gpurun_out/r04h/rounds.err || { tail -20 gpurun_out/r04h/rounds.err; exit 1; }
timeout -k 10 300 python -u tools/round_profile.py c4 1 1024 > gpurun_out/r04h/rounds_c4_m1024.json 2>> gpurun_out/r04h/rounds.err || { tail -20 gpurun_out/r04h/rounds.err; exit 1; }
echo done
