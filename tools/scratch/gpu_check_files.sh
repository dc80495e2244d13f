# GPU check of chosen test files + the c4 bench line and per-round profile, optional A/B env.
#   bash tools/gpu_check_files.sh <tag> "<test files>" ["ENV=VAL for the B bench"]
set -o pipefail
tag=${1:-q}
files=${2:-tests}
benv=${3:-}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest $files -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$tag/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$tag/pytest_gpu.log
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value'],1), 'GTEPS', round(d['ms_per_step'],1), 'ms', {k: round(v,2) for k, v in d['kernel_ms_per_step'].items() if v}, 'frac', round(d['roofline']['frac'],3))" $1; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/$tag/bench_c4.json 2> gpurun_out/$tag/bench_c4.err || { tail -20 gpurun_out/$tag/bench_c4.err; exit 1; }
summ gpurun_out/$tag/bench_c4.json
if [ -n "$benv" ]; then
  env $benv timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/$tag/bench_c4_b.json 2> gpurun_out/$tag/bench_c4_b.err || { tail -20 gpurun_out/$tag/bench_c4_b.err; exit 1; }
  summ gpurun_out/$tag/bench_c4_b.json
fi
timeout -k 10 300 python -u tools/round_profile.py c4 1 > gpurun_out/$tag/rounds_c4.json 2> gpurun_out/$tag/rounds_c4.err || { tail -20 gpurun_out/$tag/rounds_c4.err; exit 1; }
echo done
