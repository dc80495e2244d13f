# One round's evidence in one GPU session: the whole GPU suite, the default bench line (c4), the
# message-split share lines (--msgs 2048 / 1024 / 512 = one rank's work at N = 2 / 4 / 8), and
# rocprofv3 kernel stats of the c4 bench command.
#   bash tools/gpu_round.sh <tag>
set -o pipefail
tag=${1:?usage: bash tools/gpu_round.sh <tag>}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --durations=30 --timeout 700 --timeout-method thread -p no:cacheprovider > gpurun_out/$tag/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$tag/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/$tag/pytest_gpu.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/$tag/bench_c4.json 2> gpurun_out/$tag/bench_c4.err || { tail -20 gpurun_out/$tag/bench_c4.err; exit 1; }
tail -c 300 gpurun_out/$tag/bench_c4.json
for m in 2048 1024 512; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --msgs $m --no-cpu-baseline > gpurun_out/$tag/bench_c4_m$m.json 2> gpurun_out/$tag/bench_c4_m$m.err || { tail -20 gpurun_out/$tag/bench_c4_m$m.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],1), 'ms', {k: round(v,1) for k, v in d['kernel_ms_per_step'].items() if v})" gpurun_out/$tag/bench_c4_m$m.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/stats -o c4 -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/$tag/prof_bench.json 2> gpurun_out/$tag/prof.err || { tail -20 gpurun_out/$tag/prof.err; exit 1; }
echo prof ok
timeout -k 10 200 python3 tools/round_profile.py c4 1 > gpurun_out/$tag/rounds_c4.json || exit 1
echo rounds ok
