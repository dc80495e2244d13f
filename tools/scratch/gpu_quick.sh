# Quick GPU check: parity suite + c4 bench (no CPU baseline) + per-round profile.
#   bash tools/gpu_quick.sh <tag> [pytest -k expression]
set -o pipefail
tag=${1:-q}
mkdir -p gpurun_out/$tag
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/$tag/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$tag/pytest_gpu.log; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$tag/pytest_gpu.log; exit 1; }
fi
tail -1 gpurun_out/$tag/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$tag/bench_c4.json 2> gpurun_out/$tag/bench_c4.err || { tail -20 gpurun_out/$tag/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$tag/bench_c4.json')); print(round(d['value'],1), 'GTEPS', round(d['ms_per_step'],1), 'ms', {k: round(v,1) for k, v in d['kernel_ms_per_step'].items() if v}, 'frac', round(d['roofline']['frac'],3))"
timeout -k 10 300 python -u tools/round_profile.py c4 1 > gpurun_out/$tag/rounds_c4.json 2> gpurun_out/$tag/rounds_c4.err || { tail -20 gpurun_out/$tag/rounds_c4.err; exit 1; }
echo done
if [ -f python-p2p-network_amd/csrc/variants/prof/libp2pgpu.so ]; then
  P2PG_LIB=python-p2p-network_amd/csrc/variants/prof/libp2pgpu.so timeout -k 10 300 python tools/round_profile.py c4 1 > gpurun_out/$tag/rounds_prof.json 2> gpurun_out/$tag/prof_err.txt || { tail -5 gpurun_out/$tag/prof_err.txt; exit 1; }
  grep P2PG_PROF gpurun_out/$tag/prof_err.txt
fi
