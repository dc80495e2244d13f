# One GPU session: GPU parity suite, c4 bench (with CPU baseline), rocprofv3 kernel stats of the
# bench command, per-round kernel profile.  Usage: bash tools/gpu_round.sh <tag>
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
if [ -x tools/microbench/philox_rate ]; then timeout -k 10 60 tools/microbench/philox_rate > gpurun_out/$tag/philox_rate.txt 2>&1 || exit 1; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$tag/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$tag/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > gpurun_out/$tag/bench_c4.json 2> gpurun_out/$tag/bench_c4.err || { tail -20 gpurun_out/$tag/bench_c4.err; exit 1; }
cat gpurun_out/$tag/bench_c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/prof -o c4 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$tag/prof_bench.json 2> gpurun_out/$tag/prof.err || { tail -20 gpurun_out/$tag/prof.err; exit 1; }
timeout -k 10 300 python -u tools/round_profile.py c4 1 > gpurun_out/$tag/rounds_c4.json 2> gpurun_out/$tag/rounds_c4.err || { tail -20 gpurun_out/$tag/rounds_c4.err; exit 1; }
echo done
