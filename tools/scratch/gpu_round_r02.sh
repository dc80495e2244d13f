# Round evidence in one GPU session: the whole GPU suite, the default bench line (c4), the
# config-5 line (100M peers, one GPU), and rocprofv3 kernel stats of the c4 bench command.
#   bash tools/gpu_round_r02.sh <tag>
set -o pipefail
tag=${1:-r02}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/$tag/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$tag/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$tag/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/$tag/bench_c4.json 2> gpurun_out/$tag/bench_c4.err || { tail -20 gpurun_out/$tag/bench_c4.err; exit 1; }
tail -c 300 gpurun_out/$tag/bench_c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/stats -o c4 -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/$tag/prof_bench.json 2> gpurun_out/$tag/prof.err || { tail -20 gpurun_out/$tag/prof.err; exit 1; }
echo prof ok
