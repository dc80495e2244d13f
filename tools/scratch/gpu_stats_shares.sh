# rocprofv3 kernel stats of the config-4 share bench lines:  bash tools/gpu_stats_shares.sh <tag> msgs...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
for m in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/stats_m$m -o c4 -- \
    python3 bench.py --steps 5 --warmup 1 --msgs $m --no-cpu-baseline > gpurun_out/$tag/bench_m$m.json 2> gpurun_out/$tag/prof_m$m.err || { tail -20 gpurun_out/$tag/prof_m$m.err; exit 1; }
done
