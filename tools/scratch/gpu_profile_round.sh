# Round-end evidence: rocprofv3 kernel stats of the bench command, calibrated PMC traffic per
# kernel class (tools/traffic_run.sh), and the bench line with its traffic field.
#   bash tools/gpu_profile_round.sh <tag>
set -o pipefail
tag=${1:-prof}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/stats -o c4 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$tag/prof_bench.json 2> gpurun_out/$tag/prof.err || { tail -20 gpurun_out/$tag/prof.err; exit 1; }
bash tools/traffic_run.sh c4 > gpurun_out/$tag/traffic.log 2>&1 || { tail -20 gpurun_out/$tag/traffic.log; exit 1; }
cp gpurun_out/traffic_c4/traffic_c4.json profiles/traffic_c4.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > gpurun_out/$tag/bench_c4.json 2> gpurun_out/$tag/bench_c4.err || { tail -20 gpurun_out/$tag/bench_c4.err; exit 1; }
cp profiles/traffic_c4.json gpurun_out/$tag/traffic_c4.json
cat gpurun_out/$tag/bench_c4.json
