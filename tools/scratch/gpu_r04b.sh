# round 4: delivery-stream test, c4 bench line, rocprof kernel stats, PMC traffic on this build,
# per-round profile.   bash tools/scratch/gpu_r04b.sh <tag> <sha>
set -o pipefail
tag=${1:-r04b}; sha=${2:-unknown}
O=gpurun_out/$tag
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_gpu_partition.py::test_partitioned_delivery_stream" > $O/pt.log 2>&1 || { tail -40 $O/pt.log; exit 1; }
tail -1 $O/pt.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c4', round(d['ms_per_step'],1), 'ms', round(d['value'],1), 'GTEPS frac', round(d['roofline']['frac'],3), 'whole', round(d['whole_step_frac_survey_model'],3), {k: round(v,1) for k, v in d['kernel_ms_per_step'].items() if v})" $O/bench_c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o c4 -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
echo prof ok
P2PG_BUILD_SHA=$sha timeout -k 10 900 bash tools/traffic_run.sh c4 > $O/traffic.log 2>&1 || { tail -20 $O/traffic.log; exit 1; }
cp gpurun_out/traffic_c4/traffic_c4.json $O/ && echo traffic ok
timeout -k 10 300 python -u tools/round_profile.py c4 1 > $O/rounds_c4.json 2> $O/rounds_c4.err || { tail -20 $O/rounds_c4.err; exit 1; }
echo done
