# round 6 final evidence on the last build, bench first (a cool box), then traffic, the whole
# -m gpu suite and smoke(): c4 bench line, message-split shares, rocprofv3 kernel stats, per-round
# profile, config 3 with one warmup run (kernel_times now waits for a run's last launches)
set -o pipefail
export TMPDIR=/tmp
tag=r06x
mkdir -p gpurun_out/$tag
SKIP_SUITE=1 bash tools/gpu_round.sh $tag || exit 1
timeout -k 10 200 python bench.py --workload c3 --steps 20 --warmup 1 > gpurun_out/$tag/bench_c3.json 2> gpurun_out/$tag/bench_c3.err || { tail -20 gpurun_out/$tag/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$tag/bench_c3.json')); print('c3', round(d['ms_per_step'],2), 'ms', round(d['value'],1), 'GTEPS', d['roofline']['kernel'], round(d['roofline']['frac'],3), round(d['whole_step_frac_survey_model'],3))"
P2PG_BUILD_SHA=${P2PG_BUILD_SHA:-unknown} bash tools/traffic_run.sh c4 > gpurun_out/$tag/traffic.log 2>&1 || { tail -20 gpurun_out/$tag/traffic.log; exit 1; }
cp gpurun_out/traffic_c4/traffic_c4.json gpurun_out/$tag/traffic_c4.json && echo traffic ok
timeout -k 10 900 python -u -m pytest tests -m gpu -q --durations=20 --timeout 700 --timeout-method thread -p no:cacheprovider > gpurun_out/$tag/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$tag/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$tag/pytest_gpu.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1 && echo smoke ok
