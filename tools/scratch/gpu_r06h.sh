# round 6: configs 3 and 5 re-measured on the current build (c5 with the arrivals counter of churn runs)
set -o pipefail
mkdir -p gpurun_out/r06h
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload c3 --steps 20 --warmup 3 > gpurun_out/r06h/bench_c3.json 2> gpurun_out/r06h/bench_c3.err || { tail -20 gpurun_out/r06h/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r06h/bench_c3.json')); print('c3', round(d['ms_per_step'],2), 'ms', round(d['value'],1), 'GTEPS', d['roofline']['frac'], d['whole_step_frac_survey_model'])"
timeout -k 10 600 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06h/bench_c5.json 2> gpurun_out/r06h/bench_c5.err || { tail -20 gpurun_out/r06h/bench_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r06h/bench_c5.json')); print('c5', round(d['ms_per_step'],2), 'ms', round(d['value'],1), 'GTEPS', d['roofline']['frac'], d['whole_step_frac_survey_model'], d['received_per_step'], d['relays_per_step'], d['kernel_ms_per_step'])"
