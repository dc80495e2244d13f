#!/bin/bash
# Calibrated HBM traffic for bench.py's workload: PMC passes over the calibration microbench
# and over one bench step, then tools/pmc_traffic.py -> profiles/traffic_<wl>.json
# (P2PG_BUILD_SHA=<git sha of the build> is recorded in the file: the box has no .git)
set -e
WL=${1:-c4}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/traffic_$WL
mkdir -p $O/cal $O/run
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cal/pass1 -o p -- ./tools/microbench/atomics > $O/cal1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cal/pass2 -o p -- ./tools/microbench/atomics > $O/cal2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/run/pass1 -o p -- python3 bench.py --workload $WL --steps 1 --warmup 0 --no-cpu-baseline > $O/run1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/run/pass2 -o p -- python3 bench.py --workload $WL --steps 1 --warmup 0 --no-cpu-baseline > $O/run2.log 2>&1
python3 tools/pmc_traffic.py $O/cal $O/run $WL $O/traffic_$WL.json "${P2PG_BUILD_SHA:-unknown}"
