# round 6 final evidence, part 2: c4 bench line, message-split shares, rocprofv3 kernel stats,
# per-round profile, calibrated PMC traffic (P2PG_BUILD_SHA: the commit of this build)
set -o pipefail
export TMPDIR=/tmp
SKIP_SUITE=1 bash tools/gpu_round.sh r06n || exit 1
P2PG_BUILD_SHA=${P2PG_BUILD_SHA:-unknown} bash tools/traffic_run.sh c4 > gpurun_out/r06n/traffic.log 2>&1 || { tail -20 gpurun_out/r06n/traffic.log; exit 1; }
cp gpurun_out/traffic_c4/traffic_c4.json gpurun_out/r06n/traffic_c4.json && echo traffic ok
