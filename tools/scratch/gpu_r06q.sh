# round 6 final evidence on the last build: the whole -m gpu suite, c4 bench line, message-split
# shares, rocprofv3 kernel stats, per-round profile, calibrated PMC traffic (P2PG_BUILD_SHA)
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_round.sh r06q || exit 1
P2PG_BUILD_SHA=${P2PG_BUILD_SHA:-unknown} bash tools/traffic_run.sh c4 > gpurun_out/r06q/traffic.log 2>&1 || { tail -20 gpurun_out/r06q/traffic.log; exit 1; }
cp gpurun_out/traffic_c4/traffic_c4.json gpurun_out/r06q/traffic_c4.json && echo traffic ok
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06q/smoke.log 2>&1 && echo smoke ok
