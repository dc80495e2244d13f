# round 4 final build: bench line, share lines, rocprof kernel stats, calibrated PMC traffic, per-round profile
set -o pipefail
SKIP_SUITE=1 bash tools/gpu_round.sh r04z2 || exit 1
P2PG_BUILD_SHA=7d75c2aee69b bash tools/traffic_run.sh c4 || exit 1
timeout -k 10 200 python3 tools/round_profile.py c4 1 > gpurun_out/r04z2/rounds_c4.json || exit 1
echo all ok
