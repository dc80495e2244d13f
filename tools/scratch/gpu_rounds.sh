# Per-round stats + kernel ms of config 4 at 4096 and 512 broadcasts (development aid).
#   bash tools/gpu_rounds.sh <tag>
set -o pipefail
tag=${1:-rounds}
mkdir -p gpurun_out/$tag
for m in 4096 512; do
  timeout -k 10 300 python -u tools/round_profile.py c4 2 $m > gpurun_out/$tag/rounds_c4_m$m.json 2> gpurun_out/$tag/rounds_c4_m$m.err || { tail -20 gpurun_out/$tag/rounds_c4_m$m.err; exit 1; }
  python tools/rounds_summary.py gpurun_out/$tag/rounds_c4_m$m.json
done
