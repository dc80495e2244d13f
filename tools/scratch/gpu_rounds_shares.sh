# Per-round stats + kernel ms of config-4 shares (development aid):  bash tools/gpu_rounds_shares.sh <tag> m...
set -o pipefail
tag=${1:-rounds}; shift
mkdir -p gpurun_out/$tag
for m in "$@"; do
  timeout -k 10 300 python -u tools/round_profile.py c4 2 $m > gpurun_out/$tag/rounds_c4_m$m.json 2> gpurun_out/$tag/rounds_c4_m$m.err || { tail -20 gpurun_out/$tag/rounds_c4_m$m.err; exit 1; }
done
