# Per-round profiles of config 4 at several message counts / policies (development aid).
#   bash tools/gpu_rounds_sweep.sh <tag> "M:ENV=V ..." ...
set -o pipefail
tag=${1:-rounds}; shift
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
i=0
for spec in "$@"; do
  i=$((i+1))
  M=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 python tools/round_profile.py c4 2 $M > gpurun_out/$tag/r$i.json 2> gpurun_out/$tag/r$i.err || { tail -20 gpurun_out/$tag/r$i.err; exit 1; }
  echo "== $spec"; python tools/rounds_summary.py gpurun_out/$tag/r$i.json
done
