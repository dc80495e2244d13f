# Per-round c4 profile under several environment settings (runtime knobs, same build).
#   bash tools/gpu_env_variants.sh <tag> "NAME=VAL ..." "NAME=VAL ..." ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
i=0; files=""
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 300 python tools/round_profile.py c4 1 > gpurun_out/$tag/rounds_$i.json 2> gpurun_out/$tag/err_$i.txt || { tail -20 gpurun_out/$tag/err_$i.txt; exit 1; }
  files="$files gpurun_out/$tag/rounds_$i.json"
  echo "$i: $envs"
done
python3 tools/cmp_rounds.py $files > gpurun_out/$tag/cmp.txt; tail -$i gpurun_out/$tag/cmp.txt
