# Interleaved bench.py A/B of runtime settings (p2pg_run path, as the bench times it):
#   bash tools/gpu_bench_env_ab.sh <tag> <msgs> <reps> "NAME=VAL ..." "NAME=VAL ..." ...
set -o pipefail
tag=$1; msgs=$2; reps=$3; shift 3
mkdir -p gpurun_out/$tag
for rep in $(seq 1 $reps); do
  i=0
  for envs in "$@"; do
    i=$((i+1))
    f=gpurun_out/$tag/m${msgs}_v${i}_$rep.json
    env $envs timeout -k 10 180 python bench.py --steps 5 --warmup 1 --msgs $msgs --no-cpu-baseline > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 - "$f" "$envs" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), "ms", round(d["value"], 1), "GTEPS",
      {k: round(v, 1) for k, v in d["kernel_ms_per_step"].items() if v})
PY
  done
done
