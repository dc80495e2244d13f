# Interleaved bench.py A/B of library builds (p2pg_run path, as the bench times it):
#   bash tools/gpu_bench_ab.sh <tag> <msgs> <reps> variant...   ("default" = the in-tree build,
#   else python-p2p-network_amd/csrc/variants/<v>/libp2pgpu.so)
set -o pipefail
tag=$1; msgs=$2; reps=$3; shift 3
mkdir -p gpurun_out/$tag
for rep in $(seq 1 $reps); do
  for v in "$@"; do
    # variant: "default" (in-tree build), a variants/<v> build, or "env:NAME=VAL[,NAME=VAL]"
    # (the in-tree build under runtime knobs)
    lib=""; envs=""
    case "$v" in
      default) ;;
      env:*) envs=$(echo "${v#env:}" | tr ',' ' ') ;;
      *) lib=python-p2p-network_amd/csrc/variants/$v/libp2pgpu.so ;;
    esac
    f=gpurun_out/$tag/m${msgs}_$(echo "$v" | tr ':=,' '___')_$rep.json
    env P2PG_LIB=$lib $envs timeout -k 10 180 python bench.py --workload ${AB_WORKLOAD:-c4} --steps ${AB_STEPS:-5} --warmup 1 --msgs $msgs --no-cpu-baseline > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 - "$f" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), "ms", round(d["value"], 1), "GTEPS",
      "frac", round(d["roofline"]["frac"], 3), {k: round(v, 1) for k, v in d["kernel_ms_per_step"].items() if v})
PY
  done
done
