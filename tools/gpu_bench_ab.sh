# Interleaved bench.py A/B of library builds (p2pg_run path, as the bench times it):
#   bash tools/gpu_bench_ab.sh <tag> <msgs> <reps> variant...   ("default" = the in-tree build,
#   else python-p2p-network_amd/csrc/variants/<v>/libp2pgpu.so)
set -o pipefail
tag=$1; msgs=$2; reps=$3; shift 3
mkdir -p gpurun_out/$tag
for rep in $(seq 1 $reps); do
  for v in "$@"; do
    lib=""; [ "$v" != default ] && lib=python-p2p-network_amd/csrc/variants/$v/libp2pgpu.so
    f=gpurun_out/$tag/m${msgs}_${v}_$rep.json
    P2PG_LIB=$lib timeout -k 10 180 python bench.py --steps 5 --warmup 1 --msgs $msgs --no-cpu-baseline > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 - "$f" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), "ms", round(d["value"], 1), "GTEPS",
      "frac", round(d["roofline"]["frac"], 3), {k: round(v, 1) for k, v in d["kernel_ms_per_step"].items() if v})
PY
  done
done
