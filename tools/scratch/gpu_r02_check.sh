# Round-2 development check: GPU parity of the relay paths, then c4 benches at several W.
#   bash tools/gpu_r02_check.sh <tag> [pytest-selection...]
set -o pipefail
tag=${1:-chk}; shift
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
sel=${@:-tests/test_gpu_parity.py tests/test_gpu_dynamic.py tests/test_compat.py}
timeout -k 10 600 python -u -m pytest $sel -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$tag/pytest.log 2>&1 || { tail -40 gpurun_out/$tag/pytest.log; exit 1; }
tail -3 gpurun_out/$tag/pytest.log
for m in 512 1024 2048 4096; do
  timeout -k 10 120 python bench.py --steps 5 --warmup 1 --msgs $m --no-cpu-baseline > gpurun_out/$tag/c4_m$m.json 2> gpurun_out/$tag/c4_m$m.err || { tail -20 gpurun_out/$tag/c4_m$m.err; exit 1; }
  python - gpurun_out/$tag/c4_m$m.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], round(d["value"], 1), "GTEPS", round(d["ms_per_step"], 2), "ms", {k: round(v, 1) for k, v in d["kernel_ms_per_step"].items() if v})
PY
done
