# c3 flood bench: default build vs a variant, alternating (noise check).  bash tools/gpu_c3_ab.sh <tag> <variant>
set -o pipefail
tag=$1; v=$2
mkdir -p gpurun_out/$tag
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$tag/def_$i.json 2>/dev/null || exit 1
  P2PG_LIB=python-p2p-network_amd/csrc/variants/$v/libp2pgpu.so timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$tag/var_$i.json 2>/dev/null || exit 1
done
for f in gpurun_out/$tag/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],3), round(d['kernel_ms_per_step']['flood_pull'],3))"; done
