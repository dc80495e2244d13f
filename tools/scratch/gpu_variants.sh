# Per-round c4 profile of the default build and of kernel variants (A/B), no tests.
#   bash tools/gpu_variants.sh <tag> variant1 variant2 ...   (python-p2p-network_amd/csrc/variants/<v>/)
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 300 python tools/round_profile.py c4 1 > gpurun_out/$tag/rounds_c4.json 2> gpurun_out/$tag/rounds_c4.err || { tail -20 gpurun_out/$tag/rounds_c4.err; exit 1; }
for v in "$@"; do
  P2PG_LIB=python-p2p-network_amd/csrc/variants/$v/libp2pgpu.so timeout -k 10 300 python tools/round_profile.py c4 1 > gpurun_out/$tag/rounds_c4_$v.json 2> gpurun_out/$tag/rounds_c4_$v.err || { tail -20 gpurun_out/$tag/rounds_c4_$v.err; exit 1; }
done
files="gpurun_out/$tag/rounds_c4.json"; for v in "$@"; do files="$files gpurun_out/$tag/rounds_c4_$v.json"; done; python3 tools/cmp_rounds.py $files > gpurun_out/$tag/cmp.txt; tail -4 gpurun_out/$tag/cmp.txt
echo done
