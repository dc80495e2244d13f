set -o pipefail
mkdir -p gpurun_out/sw
export TMPDIR=/tmp
bash tools/gpu_env_variants.sh sw_ab "P2PG_DUMMY=1" "P2PG_LIB=python-p2p-network_amd/csrc/variants/sw64/libp2pgpu.so" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sw/trace -o t -- python3 tools/round_profile.py c4 1 > gpurun_out/sw/rp.json 2> gpurun_out/sw/rp.err || { tail -5 gpurun_out/sw/rp.err; exit 1; }
echo ok
