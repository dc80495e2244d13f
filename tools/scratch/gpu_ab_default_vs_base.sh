set -o pipefail
mkdir -p gpurun_out/mw
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mw/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/mw/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/mw/pytest_gpu.log
B=python-p2p-network_amd/csrc/variants/base/libp2pgpu.so
bash tools/gpu_env_variants.sh mwab "P2PG_DUMMY=1" "P2PG_LIB=$B" "P2PG_DUMMY=2" "P2PG_LIB=$B"
