# round 4: whole GPU suite on the slot-header build, then c4 A/B against P2PG_EHDR=0
set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04e/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r04e/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04e/pytest_gpu.log
AB_STEPS=8 bash tools/gpu_bench_ab.sh r04e 4096 3 default env:P2PG_EHDR=0
