# round 5: config 5 at full size, unpartitioned and as the 2-rank vertex partition (the new tests)
set -o pipefail
mkdir -p gpurun_out/r05b
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fullsize.py -k config5 -x -v --timeout 950 --timeout-method thread -p no:cacheprovider --durations 10 > gpurun_out/r05b/c5.log 2>&1 || { tail -60 gpurun_out/r05b/c5.log; exit 1; }
tail -16 gpurun_out/r05b/c5.log
