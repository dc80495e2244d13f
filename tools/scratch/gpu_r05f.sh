# round 5: per-round profiles of config 4 (4096) and of the N = 8 share (512 broadcasts);
# the resized run-chunks test
set -o pipefail
mkdir -p gpurun_out/r05f
timeout -k 10 200 python3 tools/round_profile.py c4 1 > gpurun_out/r05f/rounds_c4.json || exit 1
timeout -k 10 200 python3 tools/round_profile.py c4 1 512 > gpurun_out/r05f/rounds_c4_m512.json || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k run_chunks -x -q --timeout 250 --timeout-method thread -p no:cacheprovider --durations 3 > gpurun_out/r05f/pt.log 2>&1 || { tail -40 gpurun_out/r05f/pt.log; exit 1; }
tail -6 gpurun_out/r05f/pt.log
