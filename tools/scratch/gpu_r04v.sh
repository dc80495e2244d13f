# round 4: config 5's 100M x 4096 seen plane against the C oracle, a word range per call
#   bash tools/scratch/gpu_r04v.sh lo-hi
set -o pipefail
mkdir -p gpurun_out/r04v
P2PG_C5_WORDS=$1 timeout -k 10 1150 python -u -m pytest -x -v -s --timeout 1500 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_gpu_fullsize.py::test_config5_full_size_words_match_c_oracle" > gpurun_out/r04v/pt_$1.log 2>&1 || { tail -15 gpurun_out/r04v/pt_$1.log; exit 1; }
tail -3 gpurun_out/r04v/pt_$1.log
