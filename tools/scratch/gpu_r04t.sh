# round 4: config 4's whole 10M x 4096 seen plane against the C oracle, word by word (opt-in test)
set -o pipefail
mkdir -p gpurun_out/r04t
P2PG_FULL_ORACLE=1 timeout -k 10 1150 python -u -m pytest -x -v -s --timeout 1500 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_gpu_parity.py::test_config4_full_size_every_word_matches_c_oracle" > gpurun_out/r04t/pt.log 2>&1 || { tail -15 gpurun_out/r04t/pt.log; exit 1; }
tail -3 gpurun_out/r04t/pt.log
