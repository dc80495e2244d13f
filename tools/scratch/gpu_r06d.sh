# round 6: light dense rounds (k_gossip_light) -- parity, then a c4 bench A/B
set -o pipefail
mkdir -p gpurun_out/r06d
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_light.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06d/pytest.log 2>&1 || { tail -40 gpurun_out/r06d/pytest.log; exit 1; }
tail -8 gpurun_out/r06d/pytest.log
for L in 0 -1; do
  P2PG_LIGHT=$L timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r06d/bench_L$L.json 2> gpurun_out/r06d/bench_L$L.err || { tail -20 gpurun_out/r06d/bench_L$L.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],1), 'ms', d['dominant_ms_by_round'][10:25])" gpurun_out/r06d/bench_L$L.json
done
