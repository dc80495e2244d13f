# GPU parity (full -m gpu suite) + c4 bench + per-round kernel profile.
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
cat gpurun_out/c4.json
timeout -k 10 300 python tools/round_profile.py c4 1 > gpurun_out/rounds_c4.json 2> gpurun_out/rounds_c4.err || { tail -20 gpurun_out/rounds_c4.err; exit 1; }
