# GPU check of the vertex-partitioned path, compat mode, runtime sharing and the c4/c5 benches.
mkdir -p gpurun_out
timeout -k 5 120 python tools/probe_runtime_order.py lib-first > gpurun_out/probe.log 2>&1 || { tail -20 gpurun_out/probe.log; exit 1; }
tail -3 gpurun_out/probe.log
timeout -k 10 800 python -m pytest tests/test_gpu_partition.py tests/test_compat.py -m gpu -x -q > gpurun_out/part.log 2>&1 || { tail -40 gpurun_out/part.log; exit 1; }
tail -3 gpurun_out/part.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample-msgs 16 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
cat gpurun_out/c4.json
timeout -k 10 300 python bench.py --workload c5 --peers 2000000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5s_n1.json 2> gpurun_out/c5s_n1.err || { tail -20 gpurun_out/c5s_n1.err; exit 1; }
cat gpurun_out/c5s_n1.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --workload c5 --peers 2000000 --steps 2 --warmup 1 --dist-backend gloo > gpurun_out/c5s_n2.json 2> gpurun_out/c5s_n2.err || { tail -30 gpurun_out/c5s_n2.err; exit 1; }
cat gpurun_out/c5s_n2.json
