# round 4: config 4 as a vertex partition over 8 ranks on the one GPU (gloo, host-staged exchange):
# per-rank kernel time of the partitioned form next to the message split's share
set -o pipefail
mkdir -p gpurun_out/r04p
timeout -k 10 1000 python -u bench.py --workload c4 --gpus 8 --split vertex --dist-backend gloo --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04p/c4_vertex8.json 2> gpurun_out/r04p/c4_vertex8.err || { tail -30 gpurun_out/r04p/c4_vertex8.err; exit 1; }
cat gpurun_out/r04p/c4_vertex8.json
