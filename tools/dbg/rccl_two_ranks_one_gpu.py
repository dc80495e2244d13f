"""Probe: can two processes form an RCCL (nccl backend) group on ONE GPU and run
all_to_all_single with split sizes?  Launched by torch.distributed.run --nproc-per-node 2."""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.arange(10, dtype=torch.int64, device="cuda:0") + 100 * rank
ins = [3, 7] if rank == 0 else [4, 6]
outs = [3, 4] if rank == 0 else [7, 6]
y = torch.empty(sum(outs), dtype=torch.int64, device="cuda:0")
dist.all_to_all_single(y, x, outs, ins)
torch.cuda.synchronize()
print(f"rank {rank}: {y.tolist()}", flush=True)
dist.destroy_process_group()
