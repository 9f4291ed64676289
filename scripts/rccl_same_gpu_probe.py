#!/usr/bin/env python3
"""Can RCCL run several ranks on ONE GPU? (rehearsal of the multi-GPU pipeline on a 1-GPU
box). Each rank uses cuda:0; ring send/recv + an all_reduce; prints OK per rank."""
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
x = torch.full((1024,), float(rank), device=dev)
y = torch.empty_like(x)
reqs = [dist.isend(x, (rank + 1) % world), dist.irecv(y, (rank - 1) % world)]
for r in reqs:
    r.wait()
torch.cuda.synchronize()
assert float(y[0]) == (rank - 1) % world, float(y[0])
z = torch.ones(4, device=dev)
dist.all_reduce(z)
torch.cuda.synchronize()
print(f"rank {rank}: OK recv={float(y[0])} allreduce={float(z[0])}", flush=True)
dist.barrier()
dist.destroy_process_group()
