"""Probe: can two ranks share one GPU over RCCL (torch.distributed 'nccl')?
usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
           --master-port 29511 tools/probe_rccl.py"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
x = torch.full((4,), float(rank + 1), device="cuda:0")
dist.all_reduce(x)
torch.cuda.synchronize()
y = torch.zeros(4, device="cuda:0")
if rank == 0:
    dist.send(torch.arange(4.0, device="cuda:0"), 1)
elif rank == 1:
    dist.recv(y, 0)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce {x.tolist()} recv {y.tolist()}", flush=True)
dist.destroy_process_group()
