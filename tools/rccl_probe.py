#!/usr/bin/env python3
"""Probe: can two ranks share ONE GPU over RCCL (nccl backend), and can a torch CUDAGraph
capture an RCCL all-reduce? Run with: python -m butterfly_amd launch -n 2 -- python tools/rccl_probe.py
Prints one line per rank; exits non-zero on failure."""
import datetime
import os
import sys

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60),
                        device_id=torch.device("cuda", 0))
x = torch.full((1024,), float(rank + 1), device="cuda")
dist.all_reduce(x)
torch.cuda.synchronize()
ok1 = bool((x == sum(range(1, world + 1))).all())
# graph capture of an all-reduce
y = torch.full((4096,), float(rank + 1), device="cuda")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    dist.all_reduce(y)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    dist.all_reduce(y)
y.fill_(float(rank + 1))
g.replay()
torch.cuda.synchronize()
ok2 = bool((y == sum(range(1, world + 1))).all())
# send/recv
z = torch.full((256,), float(rank), device="cuda")
if rank == 0:
    dist.send(z, 1)
elif rank == 1:
    dist.recv(z, 0)
torch.cuda.synchronize()
ok3 = rank != 1 or bool((z == 0).all())
print(f"rank {rank}: allreduce={ok1} graph_allreduce={ok2} sendrecv={ok3}", flush=True)
dist.destroy_process_group()
sys.exit(0 if (ok1 and ok2 and ok3) else 1)
