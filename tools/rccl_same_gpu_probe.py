#!/usr/bin/env python3
"""Probe (not a test): can two RCCL ranks share one GPU on this image?  Rank r puts its id in a tensor on device 0 and
the ranks all_gather it over the "nccl" (RCCL) backend.  Run as
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
        tools/rccl_same_gpu_probe.py"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl")
t = torch.full((4,), float(rank), device="cuda:0")
out = torch.empty(8, device="cuda:0")
dist.all_gather_into_tensor(out, t)
torch.cuda.synchronize()
print(f"rank {rank}: all_gather ok {out.tolist()}", flush=True)
dist.destroy_process_group()
