#!/usr/bin/env python3
"""Which HIP stream does a ProcessGroupNCCL (RCCL) collective run on?

World-1 process group; under ``torch.cuda.stream(side)`` issue a non-in-place
collective (all_gather_into_tensor: at one rank RCCL copies in -> out, so a
kernel / copy lands on whatever stream the PG used) with async_op=False and
async_op=True, marking each phase with a small kernel on the side stream.  Run
under ``rocprofv3 --kernel-trace`` and compare Stream_Id of the copies with the
marker's.
"""
import os
import time

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
side = torch.cuda.Stream()
x = torch.randn(1 << 22, device="cuda")
y = torch.empty_like(x)
with torch.cuda.stream(side):
    for mode in ("sync", "async", "sync"):
        torch.ones(8, device="cuda").mul_(3)  # marker on the side stream
        w = dist.all_gather_into_tensor(y, x, async_op=(mode == "async"))
        if w is not None:
            w.wait()
        torch.ones(8, device="cuda").mul_(5)
torch.cuda.synchronize()
print("side stream", side.stream_id, "current", torch.cuda.current_stream().stream_id)
dist.destroy_process_group()
