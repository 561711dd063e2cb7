"""Which streams share a hardware queue?  Overlap ratio of two 3 ms spin
kernels (1 = concurrent, 2 = serialised), before and after a world-1 RCCL
process group is created (ops/streams.py explains why it matters)."""
import os
import socket

import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

from kubedl_amd.ops.streams import dedicated_stream, overlap_ratio

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
null = torch.cuda.default_stream(dev)
pool_a = torch.cuda.Stream(dev)
ded_a = dedicated_stream(dev)
ded_b = dedicated_stream(dev)
overlap_ratio(null, pool_a, 500)  # warm-up (kernel load)
print("before PG: null|pool", round(overlap_ratio(null, pool_a), 2), " null|ded", round(overlap_ratio(null, ded_a), 2),
      " ded|ded", round(overlap_ratio(ded_a, ded_b), 2), flush=True)
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
t = torch.ones(1, device=dev)
dist.all_reduce(t)
torch.cuda.synchronize()
pool_b = torch.cuda.Stream(dev)
ded_c = dedicated_stream(dev)
print("after PG: null|pool_a", round(overlap_ratio(null, pool_a), 2), " null|pool_b", round(overlap_ratio(null, pool_b), 2),
      " pool_a|pool_b", round(overlap_ratio(pool_a, pool_b), 2), " ded_a|ded_b", round(overlap_ratio(ded_a, ded_b), 2),
      " ded_a|ded_c", round(overlap_ratio(ded_a, ded_c), 2), " ded_c|pool_b", round(overlap_ratio(ded_c, pool_b), 2), flush=True)
dist.destroy_process_group()
