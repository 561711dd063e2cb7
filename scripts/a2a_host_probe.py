"""Host cost of one world-1 RCCL all-to-all: torch.distributed.all_to_all_single
(Python checks + dispatcher) vs the process group's alltoall_base called
directly, issue time per call with the GPU busy (no syncs inside)."""
import os
import time

import torch
import torch.distributed as dist


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29631")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    x = torch.zeros(4096, dtype=torch.bfloat16, device="cuda")  # tiny: host cost, not copy time
    y = torch.empty_like(x)
    pg = dist.distributed_c10d._get_default_group()
    opts = dist.AllToAllOptions()
    for _ in range(20):
        dist.all_to_all_single(y, x)
    torch.cuda.synchronize()
    for tag in ("all_to_all_single", "pg.alltoall_base", "all_to_all_single", "pg.alltoall_base"):
        # (no spin ahead: RCCL caps its outstanding ops, a busy GPU blocks the host ~300 us per call)
        n = 300
        t0 = time.perf_counter()
        for _ in range(n):
            if tag == "all_to_all_single":
                dist.all_to_all_single(y, x)
            else:
                pg.alltoall_base(y, x, [], [], opts)
        dt = (time.perf_counter() - t0) / n * 1e6
        torch.cuda.synchronize()
        print(f"{tag:20s} {dt:6.1f} us/call (host issue)", flush=True)
    assert torch.equal(x, y)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
