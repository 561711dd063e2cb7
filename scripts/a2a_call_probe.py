"""Host cost of one world-1 RCCL all-to-all call: torch.distributed's
all_to_all_single wrapper vs the process group's alltoall_base directly.
The fixed-capacity CTR exchange (models/ctr.py) issues three per step and its
host issue time equals its step time (profiles/r05_ctr_segment_reduce_adagrad.txt)."""
import datetime
import os
import time

import torch
import torch.distributed as dist


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, timeout=datetime.timedelta(seconds=120), device_id=dev)
    inp = torch.zeros(106497, dtype=torch.int64, device=dev)
    out = torch.empty_like(inp)
    pg = dist.distributed_c10d._get_default_group()
    opts = dist.AllToAllOptions()
    for name, fn in (("all_to_all_single", lambda: dist.all_to_all_single(out, inp)),
                     ("pg.alltoall_base", lambda: pg.alltoall_base(out, inp, [], [], opts)),
                     ("all_to_all_single", lambda: dist.all_to_all_single(out, inp)),
                     ("pg.alltoall_base", lambda: pg.alltoall_base(out, inp, [], [], opts))):
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        n = 2000
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        host = (time.perf_counter() - t0) / n * 1e6
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / n * 1e6
        print(f"{name:20s} host {host:6.1f} us/call  wall {wall:6.1f} us/call", flush=True)
    assert torch.equal(out, inp)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
