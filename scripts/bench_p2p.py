"""Time the P2P all-reduce against the process group's all-reduce per bucket size.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 scripts/bench_p2p.py

Rank i uses GPU i % device_count.  With one GPU per rank the process group is
RCCL (``nccl``); when ranks share a GPU (the 1-GPU box) it is gloo and the
numbers only show the P2P kernel's protocol latency and local bandwidth.
Rank 0 prints one JSON line per size.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from kubedl_amd.parallel.p2p import P2PAllReduce  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ngpu = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ngpu)
    torch.cuda.set_device(dev)
    shared = world > ngpu
    dist.init_process_group("gloo" if shared else "nccl", rank=rank, world_size=world)
    sizes = [int(s) for s in os.environ.get("P2P_SIZES", "65536,1048576,4194304,16777216,67108864").split(",")]
    buf = torch.randn(max(sizes) // 2, device=dev).to(torch.bfloat16)
    ar = P2PAllReduce(buf)
    iters = int(os.environ.get("P2P_ITERS", "20"))
    for nbytes in sizes:
        n = nbytes // 2
        res = {"bytes": nbytes, "world": world, "shared_gpu": shared}
        for name in ("p2p", "pg"):
            def op():
                if name == "p2p":
                    ar.all_reduce_(0, n)
                else:
                    dist.all_reduce(buf[:n])
            for _ in range(3):
                op()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                op()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / iters
            t = torch.tensor([dt])
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            us = float(t) * 1e6
            res[f"{name}_us"] = round(us, 1)
            # bus bandwidth convention of the collective benchmarks: 2(W-1)/W * bytes / time
            res[f"{name}_busbw_GBs"] = round(2 * (world - 1) / world * nbytes / (us * 1e-6) / 1e9, 1)
        if rank == 0:
            print(json.dumps(res), flush=True)
    ar.check()
    ar.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
