"""PyTorchJob distributed smoke worker (what ``kubedl/pytorch-dist-example`` does
in ``example/pytorch/pytorch_job_mnist_mpi.yaml``: a point-to-point send/recv
round between ranks), on RCCL/xGMI when a GPU is assigned, gloo otherwise.

Rank 0 sends a tensor to every other rank, each rank adds its rank and sends
it back; then one all_reduce checks the collective path.  Exits non-zero on
any mismatch, so the job's status reflects the communication health.
"""
from __future__ import annotations

import argparse
import sys

import torch
import torch.distributed as dist

from kubedl_amd.parallel import dist as kdist
from kubedl_amd.workers import common


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--numel", type=int, default=1 << 20)
    ap.add_argument("--cpu", action="store_true")
    args, _ = ap.parse_known_args(argv)
    info = kdist.init_from_env("cpu" if args.cpu else None)
    common.signal_ready({"rank": info.rank})
    dev = info.device
    ok = True
    if info.world_size > 1:
        t = torch.zeros(args.numel, device=dev)
        if info.rank == 0:
            for r in range(1, info.world_size):
                dist.send(torch.full((args.numel,), float(r), device=dev), dst=r)
            for r in range(1, info.world_size):
                dist.recv(t, src=r)
                ok &= bool(torch.all(t == 2.0 * r))
        else:
            dist.recv(t, src=0)
            dist.send(t + info.rank, dst=0)
        a = torch.full((args.numel,), float(info.rank + 1), device=dev)
        dist.all_reduce(a)
        exp = info.world_size * (info.world_size + 1) / 2
        ok &= bool(torch.all(a == exp))
    print(f"rank {info.rank}/{info.world_size} on {dev} ({info.backend}): {'OK' if ok else 'MISMATCH'}", flush=True)
    kdist.shutdown(info)
    return 0 if ok else 1


if __name__ == "__main__":
    from kubedl_amd.parallel.dist import run_rank
    sys.exit(run_rank(main))
