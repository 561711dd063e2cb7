"""Time the P2P all-reduce (one-shot and two-shot kernels) against RCCL per bucket size.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 scripts/bench_p2p.py

Rank i uses GPU i % device_count.  With one GPU per rank the process group is
RCCL (``nccl``); when ranks share a GPU (the 1-GPU box) it is gloo and the
numbers only show the P2P kernels' protocol latency and local bandwidth.

Rank 0 prints one JSON line per (dtype, size) -- microseconds (MAX over ranks)
and bus bandwidth 2(W-1)/W * bytes / time for ``p2p1`` (one-shot), ``p2p2``
(two-shot) and ``rccl`` -- then one summary line per dtype with the measured
crossovers: the largest size where one-shot beats two-shot (the value for
``KDL_TUNE p2p_oneshot_bytes``) and the sizes where P2P beats RCCL (where
``KDL_ALLREDUCE=p2p`` pays).  Env: ``P2P_SIZES`` (bytes, comma list),
``P2P_DTYPES`` (bfloat16,float32), ``P2P_ITERS``.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from kubedl_amd.parallel.p2p import P2PAllReduce  # noqa: E402

DEFAULT_SIZES = "16384,65536,262144,1048576,4194304,16777216,67108864"


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ngpu = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ngpu)
    torch.cuda.set_device(dev)
    shared = world > ngpu
    kw = {} if shared else {"device_id": dev}
    dist.init_process_group("gloo" if shared else "nccl", rank=rank, world_size=world, **kw)
    sizes = [int(s) for s in os.environ.get("P2P_SIZES", DEFAULT_SIZES).split(",")]
    iters = int(os.environ.get("P2P_ITERS", "20"))
    for dtype_name in os.environ.get("P2P_DTYPES", "bfloat16,float32").split(","):
        dt = getattr(torch, dtype_name)
        esz = torch.empty(0, dtype=dt).element_size()
        buf = torch.randn(max(sizes) // esz, device=dev).to(dt)
        ar = P2PAllReduce(buf, timeout_s=120.0)
        max_oneshot = ar._ext.p2p_oneshot_max_units() * 16
        rows = []
        for nbytes in sizes:
            n = nbytes // esz
            res = {"dtype": dtype_name, "bytes": nbytes, "world": world, "shared_gpu": shared}
            ops = {"p2p2": lambda: ar.all_reduce_(0, n, oneshot=False), "rccl": lambda: dist.all_reduce(buf[:n])}
            if nbytes <= max_oneshot:
                ops["p2p1"] = lambda: ar.all_reduce_(0, n, oneshot=True)
            for name, op in ops.items():
                for _ in range(3):
                    op()
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(iters):
                    op()
                torch.cuda.synchronize()
                t = torch.tensor([(time.perf_counter() - t0) / iters], device=dev if not shared else "cpu")
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                us = float(t) * 1e6
                res[f"{name}_us"] = round(us, 1)
                res[f"{name}_busbw_GBs"] = round(2 * (world - 1) / world * nbytes / (us * 1e-6) / 1e9, 1)
            rows.append(res)
            if rank == 0:
                print(json.dumps(res), flush=True)
        ar.check()
        ar.close()
        if rank == 0:
            best = lambda r: min(r.get("p2p1_us", 1e30), r["p2p2_us"])  # noqa: E731
            oneshot_ok = [r["bytes"] for r in rows if r.get("p2p1_us", 1e30) <= r["p2p2_us"]]
            p2p_wins = [r["bytes"] for r in rows if best(r) < r["rccl_us"]]
            print(json.dumps({"dtype": dtype_name, "world": world, "summary": True,
                              "oneshot_bytes": max(oneshot_ok) if oneshot_ok else 0,
                              "p2p_beats_rccl_at_bytes": p2p_wins}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
