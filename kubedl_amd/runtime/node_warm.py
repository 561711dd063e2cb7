"""Node warm-up: build one world-1 RCCL communicator in a throw-away process.

Why (profiles/r04_comm_init_phases.txt, r04_comgr_cache.txt): a job's first
collective spends ~3.5 s inside ``ncclCommInitRank`` on a fresh node and
~0.9 s on every later one.  The difference is the ROCm code-object manager's
on-disk cache (``$XDG_CACHE_HOME/comgr``, default ``~/.cache/comgr``): the
first process that loads librccl's device code extracts its gfx950 code
object (a ~270 MB entry) from the library's compressed offload bundle and
stores it there; every later process reads the stored object.  With
``AMD_COMGR_CACHE=0`` or an empty cache directory every process pays the
3.5 s.  The node runtime (runtime/zygote.py ``ZygoteClient``) runs this once
at start-up, beside the page-cache prefetch, so the jobs it launches find the
cache warm -- the job-level analogue of a node image that ships warm caches.

Run as ``python -m kubedl_amd.runtime.node_warm``; prints one JSON line.  It
is a separate process: the kubelet and the rank zygote never initialise the
GPU (the zygote forks ranks).
"""
from __future__ import annotations

import json
import os
import socket
import sys
import time


def main() -> int:
    t0 = time.perf_counter()
    out = {"warm": False}
    try:
        import torch
        import torch.distributed as dist
        if not torch.cuda.is_available():
            out["reason"] = "no GPU"
        else:
            torch.cuda.set_device(0)
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
            t = torch.ones(1, device="cuda")
            dist.all_reduce(t)
            torch.cuda.synchronize()
            dist.destroy_process_group()
            out["warm"] = True
    except Exception as e:  # warming is best-effort: a job still works cold
        out["error"] = f"{type(e).__name__}: {e}"
    out["warm_s"] = round(time.perf_counter() - t0, 3)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
