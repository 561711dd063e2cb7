"""Phase timings of a world-1 RCCL bootstrap in a fresh process (VERDICT r03
next-round item 7: ``comm_init_s`` is ~3.4 s for the first job on a fresh box
and ~0.8 s for the next one).

Prints one JSON line with the wall time of each phase:
  import_s      import torch
  hip_init_s    torch.cuda.init() + set_device (HIP runtime, device open)
  first_kernel_s  first libtorch kernel (its code object loads lazily)
  pg_init_s     init_process_group over the TCP store (lazy communicator)
  rccl_first_s  first all_reduce + sync: ncclCommInitRank + first RCCL kernel
  rccl_second_s second all_reduce + sync

``--no-rccl`` stops after first_kernel_s (a GPU process that never touches
RCCL), to tell "first GPU process on the box" from "first RCCL communicator on
the box".  Run with NCCL_DEBUG=INFO NCCL_DEBUG_TIMESTAMP_LEVELS=ALL to get
RCCL's own timestamped init log on stderr.
"""
import json
import os
import socket
import sys
import time

T0 = time.perf_counter()


def main() -> int:
    out = {"pid": os.getpid()}
    t = time.perf_counter()
    import torch
    import torch.distributed as dist
    out["import_s"] = time.perf_counter() - t
    t = time.perf_counter()
    torch.cuda.init()
    torch.cuda.set_device(0)
    out["hip_init_s"] = time.perf_counter() - t
    t = time.perf_counter()
    x = torch.ones(1024, device="cuda")
    torch.cuda.synchronize()
    out["first_kernel_s"] = time.perf_counter() - t
    if "--no-rccl" not in sys.argv:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        t = time.perf_counter()
        dist.init_process_group("nccl", rank=0, world_size=1)
        out["pg_init_s"] = time.perf_counter() - t
        t = time.perf_counter()
        dist.all_reduce(x)
        torch.cuda.synchronize()
        out["rccl_first_s"] = time.perf_counter() - t
        t = time.perf_counter()
        dist.all_reduce(x)
        torch.cuda.synchronize()
        out["rccl_second_s"] = time.perf_counter() - t
        dist.destroy_process_group()
    out = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}
    out["total_s"] = round(time.perf_counter() - T0, 4)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
