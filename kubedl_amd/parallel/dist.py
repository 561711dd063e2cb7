"""Process-group bootstrap for rank processes launched by the kubedl_amd runtime.

The launchers (``kubedl_amd.controllers.*``) export exactly the rendezvous
environment KubeDL injects into pods -- ``MASTER_ADDR``, ``MASTER_PORT``,
``WORLD_SIZE``, ``RANK`` (``controllers/pytorch/pytorchjob_controller.go:180-233``)
-- plus ``LOCAL_RANK`` and ``HIP_VISIBLE_DEVICES`` from the gang allocator.
One process drives one MI355X; the backend is ``nccl`` (= RCCL over xGMI on
ROCm) on GPU and ``gloo`` on CPU.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int
    world_size: int
    local_rank: int
    device: torch.device
    backend: str

    @property
    def is_master(self) -> bool:
        return self.rank == 0


def env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


MI355X_HBM_GB = 288.0


def apply_hbm_limit(dev: torch.device) -> float | None:
    """Cap this process's caching allocator to ``KDL_HBM_LIMIT_GB`` (the HBM
    slice the scheduler granted on a shared GPU, or a per-process cap).  An
    allocation beyond it raises OOM in THIS rank instead of starving the other
    tenants of the device.  Returns the fraction applied."""
    gb = os.environ.get("KDL_HBM_LIMIT_GB")
    if not gb or dev.type != "cuda":
        return None
    total = torch.cuda.get_device_properties(dev).total_memory / 1e9 or MI355X_HBM_GB
    frac = max(0.0, min(1.0, float(gb) / total))
    torch.cuda.set_per_process_memory_fraction(frac, dev)
    return frac


def local_device(use_gpu: bool = True) -> torch.device:
    """This rank's device: ``cuda:LOCAL_RANK`` (0 for a kubelet-launched rank,
    whose own GPU heads ``HIP_VISIBLE_DEVICES``, runtime/gpu_env.py; the
    node-local rank under ``torch.distributed.run``), or the CPU.  Every GPU
    worker picks its device here."""
    if not (use_gpu and torch.cuda.is_available()):
        return torch.device("cpu")
    ndev = torch.cuda.device_count()
    return torch.device("cuda", env_int("LOCAL_RANK", 0) % max(ndev, 1))


def init_from_env(device: str | None = None, timeout_s: float | None = None,
                  world1_group: bool = False) -> DistInfo:
    """``world1_group``: also build a (one-rank) process group at WORLD_SIZE=1,
    so a single-GPU job still runs its collectives through RCCL (SURVEY.md
    §7.2 step 5).  ``timeout_s`` defaults to ``KDL_PG_TIMEOUT_S`` (600 s)."""
    from kubedl_amd.utils.tune import warn_retired_env
    warn_retired_env()
    if timeout_s is None:
        timeout_s = float(os.environ.get("KDL_PG_TIMEOUT_S", 600))
    rank = env_int("RANK", 0)
    world = env_int("WORLD_SIZE", 1)
    local_rank = env_int("LOCAL_RANK", 0)
    use_gpu = device != "cpu" and torch.cuda.is_available()
    if use_gpu:
        dev = local_device()
        torch.cuda.set_device(dev)
        apply_hbm_limit(dev)
        # KDL_DIST_BACKEND=gloo: rehearse a multi-rank job on fewer GPUs than
        # ranks (gloo moves CUDA tensors through host memory; RCCL would
        # refuse two ranks on one device)
        backend = os.environ.get("KDL_DIST_BACKEND", "nccl")
    else:
        dev = torch.device("cpu")
        backend = "gloo"
    if (world > 1 or world1_group) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(_free_port())
        os.environ.setdefault("MASTER_PORT", "23456")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        # lazy RCCL communicator (KDL_TUNE pg_eager=1: eager, bound at init): the
        # rendezvous through the TCP store is what init waits for; building
        # the communicator (~1.1 s of topology discovery even at world 1) is
        # deferred to the first collective instead of delaying rank readiness
        from kubedl_amd.utils.tune import tune
        if backend == "nccl" and tune("pg_eager", False):
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    return DistInfo(rank, world, local_rank, dev, backend)


_NODE_WARM_WAITED = [None]  # seconds waited (None: not yet asked)


def wait_node_warm(timeout_s: float = 60.0) -> float:
    """Wait until the node warm-up (runtime/node_warm.py) has released its lock
    (``KDL_NODE_WARM_LOCK``, held exclusively by the node runtime while the
    throw-away communicator fills the code-object cache).  Called AFTER the
    rank signalled Ready and before its first communicator build, so the
    launch delay never includes the warm-up and no rank
    builds a communicator beside it.  Idempotent; returns the seconds waited."""
    if _NODE_WARM_WAITED[0] is not None:
        return 0.0
    import fcntl
    import time
    path = os.environ.get("KDL_NODE_WARM_LOCK")
    t0 = time.monotonic()
    if path and os.path.exists(path):
        try:
            fd = os.open(path, os.O_RDONLY | os.O_CLOEXEC)
        except OSError:
            fd = None
        if fd is not None:
            try:
                while True:
                    try:
                        fcntl.flock(fd, fcntl.LOCK_SH | fcntl.LOCK_NB)
                        fcntl.flock(fd, fcntl.LOCK_UN)
                        break
                    except BlockingIOError:
                        if time.monotonic() - t0 > timeout_s:  # best effort: a job still runs cold
                            break
                        time.sleep(0.01)
            finally:
                os.close(fd)
    _NODE_WARM_WAITED[0] = time.monotonic() - t0
    if _NODE_WARM_WAITED[0] > 0.05:
        import sys
        print(f"[kdl] waited {_NODE_WARM_WAITED[0]:.2f}s for the node warm-up before the first communicator",
              file=sys.stderr, flush=True)
    return _NODE_WARM_WAITED[0]


def barrier(info: DistInfo) -> None:
    if info.world_size > 1:
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def first_collective(info: DistInfo, stream=None) -> float:
    """Time (max over ranks) of the job's first collective -- with the lazy
    communicator (init_from_env) this is where RCCL bootstraps: topology
    discovery, the xGMI P2P/IPC transport setup, ring/tree building.  0 without
    a process group.

    ``stream``: issue it from the stream the job's collectives run on (the
    trainer's compute stream).  Call it only after the trainer's streams have
    run a kernel (workers/resnet50.py ResNetTrainer.touch_streams): the
    communicator's bootstrap creates RCCL's own streams, and streams first used
    after that shared hardware queues with them -- the weight-gradient side
    stream lost its overlap, 19.4 -> 22.0 ms per ResNet-50 step at world 1
    (26.9 ms bootstrapped from the null stream); profiles/r03_stream_touch_ab.txt."""
    import contextlib
    import time
    if not dist.is_initialized():
        return 0.0
    wait_node_warm()
    ctx = torch.cuda.stream(stream) if (stream is not None and info.device.type == "cuda") \
        else contextlib.nullcontext()
    with ctx:
        t0 = time.perf_counter()
        t = torch.ones(1, device=info.device)
        dist.all_reduce(t)
        if info.device.type == "cuda":
            torch.cuda.synchronize(info.device)
        dt = time.perf_counter() - t0
        m = torch.tensor([dt], dtype=torch.float64, device=info.device)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        return float(m.item())


def all_reduce_max(value: float, info: DistInfo) -> float:
    if info.world_size == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=info.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shutdown(info: DistInfo) -> None:
    if dist.is_initialized():
        dist.destroy_process_group()


# ---------------------------------------------------------------- failure exit
# A rank whose collective fails because a PEER died (gloo "Connection closed by
# peer", an RCCL/NCCL error or watchdog abort, a P2P all-reduce timeout) exits
# with 138 -- the reference's retryable "user retry" code
# (pkg/util/train/train_util.go:18-52) -- instead of 1 (permanent), so an
# ExitCode job restarts its gang instead of failing on the survivor's symptom.
COMM_FAILURE_EXIT = 138
# message fragments that only a vanished or hung PEER produces (gloo's TCP pair,
# RCCL's system/remote errors, the collective watchdog); anything else -- an RCCL
# usage/argument error, an uninitialised group, a user-code "timed out" -- is a
# deterministic bug and must fail the job permanently (exit 1), not loop
# through gang restarts until backoffLimit
_PEER_GONE = ("connection closed by peer", "connection reset by peer", "broken pipe",
              "remote process exited", "unhandled system error", "network error",
              "watchdog caught collective operation timeout")
_NOT_PEER = ("invalid usage", "invalid argument", "has not been initialized", "not been initialized",
             "out of memory")


def is_comm_failure(exc: BaseException) -> bool:
    """True when ``exc`` means a peer rank is gone (retryable gang restart)."""
    msg = str(exc).lower()
    if any(m in msg for m in _NOT_PEER):
        return False
    if type(exc).__name__ == "P2PError":  # parallel/p2p.py: peer missed the arrival window
        return True
    net_error = getattr(dist, "DistNetworkError", None)
    if net_error is not None and isinstance(exc, net_error):
        return True
    # rendezvous: a peer died before (or while) joining the TCP store -- rank 0
    # times out "waiting for clients", the others lose the store
    store_error = getattr(dist, "DistStoreError", None)
    if store_error is not None and isinstance(exc, store_error):
        return True
    if "waiting for clients" in msg or ("store" in msg and "timed out" in msg):
        return True
    if not isinstance(exc, (RuntimeError, ConnectionError)):
        return False
    if any(m in msg for m in _PEER_GONE):
        return True
    # gloo's collective timeout: the peer hung or died without closing its socket
    return "gloo" in msg and "timed out" in msg


def run_rank(main, *args, **kw) -> int:
    """Run a worker ``main``; a collective failure exits COMM_FAILURE_EXIT."""
    try:
        return main(*args, **kw)
    except BaseException as e:  # noqa: BLE001
        if not is_comm_failure(e):
            raise
        import sys
        import traceback
        traceback.print_exc()
        print(f"[kdl] collective failure ({type(e).__name__}): a peer rank is gone; "
              f"exiting {COMM_FAILURE_EXIT} so the job restarts its gang", file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(COMM_FAILURE_EXIT)
