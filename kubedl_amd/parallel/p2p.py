"""In-place all-reduce over IPC-mapped peer buffers (one process per GPU).

``P2PAllReduce(buf)`` registers one GPU buffer per rank (the flat gradient
buffer of a ``FlatParamSpace``): every rank exports an IPC handle of its
buffer and of a small uncached signal buffer, gathers everybody's handles
through the process group (``all_gather_object``: a few hundred bytes, once)
and maps the peers.  ``all_reduce_(lo, hi)`` then sums ``buf[lo:hi]`` over all
ranks in place with one kernel on the current stream (csrc/p2p.hip:
reduce-scatter + all-gather, every peer read concurrently over its own xGMI
link; buckets up to ``KDL_TUNE p2p_oneshot_bytes`` (256 KiB) take the one-shot
kernel instead: every rank sums the whole bucket, two barriers).

Why beside RCCL: on a fully connected 8-GPU MI355X node a ring moves each
byte over one link per step and pays 2(W-1) latency-bound steps; reading the 7
peers at once uses all links and has two dependent phases, which matters most
for the small first/last buckets of a DP step.  RCCL stays the default
(``KDL_ALLREDUCE=rccl``); ``KDL_ALLREDUCE=p2p`` switches ``FlatDDP`` to this
transport when every rank is a GPU process on one node.

Failure model: a peer that never arrives makes the kernel time out (bounded
waits, ``KDL_TUNE p2p_timeout_s``, default 300 s like a process-group timeout:
the clock starts at kernel start, so it must cover host-side skew between
ranks such as a rank-0 checkpoint write) instead of hanging the GPU; the
timeout sets a bit in a host-mapped word that ``check()`` raises on (callers
check after a device sync: before it, in-flight kernels have not reported).
The worker then exits with the retryable collective-failure code and the job
controller restarts the whole gang.

Only ranks of ONE node can map each other's memory: the transport is used
only when every rank reports the same host (else ``FlatDDP`` keeps RCCL), and
the one-shot/two-shot threshold is rank 0's, so every rank picks the same
kernel and barrier slots for a bucket.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from kubedl_amd.ops import _ext

MAX_RANKS = 8


def wanted() -> bool:
    return os.environ.get("KDL_ALLREDUCE", "rccl").lower() == "p2p"


def _host_id() -> str:
    import socket
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    return f"{socket.gethostname()}/{boot}"


def single_node(group=None) -> bool:
    """Whether every rank of ``group`` runs on this host (IPC handles are node-local)."""
    world = dist.get_world_size(group)
    if int(os.environ.get("LOCAL_WORLD_SIZE", world)) != world:
        return False
    ids = [None] * world
    dist.all_gather_object(ids, _host_id(), group=group)
    return len(set(ids)) == 1


def default_timeout_s() -> float:
    from kubedl_amd.utils.tune import tune
    return tune("p2p_timeout_s", 300.0)


class P2PError(RuntimeError):
    pass


class P2PAllReduce:
    def __init__(self, buf: torch.Tensor, group=None, timeout_s: float | None = None):
        if not buf.is_cuda:
            raise ValueError("P2PAllReduce needs a GPU buffer")
        if buf.dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("P2PAllReduce supports bf16 and fp32 buffers")
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if not 1 <= self.world <= MAX_RANKS:
            raise ValueError(f"P2PAllReduce supports 1..{MAX_RANKS} ranks")
        self.buf = buf
        self.group = group
        self.timeout_s = default_timeout_s() if timeout_s is None else float(timeout_s)
        self.esz = buf.element_size()
        self.dev = buf.device.index if buf.device.index is not None else torch.cuda.current_device()
        ext = _ext.load()
        self._ext = ext
        self.sig = ext.p2p_signal_alloc(self.dev)
        self._err_host, self._err_dev = ext.p2p_error_word()
        from kubedl_amd.utils.tune import tune
        oneshot = min(tune("p2p_oneshot_bytes", 256 * 1024), ext.p2p_oneshot_max_units() * 16)
        mine = (ext.ipc_handle(buf), ext.ipc_handle(self.sig), os.getpid(), oneshot)
        allh = [None] * self.world
        dist.all_gather_object(allh, mine, group=group)
        self._mapped: list[int] = []
        self.buf_ptrs: list[int] = []
        self.sig_ptrs: list[int] = []
        for j, ((bh, boff), (sh, soff), _pid, _os) in enumerate(allh):
            if j == self.rank:
                self.buf_ptrs.append(buf.data_ptr())
                self.sig_ptrs.append(self.sig.data_ptr())
                continue
            bbase = ext.ipc_open(bh, self.dev)
            self._mapped.append(bbase)
            sbase = ext.ipc_open(sh, self.dev)
            self._mapped.append(sbase)
            self.buf_ptrs.append(bbase + boff)
            self.sig_ptrs.append(sbase + soff)
        self.epoch = 0
        # buckets up to this size take the one-shot kernel (latency-bound
        # regime); rank 0's value, so every rank picks the same kernel
        self.oneshot_bytes = int(allh[0][3])
        # every rank has zeroed its signals and mapped its peers before anyone signals
        torch.cuda.synchronize(self.dev)
        dist.barrier(group=group)

    def all_reduce_(self, lo: int = 0, hi: int | None = None, scale: float = 1.0,
                    oneshot: bool | None = None) -> torch.Tensor:
        """Sum ``buf[lo:hi]`` over ranks in place (times ``scale``), on the current stream.
        ``oneshot`` = None picks by size (must agree on every rank; it does, as the
        threshold is the same everywhere)."""
        hi = self.buf.numel() if hi is None else hi
        nbytes = (hi - lo) * self.esz
        if (lo * self.esz) % 16 or nbytes % 16 or nbytes <= 0:
            raise ValueError("P2PAllReduce: the slice must start and end on 16-byte boundaries")
        if oneshot is None:
            oneshot = nbytes <= self.oneshot_bytes
        self.epoch = (self.epoch + 1) & 0xFFFFFFFF
        off = lo * self.esz
        self._ext.p2p_allreduce([p + off for p in self.buf_ptrs], self.sig_ptrs, self._err_dev, self.rank,
                                nbytes, self.epoch, float(scale), self.buf.dtype == torch.bfloat16,
                                float(self.timeout_s), bool(oneshot))
        return self.buf[lo:hi]

    def errors(self) -> int:
        """Timeout bits set by kernels so far (reads host-mapped memory; no sync)."""
        return ctypes.c_uint32.from_address(self._err_host).value

    def check(self) -> None:
        e = self.errors()
        if e:
            raise P2PError(f"p2p all-reduce: a peer did not arrive within {self.timeout_s} s "
                           f"(phase bits {e:#x}); the gang must be restarted")

    def close(self) -> None:
        if self._mapped:
            torch.cuda.synchronize(self.dev)
            for p in self._mapped:
                self._ext.ipc_close(p)
            self._mapped = []
        if self._err_host:
            self._ext.p2p_error_free(self._err_host)
            self._err_host = 0

    def __del__(self):  # best effort; explicit close() is preferred
        try:
            self.close()
        except Exception:
            pass


class _StreamHandle:
    """``Work``-like handle: ``wait()`` makes the current stream wait for the event."""

    __slots__ = ("event",)

    def __init__(self, event: torch.cuda.Event):
        self.event = event

    def wait(self) -> None:
        torch.cuda.current_stream().wait_event(self.event)


class P2PTransport:
    """Async launcher for ``FlatDDP``: runs ``P2PAllReduce`` on a side stream
    after the gradients produced so far on the compute stream.

    Self-check: the kernel has only run with two ranks
    sharing one GPU, so its FIRST bucket is reduced twice -- through the
    process group (RCCL on a node) on an fp32 copy, and through the P2P
    kernel -- and compared before training consumes it.  A mismatch on any
    rank (agreed by a MAX all-reduce, so every rank raises together) raises
    ``P2PError``: a cross-device coherence bug stops the job instead of
    silently corrupting its gradients."""

    # test hook: this rank perturbs its own bucket after the reference copy --
    # what its peers would read through a stale or incoherent mapping
    inject_corrupt_rank: int | None = None

    def __init__(self, buf: torch.Tensor, group=None):
        self.ar = P2PAllReduce(buf, group)
        self.group = group
        self.stream = torch.cuda.Stream(device=buf.device)
        self.verified = False
        self.self_check_max_err: float | None = None

    def launch(self, lo: int, hi: int) -> _StreamHandle:
        ready = torch.cuda.Event()
        ready.record()
        self.stream.wait_event(ready)
        if not self.verified:
            self._self_check(lo, hi)
            done = torch.cuda.Event()
            done.record(self.stream)
            return _StreamHandle(done)
        with torch.cuda.stream(self.stream):
            self.ar.all_reduce_(lo, hi)
            done = torch.cuda.Event()
            done.record()
        return _StreamHandle(done)

    def _self_check(self, lo: int, hi: int) -> None:
        buf = self.ar.buf
        with torch.cuda.stream(self.stream):
            ref = buf[lo:hi].float()
            dist.all_reduce(ref, group=self.group)  # ordered before the kernel on this stream
            if self.inject_corrupt_rank is not None and self.inject_corrupt_rank == self.ar.rank:
                buf[lo:hi].add_(1.0)
            self.ar.all_reduce_(lo, hi)
        self.stream.synchronize()
        self.ar.check()
        with torch.cuda.stream(self.stream):
            want = ref.to(buf.dtype).float()  # the kernel rounds its fp32 sum once
            got = buf[lo:hi].float()
            err = (got - want).abs()
            # bf16: one rounding of two fp32 sums taken in different orders may
            # land one ulp apart; fp32: summation-order noise only
            rel = 2.0 ** -7 if buf.dtype == torch.bfloat16 else 1e-5
            tol = rel * want.abs() + 1e-6 * float(want.abs().max()) + 1e-30
            bad = torch.tensor([float((err > tol).any())], device=buf.device)
            self.self_check_max_err = float(err.max())
            dist.all_reduce(bad, op=dist.ReduceOp.MAX, group=self.group)
        self.stream.synchronize()
        if float(bad.item()) > 0:
            raise P2PError(f"p2p self-check: the P2P all-reduce of bucket [{lo}, {hi}) differs from the "
                           f"process group's on at least one rank (max |diff| here {self.self_check_max_err:.3g}); "
                           f"refusing to train on it -- run with KDL_ALLREDUCE=rccl")
        self.verified = True

    def check(self) -> None:
        self.ar.check()
