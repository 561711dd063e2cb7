"""Data-parallel gradient synchronisation over RCCL/xGMI with backward overlap.

Works on a ``FlatParamSpace``: gradients already live in one flat buffer laid
out in (approximately) the order backward produces them, so a bucket is just
a contiguous slice ``grad[lo:hi]``.  A post-accumulate-grad hook per
parameter counts down its bucket; when a bucket is complete its all-reduce
(SUM, averaging is folded into the fused optimizer's ``grad_scale``) is
issued asynchronously, overlapping the rest of backward.  ``finish()`` waits
for the outstanding collectives before the optimizer step.

Bucket sizing for MI355X: 8 GPUs on point-to-point xGMI (7 links x ~153 GB/s
per GPU) means a ring all-reduce of B bytes costs ~2(n-1)/n * B / link-bw plus
a per-collective latency of tens of microseconds.  ResNet-50 has 51 MB of
bf16 gradients; ~12 MB buckets give 4-5 collectives, enough to overlap all but
the last (smallest, first-layer) bucket with backward while staying far above
the latency-bound regime.  The first bucket is capped smaller so the first
collective starts early.

Transport: RCCL (``dist.all_reduce``) by default; ``KDL_ALLREDUCE=p2p`` runs
each bucket through ``kubedl_amd.parallel.p2p`` instead (one kernel reading
all peers' IPC-mapped gradient buffers over their own xGMI links), on a side
stream ordered after the bucket's producers.

The reference has no collective code; this is the DP
strategy a PyTorchJob's env (``MASTER_ADDR/PORT``, ``WORLD_SIZE``, ``RANK``)
exists to enable.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from kubedl_amd.ops.optim import FlatParamSpace
from kubedl_amd.parallel import p2p


class Bucket:
    __slots__ = ("lo", "hi", "slots", "pending", "handle", "packer", "wide")

    def __init__(self, lo: int, hi: int, slots):
        self.lo, self.hi, self.slots = lo, hi, slots
        self.pending = len(slots)
        self.handle = None
        self.packer = None
        self.wide = None  # fp32 copy of a bf16 bucket being reduced (reduce_fp32)


def reduce_fp32_wanted() -> bool:
    """``KDL_TUNE ddp_reduce=fp32``: RCCL buckets of a bf16 gradient buffer are summed in
    fp32 (2x the bytes on the links, one bf16 rounding at the end instead of one
    per ring step; tests/test_multigpu.py bounds the bf16 error at world 8)."""
    from kubedl_amd.utils.tune import tune
    return tune("ddp_reduce", "bf16").lower() == "fp32"


class FlatDDP:
    def __init__(self, space: FlatParamSpace, world_size: int, process_group=None,
                 bucket_cap_mb: float = 12.0, first_bucket_mb: float = 2.0,
                 broadcast_from: int | None = 0, direct: bool = False):
        """``direct``: gradients are written straight into ``space.grad`` by the
        caller (the ResNet engine), which announces each finished parameter with
        ``ready(param)`` -- no autograd hooks, no pack kernels."""
        self.space = space
        self.direct = direct
        self.world = world_size
        # KDL_TUNE ddp_world1=1: a world-1 job still buckets and all-reduces (RCCL's
        # one-rank all-reduce) -- exercises the collective path the N-GPU job
        # takes; off by default (it is an identity).  RCCL's one-rank in-place
        # all-reduce launches nothing, so ddp_world1=copy issues each bucket
        # as a one-rank all_gather into a scratch buffer instead: a bucket-sized
        # RCCL copy on the process group's own stream, event-joined like the
        # N-GPU collective (the stream / hardware-queue shape of world 8)
        from kubedl_amd.utils.tune import tune
        w1 = tune("ddp_world1", "0")
        self.active = world_size > 1 or (w1 in ("1", "copy") and dist.is_initialized())
        self.world1_copy = world_size == 1 and w1 == "copy" and self.active
        self._w1_scratch = None
        self.pg = process_group
        self.buckets: list[Bucket] = []
        self._hooks = []
        self.transport = None
        self.reduce_fp32 = reduce_fp32_wanted()
        # timing: per-step device time the caller's stream waits for the buckets
        # in finish() (the EXPOSED all-reduce time; everything else overlapped the
        # backward) -- CUDA events, read once by exposed_ms()
        self.timing = False
        self._tev = []
        # producers on a second stream (the ResNet engine's weight-gradient
        # stream): a bucket's collective is issued on that stream after it has
        # joined the current one, so it waits for both without stalling the
        # current stream's remaining backward work
        self.join_stream = None
        if self.active:
            if broadcast_from is not None and world_size > 1:
                from kubedl_amd.parallel.dist import wait_node_warm
                wait_node_warm()  # (no-op unless this is the rank's first communicator build)
                with torch.no_grad():
                    dist.broadcast(space.param, broadcast_from, group=process_group)
                    space.sync_master_from_params()
            self._build_buckets(bucket_cap_mb, first_bucket_mb)
            if p2p.wanted() and space.grad.is_cuda and p2p.single_node(process_group):
                self.transport = p2p.P2PTransport(space.grad, process_group)
            if not direct:
                self._install_hooks()

    def _build_buckets(self, cap_mb: float, first_mb: float) -> None:
        esz = self.space.grad.element_size()
        cur, lo = [], None
        cap = first_mb * 2 ** 20
        for s in self.space.slots:
            if lo is None:
                lo = s.offset
            cur.append(s)
            hi = s.offset + s.numel
            if (hi - lo) * esz >= cap:
                self.buckets.append(Bucket(lo, _end(self.space, s), cur))
                cur, lo = [], None
                cap = cap_mb * 2 ** 20
        if cur:
            self.buckets.append(Bucket(lo, _end(self.space, cur[-1]), cur))
        if self.space.grad_mode == "pack" and not self.direct:
            for b in self.buckets:
                b.packer = self.space.packer(b.slots)
        self._slot_bucket = {}
        for b in self.buckets:
            for s in b.slots:
                self._slot_bucket[id(s.param)] = b

    def _install_hooks(self) -> None:
        for b in self.buckets:
            for s in b.slots:
                self._hooks.append(s.param.register_post_accumulate_grad_hook(self._on_grad))

    def _launch(self, b: Bucket) -> None:
        if b.packer is not None:
            b.packer.pack()
            for s in b.slots:  # gradients now live in the bucket: free autograd's copies
                s.param.grad = None
        js = self.join_stream
        if js is not None:
            js.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(js):
                self._issue(b)
        else:
            self._issue(b)

    def _issue(self, b: Bucket) -> None:
        if self.world1_copy:
            if self._w1_scratch is None:
                self._w1_scratch = torch.empty_like(self.space.grad)
            b.handle = dist.all_gather_into_tensor(self._w1_scratch[b.lo:b.hi], self.space.grad[b.lo:b.hi],
                                                   group=self.pg, async_op=True)
            return
        if self.transport is not None:
            b.handle = self.transport.launch(b.lo, b.hi)
        elif self.reduce_fp32 and self.space.grad.dtype != torch.float32:
            b.wide = self.space.grad[b.lo:b.hi].float()
            b.handle = dist.all_reduce(b.wide, group=self.pg, async_op=True)
        else:
            b.handle = dist.all_reduce(self.space.grad[b.lo:b.hi], group=self.pg, async_op=True)

    def _on_grad(self, p: torch.Tensor) -> None:
        b = self._slot_bucket[id(p)]
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    def ready(self, p: torch.Tensor) -> None:
        """Direct mode: ``p``'s gradient slice is final (launches its bucket's
        all-reduce when it was the bucket's last parameter)."""
        if self.active:
            self._on_grad(p)

    def finish(self) -> None:
        """Wait for every bucket (launching any whose params got no gradient)."""
        if not self.active:
            return  # the optimizer packs (FlatParamSpace.pack_grads)
        for b in self.buckets:
            if b.handle is None:
                self._launch(b)
        timed = self.timing and self.space.grad.is_cuda
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        for b in self.buckets:
            b.handle.wait()
            b.handle = None
            b.pending = len(b.slots)
            if b.wide is not None:
                self.space.grad[b.lo:b.hi].copy_(b.wide)
                if b.wide.is_cuda:  # allocated on the join stream, last read here
                    b.wide.record_stream(torch.cuda.current_stream())
                b.wide = None
        if timed:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self._tev.append((e0, e1))
        if self.transport is not None:
            # bits of EARLIER steps only (no sync here); the authoritative check
            # follows a device sync: ResNetTrainer.check_transport, run before
            # every checkpoint and after the last step
            self.transport.check()
        self.space.mark_packed()

    def exposed_ms(self, reset: bool = True) -> float | None:
        """Mean device time per step the compute stream waited for the bucket
        collectives (syncs on the recorded events)."""
        if not self._tev:
            return None
        self._tev[-1][1].synchronize()
        ms = sum(a.elapsed_time(b) for a, b in self._tev) / len(self._tev)
        if reset:
            self._tev.clear()
        return ms

    def describe(self) -> dict:
        """The bucket plan (bench JSON ``ddp`` block)."""
        esz = self.space.grad.element_size()
        return {"active": self.active, "world": self.world,
                "transport": ("p2p" if self.transport is not None else "rccl") if self.active else None,
                "buckets": len(self.buckets),
                "bucket_mb": [round((b.hi - b.lo) * esz / 2 ** 20, 2) for b in self.buckets],
                "grad_mb": round(self.space.numel * esz / 2 ** 20, 2),
                "reduce_dtype": "fp32" if self.reduce_fp32 else str(self.space.grad.dtype).replace("torch.", "")}

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks.clear()


def _end(space: FlatParamSpace, s) -> int:
    """Bucket end = start of the next slot's region (include the zero pad)."""
    idx = space.slots.index(s)
    if idx + 1 < len(space.slots):
        return space.slots[idx + 1].offset
    return space.numel
