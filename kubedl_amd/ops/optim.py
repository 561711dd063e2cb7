"""Flat parameter space + fused SGD / Adam(W) driven by ``csrc/optim.hip``.

``FlatParamSpace`` relocates every trainable parameter of a module into one
flat buffer (``param``, model dtype, typically bf16) and points each ``.grad``
at a view of one flat gradient buffer (``grad``).  Consequences:

* autograd accumulates straight into the flat gradient buffer, so the DP
  all-reduce buckets (``kubedl_amd.parallel.ddp``) are plain slices -- no
  flatten/unflatten copies on the critical path;
* the optimizer is ONE kernel launch over a precomputed chunk table, with an
  fp32 master copy and fp32 state, and writes the bf16 model weights in the
  same pass.

Layout order is reverse registration order (~ the order backward produces
gradients), each region aligned to 64 elements (128 B in bf16) and padded
with zeros so every chunk is a whole number of 16-byte vectors.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from kubedl_amd.ops import _ext

ALIGN = 64
CHUNK = 16384          # elements per chunk (one thread block) for a large parameter space
CHUNK_MIN_BLOCKS = 1024


def chunk_for(total: int) -> int:
    """Elements per optimizer / pack chunk: CHUNK, halved (down to 2048) until the
    space is at least CHUNK_MIN_BLOCKS chunks -- a 2.4M-parameter CTR tower made
    150 blocks of 16384 on 256 CUs (Adam at 3.8 TB/s); ResNet-50's 25.6M keep 16384."""
    c = CHUNK
    while c > 2048 and total < c * CHUNK_MIN_BLOCKS:
        c //= 2
    return c


def _round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


@dataclass
class ParamSlot:
    name: str
    param: torch.nn.Parameter
    offset: int
    numel: int
    group: int  # 0 = weight decay, 1 = no decay


def default_no_decay(name: str, p: torch.Tensor) -> bool:
    """BN/LN affine params and biases are not decayed (standard practice)."""
    return p.dim() <= 1


class _PinnedRing:
    """Ring of pinned host int64 buffers for small per-step H2D uploads.

    The host may run a full step ahead of the GPU, so a pinned buffer is only
    rewritten after the event recorded behind its previous copy has fired.
    """

    def __init__(self, n: int, device, depth: int = 8):
        self.bufs = [torch.zeros(n, dtype=torch.int64).pin_memory() for _ in range(depth)]
        self.dev = torch.zeros(n, dtype=torch.int64, device=device)
        self.devs = [torch.zeros(n, dtype=torch.int64, device=device) for _ in range(depth)]
        self.events = [None] * depth
        self.i = 0

    def upload(self, values) -> torch.Tensor:
        k = self.i
        self.i = (self.i + 1) % len(self.bufs)
        ev = self.events[k]
        if ev is not None:
            ev.synchronize()
        hb = self.bufs[k]
        hb.numpy()[:] = values
        db = self.devs[k]
        db.copy_(hb, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.events[k] = ev
        return db


class GradPacker:
    """Gathers the autograd-owned ``.grad`` tensors of ``slots`` into the flat
    gradient buffer with one ``_C.pack_grads`` launch (csrc/multi_tensor.hip)."""

    def __init__(self, space: "FlatParamSpace", slots):
        self.space = space
        self.slots = list(slots)
        rows = []
        chunk = getattr(space, "chunk", CHUNK)
        for i, s in enumerate(self.slots):
            for st in range(0, s.numel, chunk):
                ln = min(chunk, s.numel - st)
                rows.append((i | (ln << 32), st, s.offset + st))
        self.nchunks = len(rows)
        self.chunks = torch.tensor(rows, dtype=torch.int64, device=space.device)
        self.ring = _PinnedRing(max(len(self.slots), 1), space.device) \
            if space.device.type == "cuda" else None

    def pack(self, scale: float = 1.0) -> None:
        sp = self.space
        if sp.device.type != "cuda":
            with torch.no_grad():
                for s in self.slots:
                    dst = sp._view(sp.grad, s)
                    if s.param.grad is None:
                        dst.zero_()
                    else:
                        dst.copy_(s.param.grad * scale if scale != 1.0 else s.param.grad)
            return
        ptrs = []
        for s in self.slots:
            g = s.param.grad
            if g is None:
                ptrs.append(0)
                continue
            if g.dtype != sp.grad.dtype or g.stride() != s.param.stride() or g.device != sp.device:
                g = torch.empty_strided(s.param.shape, s.param.stride(), dtype=sp.grad.dtype,
                                        device=sp.device).copy_(g)
                s.param.grad = g
            ptrs.append(g.data_ptr())
        ext = _ext.load()
        if len(ptrs) <= getattr(ext, "pack_arg_ptrs", 0):
            # pointers in the kernel arguments: no pinned upload, copy or event per call
            ext.pack_grads_ptrs(self.chunks, ptrs, sp.grad, float(scale))
            return
        src = self.ring.upload(ptrs)
        ext.pack_grads(self.chunks, src, sp.grad, float(scale))


class FlatParamSpace:
    def __init__(self, module: torch.nn.Module, dtype: torch.dtype | None = None,
                 device: torch.device | None = None, no_decay=default_no_decay,
                 reverse: bool = True, grad_mode: str = "auto"):
        named = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        if not named:
            raise ValueError("module has no trainable parameters")
        if reverse:
            named = named[::-1]
        first = named[0][1]
        self.dtype = dtype or first.dtype
        self.device = torch.device(device) if device is not None else first.device
        self.slots: list[ParamSlot] = []
        off = 0
        for n, p in named:
            if not _is_dense(p):
                raise ValueError(f"parameter {n} is not dense (strides {p.stride()})")
            self.slots.append(ParamSlot(n, p, off, p.numel(), 1 if no_decay(n, p) else 0))
            off = _round_up(off + p.numel(), ALIGN)
        self.numel = off
        self.param = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        # "pack": autograd owns .grad (no pre-set views => no per-parameter
        # accumulate-add launches); gradients are gathered into ``grad`` by one
        # multi-tensor launch.  "view": .grad are views of ``grad`` (CPU path).
        if grad_mode == "auto":
            grad_mode = "pack" if (self.device.type == "cuda" and _ext.available()) else "view"
        self.grad_mode = grad_mode
        self._gen = 0
        self._packed_gen = -1
        with torch.no_grad():
            for s in self.slots:
                view = self._view(self.param, s)
                view.copy_(s.param.data)
                s.param.data = view
                s.param.grad = self._view(self.grad, s) if grad_mode == "view" else None
        self.master = self.param.float()
        self.chunk = chunk_for(self.param.numel())
        self.chunks_cpu = self._chunk_table()
        self.chunks = self.chunks_cpu.to(self.device) if self.device.type == "cuda" else self.chunks_cpu

    @staticmethod
    def _view(flat: torch.Tensor, s: ParamSlot) -> torch.Tensor:
        return torch.as_strided(flat, s.param.shape, s.param.stride(), s.offset)

    def grad_view(self, param: torch.Tensor) -> torch.Tensor:
        """The slice of the flat gradient buffer that holds ``param``'s gradient
        (for code that writes gradients directly, e.g. the ResNet engine)."""
        idx = getattr(self, "_slot_of", None)
        if idx is None:
            idx = self._slot_of = {id(s.param): s for s in self.slots}
        return self._view(self.grad, idx[id(param)])

    def _chunk_table(self) -> torch.Tensor:
        rows = []
        for s in self.slots:
            n8 = _round_up(s.numel, 8)
            for st in range(0, n8, self.chunk):
                ln = min(self.chunk, n8 - st)
                rows.append((s.offset + st, ln | (s.group << 32)))
        return torch.tensor(rows, dtype=torch.int64)

    def zero_grad(self) -> None:
        self._gen += 1
        if self.grad_mode == "pack":
            for s in self.slots:
                s.param.grad = None
        else:
            self.grad.zero_()

    def packer(self, slots=None) -> GradPacker:
        return GradPacker(self, self.slots if slots is None else slots)

    def pack_grads(self) -> None:
        """Make ``grad`` hold this step's gradients (no-op in view mode or when
        already packed since the last ``zero_grad``, e.g. by the DP buckets).

        If no parameter holds a ``.grad`` the flat buffer is assumed to have
        been written directly and is left alone.  Parameters without a
        gradient contribute zeros (the fused update still applies weight decay
        and momentum to them, unlike ``torch.optim`` which skips them)."""
        if self.grad_mode != "pack" or self._packed_gen == self._gen:
            return
        if all(s.param.grad is None for s in self.slots):
            return
        if getattr(self, "_packer", None) is None:
            self._packer = self.packer()
        self._packer.pack()
        self._packed_gen = self._gen

    def mark_packed(self) -> None:
        self._packed_gen = self._gen

    def reattach_grads(self) -> None:
        """Re-point ``.grad`` at the flat buffer (after user code set it to None)."""
        for s in self.slots:
            if s.param.grad is None or s.param.grad.data_ptr() != self.grad.data_ptr() + \
                    s.offset * self.grad.element_size():
                s.param.grad = self._view(self.grad, s)

    def sync_params_from_master(self) -> None:
        with torch.no_grad():
            self.param.copy_(self.master)

    def sync_master_from_params(self) -> None:
        with torch.no_grad():
            self.master.copy_(self.param)

    def state_dict(self) -> dict:
        return {"master": self.master, "names": [s.name for s in self.slots],
                "offsets": [s.offset for s in self.slots]}


def _is_dense(p: torch.Tensor) -> bool:
    # non-overlapping and dense: the strided span equals numel
    if p.numel() == 0:
        return True
    span = 1 + sum((sz - 1) * st for sz, st in zip(p.shape, p.stride()))
    return span == p.numel() and all(st > 0 for st in p.stride())


class _FusedBase:
    def __init__(self, space: FlatParamSpace, lr: float, weight_decay: float):
        self.space = space
        self.lr = lr
        self.weight_decay = weight_decay
        self.step_count = 0
        self.grad_scale = 1.0  # set to 1/world by the DP wrapper

    def _use_hip(self) -> bool:
        if self.space.device.type != "cuda":
            return False
        if _ext.available():
            return True
        _ext.require_on_gpu(type(self).__name__)
        return False

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.space.zero_grad()

    def _groups_mask(self) -> torch.Tensor:
        m = getattr(self, "_wd_mask", None)
        if m is None:
            m = torch.zeros(self.space.numel, dtype=torch.float32, device=self.space.device)
            for s in self.space.slots:
                if s.group == 0:
                    m[s.offset:s.offset + s.numel] = 1.0
            self._wd_mask = m
        return m


class FusedSGD(_FusedBase):
    """SGD with momentum/dampening/nesterov, PyTorch ``torch.optim.SGD`` semantics."""

    def __init__(self, space: FlatParamSpace, lr: float, momentum: float = 0.9,
                 dampening: float = 0.0, weight_decay: float = 0.0, nesterov: bool = False):
        super().__init__(space, lr, weight_decay)
        self.momentum = momentum
        self.dampening = dampening
        self.nesterov = nesterov
        self.mom = torch.zeros_like(space.master)

    @torch.no_grad()
    def step(self) -> None:
        sp = self.space
        sp.pack_grads()
        first = self.step_count == 0
        if self._use_hip():
            _ext.load().sgd_step(sp.chunks, sp.master, self.mom, sp.grad, sp.param, float(self.lr),
                                 float(self.momentum), float(self.dampening), float(self.grad_scale),
                                 bool(self.nesterov), bool(first), [float(self.weight_decay), 0.0],
                                 [1.0, 1.0])
        else:
            g = sp.grad.float() * self.grad_scale + self.weight_decay * self._groups_mask() * sp.master
            if self.momentum != 0:
                if first:
                    self.mom.copy_(g)
                else:
                    self.mom.mul_(self.momentum).add_(g, alpha=1 - self.dampening)
                g = g + self.momentum * self.mom if self.nesterov else self.mom
            sp.master.add_(g, alpha=-self.lr)
            sp.param.copy_(sp.master)
        self.step_count += 1


class FusedAdam(_FusedBase):
    """Adam / AdamW (decoupled decay when ``adam_w``), ``torch.optim.Adam(W)`` semantics."""

    def __init__(self, space: FlatParamSpace, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, adam_w: bool = True):
        super().__init__(space, lr, weight_decay)
        self.betas = betas
        self.eps = eps
        self.adam_w = adam_w
        self.m1 = torch.zeros_like(space.master)
        self.m2 = torch.zeros_like(space.master)

    @torch.no_grad()
    def step(self) -> None:
        sp = self.space
        sp.pack_grads()
        self.step_count += 1
        b1, b2 = self.betas
        if self._use_hip():
            _ext.load().adam_step(sp.chunks, sp.master, self.m1, self.m2, sp.grad, sp.param,
                                  float(self.lr), float(b1), float(b2), float(self.eps),
                                  int(self.step_count), float(self.grad_scale), bool(self.adam_w),
                                  [float(self.weight_decay), 0.0], [1.0, 1.0])
            return
        mask = self._groups_mask()
        g = sp.grad.float() * self.grad_scale
        if self.adam_w:
            sp.master.mul_(1 - self.lr * self.weight_decay * mask)
        else:
            g = g + self.weight_decay * mask * sp.master
        self.m1.mul_(b1).add_(g, alpha=1 - b1)
        self.m2.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        denom = (self.m2.sqrt() / math.sqrt(bc2)).add_(self.eps)
        sp.master.addcdiv_(self.m1, denom, value=-self.lr / bc1)
        sp.param.copy_(sp.master)
