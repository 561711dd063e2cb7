"""Sparse-embedding CTR model for the XDLJob data plane.

XDL (the reference's XDLJob payload, ``example/xdl/xdl_job_mnist.yaml``) trains
click-through-rate models whose sparse embeddings live on parameter servers.
MI355X-first re-design:

* **Embedding shards on GPUs, collective push/pull.**  The PS role becomes
  "owner of a row shard" (row ``id % n_owners``): a pull is an RCCL
  all-to-all of de-duplicated ids to their owners, a HIP row gather on the
  owner (``embed_gather``), and an all-to-all of the rows back; a push is the
  reverse with the owner summing duplicate contributions and applying the
  sparse optimizer in ONE kernel (``segment_adagrad``: sort-based segment
  sum + Adagrad on the owned rows, no atomics, bitwise reproducible).  With
  PS replicas in the job the PS ranks own the shards; without, the workers do.
* **De-duplication before communication.**  Each worker ``torch.unique``s
  its batch ids; gradient rows of repeated ids are pre-summed locally
  (``segment_reduce``) so only one row per unique id crosses xGMI.
* **Dense tower on MFMA.**  ``FusedLinear`` runs forward as the hand-written
  ``gemm_bias_act`` kernel (v_mfma_f32_32x32x16_bf16, bias + ReLU fused in the
  epilogue; the wide layers on the LDS-DMA igemm loop); the training step
  folds each ReLU mask + bias gradient into the launch that produces the
  gradient (``head_bce_bwd`` relu_x, ``gemm_dgrad_relu``: dx = dz W masked,
  with its column sums; the autograd path keeps ``relu_bwd_dbias``), and dW
  runs on the LDS-DMA weight-gradient kernel
  (csrc/wgrad_dma.hip); the 1-wide logit layer is fused with the sigmoid-BCE
  loss (``head_bce_fwd/bwd``: a GEMV per row + loss + dlogit in one pass,
  dx / dw / db in one backward pass) -- no vendor GEMM in the step.

On CPU (tests) every op has a torch composition with the same semantics.
"""
from __future__ import annotations

import collections
import math
import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from kubedl_amd.ops import _ext


# ---------------------------------------------------------------- dense tower
class _FusedLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu):
        ext = _ext.load()
        y = ext.gemm_bias_act(x.contiguous(), w.contiguous(), b, bool(relu))
        ctx.save_for_backward(x, w, y)
        ctx.relu = relu
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dx, dw, db = _linear_bwd(dy, x, w, y, ctx.relu, ctx.has_b)
        return dx, dw, db, None


def _linear_bwd(dy, x, w, y, relu: bool, has_b: bool):
    """(dx, dW, db) of y = act(x W^T + b) on the kdl kernels (the backward of
    _FusedLinearFn; DenseTower.train_step fuses the ReLU backward and the bias
    gradient into the producing launches instead, _tower_layer_bwd)."""
    ext = _ext.load()
    dy = dy.contiguous()
    # db straight in the parameter dtype (bf16): no zero-fill, no conversion launch
    dz, db = ext.relu_bwd_dbias(dy, y if relu else None, w.dtype == torch.bfloat16)
    fout, fin = w.shape
    # dx = dz . W on the same MFMA kernel as the forward, W read as [K, N]
    # (transposed LDS reads: no per-step W^T copy)
    if fin % 8 == 0:
        dx = ext.gemm_bias_act(dz, w.contiguous(), None, False, True)
    else:
        dx = ext.gemm_bias_act(dz, w.t().contiguous(), None, False)
    dw = _dw_of(ext, dz, x, w)
    return dx, dw, ((db if db.dtype == w.dtype else db.to(w.dtype)) if has_b else None)


_WS = {}


def _wgrad_workspace(ext, M, N, K, device):
    key = (M, N, K, str(device))
    need = ext.conv1x1_wgrad_splits(M, N, K, True) * N * K  # (the tile mode may change: set_wgrad_big)
    ws = _WS.get(key)
    if ws is None or ws.numel() < need:
        ws = _WS[key] = torch.empty(need, device=device)
    return ws


def fused_linear(x, w, b=None, relu=False):
    if x.is_cuda and _ext.available() and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0:
        return _FusedLinearFn.apply(x, w, b, relu)
    if x.is_cuda and not _ext.available():
        _ext.require_on_gpu("fused_linear")
    y = torch.nn.functional.linear(x, w, b)
    return torch.relu(y) if relu else y


class _HeadBCEFn(torch.autograd.Function):
    """mean_m BCEWithLogits(x[m] . w + b, y[m]) for a [K] -> 1 head."""

    @staticmethod
    def forward(ctx, x, w, b, y):
        x = x.contiguous()
        loss, logit, dlogit = _head_fwd(x, w, b, y)
        ctx.save_for_backward(x, w, dlogit)
        ctx.b_dtype = b.dtype
        ctx.mark_non_differentiable(logit)
        return loss.view(()), logit

    @staticmethod
    def backward(ctx, gloss, _glogit):
        x, w, dlogit = ctx.saved_tensors
        dx, dw, db = _head_bwd(x, w, ctx.b_dtype, dlogit, gloss.float().reshape(1).contiguous())
        return dx, dw, db, None


def _head_fwd(x, w, b, y):
    """(mean loss [1], logits, dloss/dlogit) of the fused logit head + BCE."""
    ext = _ext.load()
    bb = b.reshape(1) if b.dtype in (torch.bfloat16, torch.float32) else b.float().reshape(1)
    # the kernel's last block folds the per-block losses into the mean (no reduce launch)
    logit, dlogit, _part, loss = ext.head_bce_fwd(x, w.reshape(-1).contiguous(), bb.contiguous(),
                                                  y.float().contiguous())
    return loss, logit, dlogit


def _head_bwd(x, w, b_dtype, dlogit, gloss, relu_x: bool = False):
    """(dx, dW, db) of the logit head; ``relu_x`` (x is the last tower layer's
    ReLU output): dx comes back masked by x > 0 -- that layer's pre-activation
    gradient -- and a fourth value, that layer's bias gradient (bf16), is
    summed in the same launch (no relu_bwd_dbias pass)."""
    ext = _ext.load()
    # dW / db summed over the per-block partials in a fixed order by the kernel's
    # last block (deterministic), already bf16
    out = ext.head_bce_bwd(x, w.reshape(-1).contiguous(), dlogit, 1.0 / x.shape[0], gloss, relu_x)
    dx, dw, db = out[0], out[1], out[2]
    dw = dw.reshape(w.shape) if w.dtype == dw.dtype else dw.to(w.dtype).reshape(w.shape)
    db = db if b_dtype == db.dtype else db.to(b_dtype)
    if relu_x:
        return dx, dw, db, out[5]
    return dx, dw, db


_FUSED_RELU_BWD = []


def _fused_relu_bwd() -> bool:
    if not _FUSED_RELU_BWD:
        from ..utils.tune import tune
        # each fused launch ends in a ticketed cross-block reduction: with the
        # release / acquire hand-off (KDL_TUNE ctr_handoff=0) the release wrote
        # back the freshly stored gradient tile and the fusion lost (10.94-10.96
        # vs 11.01-11.02 M samples/s, profiles/r06_ctr_fused_relu_bwd.txt); with
        # the fence-free sc1 hand-off (default) it wins: 11.54-11.58 vs 11.43-11.47
        # (profiles/r06_ctr_handoff.txt)
        _FUSED_RELU_BWD.append(bool(tune("ctr_fused_relu_bwd", 1)))
    return _FUSED_RELU_BWD[0]


def _tower_layer_bwd(dz, x, w, x_relu: bool):
    """(dx, dW, dbx) of z = x W^T + b given dz = dL/dz.  ``x_relu`` (x is the
    previous layer's ReLU output): dx comes back masked by x > 0 (that layer's
    dz) with dbx = its column sums, that layer's bias gradient, from the same
    launch (``gemm_dgrad_relu``); else dbx is None."""
    ext = _ext.load()
    fout, fin = w.shape
    dbx = None
    if fin % 8 == 0:
        if x_relu:
            dx, dbx = ext.gemm_dgrad_relu(dz, w.contiguous(), x)
        else:
            dx = ext.gemm_bias_act(dz, w.contiguous(), None, False, True)
    else:
        dx = ext.gemm_bias_act(dz, w.t().contiguous(), None, False)
        if x_relu:
            dx, dbx = ext.relu_bwd_dbias(dx, x, True)
    return dx, _dw_of(ext, dz, x, w), dbx


def _dw_of(ext, dz, x, w):
    """dW = dz^T x: the reduction over the batch is the weight-gradient form of
    csrc/wgrad_dma.hip (both operands row-major, LDS-DMA + transposed LDS reads;
    split-batch fp32 slabs, fixed-order reduce); solo: no weight-gradient side
    stream here, so the split count that fills the chip."""
    fout, fin = w.shape
    if fout % 64 == 0 and fin % 64 == 0:
        B = x.shape[0]
        ws = _wgrad_workspace(ext, B, fout, fin, x.device)
        dw = torch.empty(fout, fin, dtype=w.dtype, device=w.device)
        ext.conv1x1_wgrad(dz, x, None, ws, dw, 1.0, B, fout, fin, 0, 0, 0, 0, 1, True)
        return dw
    return (dz.t() @ x).to(w.dtype)


def head_bce(x, w, b, y):
    """(loss, logits) of the logit layer + mean sigmoid BCE."""
    if x.is_cuda and _ext.available() and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0:
        return _HeadBCEFn.apply(x, w, b, y)
    if x.is_cuda and not _ext.available():
        _ext.require_on_gpu("head_bce")
    logit = torch.nn.functional.linear(x, w, b).float().squeeze(-1)
    return torch.nn.functional.binary_cross_entropy_with_logits(logit, y.float()), logit.detach()


class FusedLinear(nn.Module):
    def __init__(self, fin: int, fout: int, relu: bool):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(fout, fin))
        self.bias = nn.Parameter(torch.zeros(fout))
        self.relu = relu
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))

    def forward(self, x):
        return fused_linear(x, self.weight, self.bias, self.relu)


class DenseTower(nn.Module):
    def __init__(self, fin: int, hidden=(1024, 512, 256)):
        super().__init__()
        dims = [fin] + list(hidden)
        self.layers = nn.ModuleList([FusedLinear(a, b, True) for a, b in zip(dims[:-1], dims[1:])])
        self.head = nn.Linear(dims[-1], 1)

    def forward(self, x):
        for l in self.layers:
            x = l(x)
        return self.head(x).float().squeeze(-1)

    def fused_ok(self, x) -> bool:
        return (x.is_cuda and _ext.available() and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0
                and all(l.weight.dtype == torch.bfloat16 for l in self.layers))

    @torch.no_grad()
    def train_step(self, x, y, on_ready=None):
        """Forward + backward of the tower without the autograd engine: the same
        kernels as ``loss`` + ``backward`` (_FusedLinearFn, _HeadBCEFn) called in
        order -- bitwise the same loss and gradients (tests/test_ctr.py), a
        fraction of the host time of a 4-node autograd graph in a ~0.4 ms step.
        Parameter gradients are assigned to ``.grad`` (``on_ready(p)`` after each,
        e.g. FlatDDP.ready); returns (loss, dL/dx)."""
        acts = [x.contiguous()]
        for l in self.layers:
            acts.append(_ext.load().gemm_bias_act(acts[-1], l.weight.contiguous(), l.bias, bool(l.relu)))
        hw, hb = self.head.weight, self.head.bias
        loss, _logit, dlogit = _head_fwd(acts[-1], hw, hb, y)
        one = getattr(self, "_one", None)
        if one is None or one.device != x.device:
            one = self._one = torch.ones(1, device=x.device)
        # every ReLU backward and bias gradient fused into the launch that
        # produces the gradient (head backward, then each layer's data-gradient
        # GEMM): dz is the pre-activation gradient of layer i, db its bias grad
        # (KDL_TUNE ctr_fused_relu_bwd=0: the relu_bwd_dbias pass above)
        if not _fused_relu_bwd():  # A/B: the separate relu_bwd_dbias pass per layer
            dy, dw, db = _head_bwd(acts[-1], hw, hb.dtype, dlogit, one)
            for p, g in ((hw, dw), (hb, db)):
                p.grad = g
                if on_ready is not None:
                    on_ready(p)
            for i in range(len(self.layers) - 1, -1, -1):
                l = self.layers[i]
                dy, dw, db = _linear_bwd(dy, acts[i], l.weight, acts[i + 1], l.relu, True)
                for p, g in ((l.weight, dw), (l.bias, db)):
                    p.grad = g
                    if on_ready is not None:
                        on_ready(p)
            return loss.view(()), dy
        last = self.layers[-1]
        if last.relu:
            dz, dw, db, db_z = _head_bwd(acts[-1], hw, hb.dtype, dlogit, one, relu_x=True)
        else:
            dz, dw, db = _head_bwd(acts[-1], hw, hb.dtype, dlogit, one)
            db_z = None
        for p, g in ((hw, dw), (hb, db)):
            p.grad = g
            if on_ready is not None:
                on_ready(p)
        for i in range(len(self.layers) - 1, -1, -1):
            l = self.layers[i]
            if db_z is None:  # a layer without ReLU: its bias gradient from dz itself
                dz, db_z = _ext.load().relu_bwd_dbias(dz, None, True)
            x_relu = i > 0 and self.layers[i - 1].relu
            dx, dw, db_prev = _tower_layer_bwd(dz, acts[i], l.weight, x_relu)
            db = db_z if db_z.dtype == l.bias.dtype else db_z.to(l.bias.dtype)
            for p, g in ((l.weight, dw), (l.bias, db)):
                p.grad = g
                if on_ready is not None:
                    on_ready(p)
            dz, db_z = dx, db_prev
        return loss.view(()), dz

    def loss(self, x, y):
        """Training step forward: (mean BCE loss, logits); the head runs fused
        with the loss (``head_bce``)."""
        for l in self.layers:
            x = l(x)
        return head_bce(x, self.head.weight, self.head.bias, y)


# ---------------------------------------------------------------- sparse embedding
class DeviceDedup:
    """Sync-free de-duplication of a step's ids on the GPU (csrc/ctr.hip
    ``dedup_csr``): every output is sized by the CAPACITY n (the id count) and
    the number of unique ids stays on the device, so the exchange never copies
    a size to the host (``torch.unique`` / ``argsort`` / ``bincount`` do, and
    run rocprim merge sorts).  Workspaces are kept per n; the hash table
    cleans itself in each call."""

    def __init__(self, device):
        self.device = torch.device(device)
        self._ws = None   # ONE workspace, sized for the largest n seen (one per n leaked)
        self._ws_n = 0
        self._ar = {}

    def _buffers(self, n: int):
        """The workspace for n ids: views of the one held for the largest n so far
        (a bigger hash table serves a smaller n; it is left clean by every call)."""
        if self._ws is None or n > self._ws_n:
            ext = _ext.load()
            T = ext.dedup_table_slots(n)
            i32 = dict(dtype=torch.int32, device=self.device)
            i64 = dict(dtype=torch.int64, device=self.device)
            self._ws = dict(keys=torch.full((T,), -1, **i64), slot_of=torch.empty(n, **i32),
                            slot_uid=torch.empty(T, **i32), bsum=torch.empty(T // 1024 + (n + 1) // 1024 + 2, **i32),
                            sizes=torch.empty(n + 1, **i32), cursor=torch.empty(n + 1, **i32))
            self._ws_n = n
        ws = self._ws
        if n == self._ws_n:
            return ws
        return dict(keys=ws["keys"], slot_uid=ws["slot_uid"], bsum=ws["bsum"], slot_of=ws["slot_of"][:n],
                    sizes=ws["sizes"][: n + 1], cursor=ws["cursor"][: n + 1])

    def arange(self, n: int):
        """(order, seg) of n distinct segments of one row each (a push of the
        pull's already-unique ids)."""
        a = self._ar.get(n)
        if a is None:
            self._ar.clear()  # one size at a time (the batch's id count)
            a = self._ar[n] = (torch.arange(n, device=self.device), torch.arange(n + 1, device=self.device))
        return a

    def __call__(self, ids: torch.Tensor, csr: bool = True):
        """ids [n] int64 -> (uniq [n], inv [n], count [1] int32, seg [n+1], order [n])
        with uniq[:count] the distinct ids (padded with uniq[0]) and order/seg
        the positions of each unique id, ascending (valid when ``csr``)."""
        n = ids.numel()
        ws = self._buffers(n)
        uniq = torch.empty(n, dtype=torch.int64, device=self.device)
        inv = torch.empty(n, dtype=torch.int64, device=self.device)
        count = torch.empty(1, dtype=torch.int32, device=self.device)
        seg = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        order = torch.empty(n, dtype=torch.int64, device=self.device)
        _ext.load().dedup_csr(ids.contiguous(), ws["keys"], ws["slot_of"], ws["slot_uid"], ws["bsum"], ws["sizes"],
                              ws["cursor"], uniq, inv, count, seg, order, csr)
        return uniq, inv, count, seg, order


def _a2a(out_splits: List[int], in_splits: List[int], t: torch.Tensor, group) -> torch.Tensor:
    out = t.new_empty((sum(out_splits),) + tuple(t.shape[1:]))
    dist.all_to_all_single(out, t.contiguous(), out_splits, in_splits, group=group)
    return out


class ShardedEmbedding:
    """One logical [vocab, dim] fp32 table sharded by ``id % n_owners`` across
    the owner ranks of ``group``; Adagrad state lives next to each shard."""

    LAG = 2            # pulls between a fill's exchange and every rank reading it
    FILL_WINDOW = 8    # recent agreed fills the capacity is sized from

    def __init__(self, vocab: int, dim: int, owners: List[int], rank: int, world: int, device,
                 group=None, lr: float = 0.05, eps: float = 1e-8, init_std: float = 0.01, seed: int = 0,
                 max_ids: Optional[int] = None, slack: Optional[float] = None, force_fixed: bool = False,
                 rows_bf16: bool = False):
        self.vocab, self.dim = vocab, dim
        # the fixed exchange's row dtype: ONE value per embedding, the same on
        # every rank (the job config), so the row all-to-all's byte counts match
        # between a worker's pull_into / pull and a PS rank's participate()
        self.rows_bf16 = bool(rows_bf16)
        self.owners = list(owners)
        self.n_own = len(owners)
        self.rank, self.world = rank, world
        self.device = torch.device(device)
        self.group = group
        self.lr, self.eps = lr, eps
        self.is_owner = rank in self.owners
        self.me = self.owners.index(rank) if self.is_owner else -1
        rows = (vocab - self.me + self.n_own - 1) // self.n_own if self.is_owner else 0
        g = torch.Generator(device="cpu").manual_seed(seed + 7919 * max(self.me, 0))
        self.table = (torch.randn(rows, dim, generator=g) * init_std).to(self.device)
        self.accum = torch.zeros(rows, dim, device=self.device)
        self.use_hip = self.device.type == "cuda" and _ext.available()
        self._ctx = None
        # the sync-free path (DeviceDedup, capacity-sized buffers, device-side
        # counts) serves one-owner embeddings on the GPU
        self.dedup = DeviceDedup(self.device) if self.use_hip else None
        # Multi-rank exchange at a capacity every rank agrees on: each rank sends
        # every owner a slot block of ``cap`` ids (+ one header slot), so
        # all_to_all_single runs with equal splits and no per-step size exchange
        # to the host.  ``max_ids`` = the per-pull id bound every rank knows from
        # the job config (batch x fields).  By default cap = max_ids for the whole
        # run: exact, an overflow is impossible.  Adaptive capacity is opt-in
        # (``slack`` / KDL_TUNE ctr_a2a_slack > 0): the header carries the sender's
        # largest per-owner fill, so after the id exchange every rank holds the
        # same global max fill; LAG steps later (its pinned copy long landed)
        # every rank reads it and resizes ``cap`` by the same rule to slack x the
        # recent max fill.  A step whose fill exceeds its cap (the id distribution
        # shifted within LAG steps) would drop the excess ids to a dump slot --
        # their rows read as zeros and their gradients are lost for that step --
        # so an overflow RAISES (the rank exits non-zero) unless lossy mode is
        # asked for explicitly (KDL_TUNE ctr_a2a_strict=0: counted in
        # ``overflow_steps``, reported by ``finalize()``, capacity doubled).
        # ``force_fixed``: take this exchange at world 1 too (the one-GPU
        # rehearsal of the PS + worker path; RCCL all-to-alls on a 1-rank group).
        self.force_fixed = bool(force_fixed)
        self.max_ids = max_ids
        if max_ids is not None:
            from kubedl_amd.utils.tune import tune
            sl = slack if slack is not None else tune("ctr_a2a_slack", 0.0)
            self.slack = sl
            self.cap = max(int(max_ids), 1)
            self.strict = tune("ctr_a2a_strict", True)
            self._owner_rank = torch.tensor(self.owners, dtype=torch.int64, device=self.device)
            self._fills = collections.deque(maxlen=self.FILL_WINDOW)  # agreed max fills, oldest first
            self._pending = collections.deque()  # (cap used, pinned fill, event) per pull not yet read
            self.overflow_steps = 0
            self.exchange_bytes = 0  # bytes this rank sent in its fixed exchanges (ids + rows)

    # ------------------------------------------------------------ helpers
    def _local_gather(self, local_rows: torch.Tensor) -> torch.Tensor:
        if local_rows.numel() == 0:
            return self.table.new_empty(0, self.dim)
        if self.use_hip:
            out = self.table.new_empty(local_rows.numel(), self.dim)
            _ext.load().embed_gather(self.table, local_rows.contiguous(), 1, out, 0)
            return out
        return self.table[local_rows]

    def _apply_updates(self, ids_local: torch.Tensor, grads: torch.Tensor, scale: float,
                       distinct: bool = False) -> None:
        """Sum duplicate rows and apply Adagrad on the owned shard.  ``distinct``:
        the caller's ids are already unique (a world-1 push of the pull's
        de-duplicated ids) -- every segment is one row, no sort needed."""
        if not self.use_hip and not distinct:
            keep = ids_local >= 0  # exchange padding (negative sentinels)
            if not bool(keep.all()):
                ids_local, grads = ids_local[keep], grads[keep]
        n = ids_local.numel()
        if n == 0:
            return
        if distinct:
            uniq, inv = ids_local, torch.arange(n, device=self.device)
            order, seg = inv, torch.arange(n + 1, device=self.device)
        else:
            uniq, inv = torch.unique(ids_local, return_inverse=True)
            order = torch.argsort(inv, stable=True)
            counts = torch.bincount(inv, minlength=uniq.numel())
            seg = torch.zeros(uniq.numel() + 1, dtype=torch.int64, device=self.device)
            seg[1:] = torch.cumsum(counts, 0)
        if self.use_hip:
            _ext.load().segment_adagrad(grads.contiguous().float(), order, seg, uniq, self.table, self.accum,
                                        self.lr, self.eps, scale, None)
            return
        g = torch.zeros(uniq.numel(), self.dim, device=self.device).index_add_(0, inv, grads.float()) * scale
        a = self.accum[uniq] + g * g
        self.accum[uniq] = a
        self.table[uniq] -= self.lr * g / (a.sqrt() + self.eps)

    # ------------------------------------------------------------ pull / push
    # ------------------------------------------------------------ fixed-capacity exchange
    def _dedup_any(self, ids: torch.Tensor):
        """(uniq [n] padded, inv [n], count [1] int32) on the device (GPU kernel) or by
        torch.unique on the CPU, in the capacity format either way."""
        n = ids.numel()
        if self.dedup is not None and n > 0:
            uniq, inv, count, _, _ = self.dedup(ids, csr=False)
            return uniq, inv, count
        u, inv = torch.unique(ids, return_inverse=True)
        uniq = torch.zeros(n, dtype=torch.int64, device=ids.device)
        uniq[: u.numel()] = u
        if 0 < u.numel() < n:
            uniq[u.numel():] = u[0]
        return uniq, inv, torch.tensor([u.numel()], dtype=torch.int32, device=ids.device)

    def _agree(self, drain: bool = False) -> None:
        """Read the agreed fills of pulls at least LAG back (all of them with
        ``drain``) and resize ``cap`` -- a pure function of values every rank
        holds, evaluated at the same pull on every rank."""
        changed = False
        while self._pending and (drain or len(self._pending) > self.LAG):
            cap_used, host, evt = self._pending.popleft()
            if evt is not None:
                evt.synchronize()
            fill = int(host[0])
            self._fills.append(fill)
            if fill > cap_used:
                self.overflow_steps += 1
                if self.strict:
                    raise RuntimeError(f"CTR exchange overflow: {fill} ids for one owner > capacity {cap_used} "
                                       f"(ctr_a2a_slack={self.slack}); that step's excess rows were dropped. "
                                       f"Run with a larger slack, KDL_TUNE ctr_a2a_slack=0 (exact), or accept "
                                       f"lossy steps with KDL_TUNE ctr_a2a_strict=0")
            changed = True
        if not changed or self.slack <= 0 or drain:
            return
        need = min(self.max_ids, int(math.ceil(self.slack * max(self._fills))) + 64)
        need = min(self.max_ids, (need + 63) // 64 * 64)
        if self._fills[-1] > self.cap:  # overflowed at the current cap: grow at least 2x
            self.cap = min(self.max_ids, max(need, 2 * self.cap))
        elif need > self.cap or need < 0.75 * self.cap:
            self.cap = max(need, 1)

    def finalize(self) -> dict:
        """Read every outstanding agreed fill (syncs): call after the last step so
        an overflow in the final LAG pulls is counted (and raised if strict)."""
        if self._fixed():
            self._agree(drain=True)
            return {"exchange_cap": self.cap, "exchange_overflow_steps": self.overflow_steps,
                    "exchange_bytes": self.exchange_bytes}
        return {}

    def _pull_fixed(self, ids: torch.Tensor):
        """The fixed-capacity exchange of a pull -> (received rows [W * cap + 1, dim]
        (the last row zero), rslot [n], inverse [n]).  ``self.rows_bf16``: the rows
        travel as bf16 (the caller casts them to the bf16 tower input anyway:
        the owner rounds once, bit-identical, half the bytes) -- fixed at
        construction, so every rank of the exchange sends and receives one dtype."""
        rows_bf16 = self.rows_bf16
        self._agree()
        W, cap, dev = self.world, self.cap, self.device
        n = ids.numel()
        if n > self.max_ids:
            raise ValueError(f"pull of {n} ids > max_ids {self.max_ids}")
        # id blocks of cap + 1 slots per destination; slot cap = header (the
        # sender's largest per-owner fill, the same value to every destination)
        uniq, inv, count = self._dedup_any(ids)
        if self.use_hip:
            # csrc/ctr.hip a2a_route: a block-stable counting sort of the unique ids
            # by owner straight into the send blocks, padding and headers written by
            # the same launch; no one-hot [n, W + 1], no fill of the send buffer
            send = self._buf("send", (W * (cap + 1),), torch.int64)
            rslot = self._buf("rslot", (n,), torch.int64)
            _ext.load().a2a_route(uniq, count if n else None, self._owner_rank, W, cap, send, rslot)
        else:
            send = torch.full((W * (cap + 1) + 1,), -1, dtype=torch.int64, device=dev)
            if n:
                valid = torch.arange(n, device=dev) < count.to(torch.int64)
                dest = torch.where(valid, self._owner_rank[uniq % self.n_own], torch.full_like(uniq, W))
                onehot = torch.zeros(n, W + 1, dtype=torch.int64, device=dev).scatter_(1, dest[:, None], 1)
                pos = (torch.cumsum(onehot, 0) - onehot).gather(1, dest[:, None]).squeeze(1)
                ok = valid & (pos < cap)
                rslot = torch.where(ok, dest * cap + pos, torch.full_like(pos, W * cap))  # W * cap: dump slot
                send.scatter_(0, torch.where(ok, dest * (cap + 1) + pos, torch.full_like(pos, W * (cap + 1))), uniq)
                send[cap: W * (cap + 1): cap + 1] = onehot[:, :W].sum(0).max()
            else:
                rslot = torch.empty(0, dtype=torch.int64, device=dev)
                send[cap: W * (cap + 1): cap + 1] = 0
        recv = self._buf("recv", (W * (cap + 1),), torch.int64) if self.use_hip else \
            torch.empty(W * (cap + 1), dtype=torch.int64, device=dev)
        dist.all_to_all_single(recv, send[: W * (cap + 1)], group=self.group)  # equal splits: no size exchange
        rv = recv.view(W, cap + 1)
        req = rv[:, :cap].reshape(-1)       # ids asked of me, -1 = padding
        if self.slack > 0 or cap < self.max_ids:
            # adaptive capacity: the global max fill (identical on every rank) is
            # read LAG pulls later.  At the exact capacity (cap = max_ids >= n,
            # checked above) no block can overflow and nothing adapts: no fill
            # reduction, no device->host copy, no event to wait on
            fill = rv[:, cap].max().reshape(1)
            if dev.type == "cuda":
                host = torch.empty(1, dtype=torch.int64, pin_memory=True)
                host.copy_(fill, non_blocking=True)
                evt = torch.cuda.Event()
                evt.record()
            else:
                host, evt = fill.clone(), None
            self._pending.append((cap, host, evt))
        local, call = None, 0
        if self.is_owner and self.use_hip:
            # csrc/ctr.hip a2a_serve: requested rows (padding rows zero) + every
            # slot's local row for the push (padding -> distinct negative sentinels)
            # + the push's owner-update stamps (_owner_update)
            slotmap, call = self._stamp_call()
            rows, local = _ext.load().a2a_serve(self.table, req, self.n_own, rows_bf16, slotmap, call, cap, W)
        elif self.is_owner:
            lrow = torch.where(req >= 0, req // self.n_own, torch.zeros_like(req))
            ok = (req >= 0) & (lrow < self.table.shape[0])  # ids past the shard read as zero rows
            rows = self._local_gather(torch.where(ok, lrow, torch.zeros_like(lrow)))
            rows = torch.where(ok[:, None], rows, torch.zeros_like(rows))
            if rows_bf16:
                rows = rows.to(torch.bfloat16)
        elif self.use_hip:  # no id is routed to a non-owner: never read
            rows = torch.empty(W * cap, self.dim, device=dev, dtype=torch.bfloat16 if rows_bf16 else torch.float32)
        else:
            rows = torch.zeros(W * cap, self.dim, device=dev,
                               dtype=torch.bfloat16 if rows_bf16 else torch.float32)
        got = self._got_buffer(W * cap, rows.dtype)
        dist.all_to_all_single(got[: W * cap], rows.contiguous(), group=self.group)
        self.exchange_bytes += W * (cap + 1) * 8 + W * cap * self.dim * rows.element_size()
        self._ctx = ("fixed", rslot, req, count, cap, local, call)
        return got, rslot, inv

    def _buf(self, name: str, shape, dtype) -> torch.Tensor:
        """A per-step exchange buffer kept across steps (the HIP path: five fewer
        allocations per step; reuse is ordered -- every collective that reads or
        writes one is joined by the compute stream before the next step's writes)."""
        bufs = self.__dict__.setdefault("_bufs", {})
        b = bufs.get(name)
        if b is None or b.shape != torch.Size(shape) or b.dtype != dtype:
            b = bufs[name] = torch.empty(shape, dtype=dtype, device=self.device)
        return b

    def _got_buffer(self, rows: int, dtype) -> torch.Tensor:
        """[rows + 1, dim] receive buffer of the row exchange; row ``rows`` is the
        zero row every dump slot reads (kept zero: the exchange writes [:rows])."""
        g = getattr(self, "_got", None)
        if g is None or g.shape[0] != rows + 1 or g.dtype != dtype:
            g = self._got = torch.empty(rows + 1, self.dim, device=self.device, dtype=dtype)
            g[rows].zero_()
        return g

    def fixed_send_buffer(self, dump_row: bool = False) -> torch.Tensor:
        """[W * cap (+1), dim] gradient send buffer of the last fixed pull.  On the
        GPU rows no id was routed to stay unwritten: their slots are padding the
        owner never reads (no W * cap x dim zero fill).  ``dump_row``: one extra
        row past the exchange for ids that did not fit."""
        rows = self.world * self._ctx[4] + (1 if dump_row else 0)
        if self.use_hip:
            return self._buf("gsend", (rows, self.dim), torch.float32)
        return torch.zeros(rows, self.dim, device=self.device)

    def _push_fixed(self, grad_unique: torch.Tensor, scale: float) -> None:
        rslot = self._ctx[1]
        gsend = self.fixed_send_buffer(dump_row=True)
        if rslot.numel():
            gsend[rslot] = grad_unique.float()  # (the dump slot may take several rows: never sent)
        self.push_send(gsend, scale)

    def push_send(self, gsend: torch.Tensor, scale: float) -> None:
        """Exchange a filled gradient send buffer of the last fixed pull and apply
        the owner update."""
        _, _, req, _, cap, local, call = self._ctx
        W, dev = self.world, self.device
        grecv = self._buf("grecv", (W * cap, self.dim), torch.float32) if self.use_hip else \
            torch.empty(W * cap, self.dim, device=dev)
        dist.all_to_all_single(grecv, gsend[: W * cap], group=self.group)
        self.exchange_bytes += W * cap * self.dim * 4
        if self.is_owner:
            if local is None:
                # padding slots (id -1, zero gradient) become DISTINCT negative rows:
                # one-row segments that the update skips -- never one giant segment
                # (so do ids past the shard: served as zero rows, never updated)
                pad = -2 - torch.arange(req.numel(), device=dev)
                lrow = req // self.n_own
                local = torch.where((req >= 0) & (lrow < self.table.shape[0]), lrow, pad)
            if self.use_hip and self.dedup is not None:
                self._owner_update(local, grecv, cap, scale, call)
            else:
                self._apply_updates_dev(local, grecv, scale)

    def _stamp_call(self):
        """(slot map, call id) of the next owner update: the map is persistent
        (zeros), the id grows by one per pull (entries of earlier calls are stale).

        Memory: the map is int64 [owned rows x world] -- 8 W bytes per owned row
        for the whole run (W = 8: 64 B per row, the size of a D = 8 fp32 row
        plus its Adagrad state; the CTR config's D = 64 rows take 512 B).  It is
        checked against the device's free memory when first allocated."""
        if getattr(self, "_slotmap", None) is None or self._calls >= (1 << 31) - 1:
            need = self.table.shape[0] * self.world * 8
            if self.device.type == "cuda":
                free, _total = torch.cuda.mem_get_info(self.device)
                if need > free // 2:
                    raise MemoryError(f"CTR owner-update slot map needs {need / 2**30:.2f} GiB "
                                      f"({self.table.shape[0]} owned rows x {self.world} ranks x 8 B), more than "
                                      f"half of the {free / 2**30:.2f} GiB free: shard the table over more owners")
            self._slotmap = torch.zeros(self.table.shape[0] * self.world, dtype=torch.int64, device=self.device)
            self._calls = 0
        self._calls += 1
        return self._slotmap, self._calls

    def _owner_update(self, local: torch.Tensor, grecv: torch.Tensor, cap: int, scale: float, call: int = 0) -> None:
        """Owner update without a de-duplication pass (csrc/ctr.hip a2a_owner_update):
        each sender routes a row once, so duplicates are only across senders --
        a per-row, per-sender slot stamp (no atomics; written by the pull's
        a2a_serve when ``call`` is its id) replaces the hash dedup + CSR sort of
        the W * cap received slots; each row's lowest sender sums the row in slot
        order (bitwise the segment_adagrad result)."""
        stamped = call > 0
        if not stamped:
            _, call = self._stamp_call()
        _ext.load().a2a_owner_update(grecv, local, cap, self.world, self._slotmap, call, self.table, self.accum,
                                     self.lr, self.eps, scale, stamped)

    def _apply_updates_dev(self, ids_local: torch.Tensor, grads: torch.Tensor, scale: float) -> None:
        """Owner update with the duplicate-sum on the device (no size to the host):
        DeviceDedup's CSR gives each row's contributions in position order."""
        if self.dedup is None:
            self._apply_updates(ids_local, grads, scale)
            return
        uniq, inv, count, seg, order = self.dedup(ids_local, csr=True)
        _ext.load().segment_adagrad(grads.contiguous().float(), order, seg, uniq, self.table, self.accum,
                                    self.lr, self.eps, scale, count)

    def _sync_free(self, ids: torch.Tensor) -> bool:
        return (self.dedup is not None and ids.numel() > 0 and self.n_own == 1 and not self.force_fixed and
                (self.world == 1 or self.group is None and not dist.is_initialized()))

    def pull_into(self, ids: torch.Tensor, out: torch.Tensor, F: int, col0: int = 0,
                  dense: Optional[torch.Tensor] = None, tail: int = 0) -> Optional[torch.Tensor]:
        """One-owner sync-free pull written straight into the bf16 tower input:
        ``out[b, col0 + f*D : +D] = table[ids[b*F + f]]`` (csrc/ctr.hip
        ``embed_gather_cast``: no fp32 [n, D] gather, no cast pass).  ``tail``:
        the same launch writes the ``tail`` columns after the last field --
        ``dense`` (fp32 [B, nd]) cast to bf16, then zeros.  Returns the inverse
        map, or None when this path does not apply (then use ``pull``)."""
        if not (out.dtype == torch.bfloat16 and self.table.dtype == torch.float32 and self.use_hip
                and self.dim % 8 == 0 and out.stride(0) % 8 == 0 and col0 % 8 == 0 and ids.numel() > 0):
            return None
        if self._fixed():
            # fixed exchange: the received rows go straight into the bf16 input
            # through rslot (dump slots read the zero row)
            got, rslot, inv = self._pull_fixed(ids)
            _ext.load().embed_gather_cast(got, rslot, inv, F, out, col0, dense, tail)
            return inv
        if not self._sync_free(ids):
            return None
        uniq, inv, count, _, _ = self.dedup(ids, csr=False)
        _ext.load().embed_gather_cast(self.table, uniq, inv, F, out, col0, dense, tail)
        self._ctx = ("dev", uniq, count)
        return inv

    def _fixed(self) -> bool:
        return self.max_ids is not None and (self.world > 1 or self.force_fixed)

    def pull(self, ids: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """ids [n] int64 (any, may repeat) -> (unique rows [U, dim], inverse [n]).
        On the sync-free path U is the capacity n: rows past the live count are
        gathered from a valid id and never referenced by ``inverse``."""
        if self._sync_free(ids):
            uniq, inv, count, _, _ = self.dedup(ids, csr=False)
            emb = self._local_gather(uniq)
            self._ctx = ("dev", uniq, count)
            return emb, inv
        if self._fixed():
            got, rslot, inv = self._pull_fixed(ids)
            return (got[rslot] if ids.numel() else got[:0]), inv
        uniq, inv = torch.unique(ids, return_inverse=True)
        owner = uniq % self.n_own
        order = torch.argsort(owner, stable=True)
        uniq_sorted = uniq[order]
        send_counts = torch.bincount(owner, minlength=self.n_own)
        if self.world == 1 or self.group is None and not dist.is_initialized():
            rows = self._local_gather(uniq_sorted // self.n_own)
            emb = torch.empty_like(rows)
            emb[order] = rows
            self._ctx = (uniq_sorted, order, None, None)
            return emb, inv
        # counts per destination RANK (owners are a subset of ranks)
        full_send = torch.zeros(self.world, dtype=torch.int64, device=self.device)
        full_send[torch.tensor(self.owners, device=self.device)] = send_counts
        full_recv = torch.empty_like(full_send)
        dist.all_to_all_single(full_recv, full_send, group=self.group)
        send_l, recv_l = full_send.tolist(), full_recv.tolist()
        req = _a2a(recv_l, send_l, uniq_sorted, self.group)           # ids asked of me
        rows = self._local_gather(req // self.n_own) if self.is_owner else self.table.new_empty(0, self.dim)
        got = _a2a(send_l, recv_l, rows, self.group)                    # rows for my ids
        emb = torch.empty_like(got)
        emb[order] = got
        self._ctx = (uniq_sorted, order, send_l, recv_l, req)
        return emb, inv

    def push(self, grad_unique: torch.Tensor, scale: float = 1.0) -> None:
        """grad rows aligned with the unique ids of the last pull."""
        ctx = self._ctx
        kind = ctx[0] if isinstance(ctx[0], str) else None
        if kind == "fixed":
            self._push_fixed(grad_unique, scale)
            return
        if kind == "dev":  # one row per unique id, count on the device
            _, uniq, count = ctx
            order, seg = self.dedup.arange(uniq.numel())
            _ext.load().segment_adagrad(grad_unique.contiguous().float(), order, seg, uniq, self.table, self.accum,
                                        self.lr, self.eps, scale, count)
            return
        uniq_sorted, order = ctx[0], ctx[1]
        g_sorted = grad_unique[order]
        if ctx[2] is None:
            self._apply_updates(uniq_sorted // self.n_own, g_sorted, scale, distinct=True)
            return
        send_l, recv_l, req = ctx[2], ctx[3], ctx[4]
        g_recv = _a2a(recv_l, send_l, g_sorted.float(), self.group)
        if self.is_owner:
            self._apply_updates(req // self.n_own, g_recv, scale)

    def push_rows(self, rows: torch.Tensor, F: int, col0: int, order: torch.Tensor, seg: torch.Tensor,
                  scale: float = 1.0) -> bool:
        """Sync-free one-owner push straight from the activation-gradient rows
        (row j = b*F + f at ``rows[b, col0 + f*dim:]``): each unique id's rows
        order[seg[u]:seg[u+1]] are summed and applied by Adagrad in one launch
        (csrc/ctr.hip ``segment_reduce_adagrad``: bitwise ``segment_reduce`` +
        ``push``, without the [U, dim] fp32 sums between them).  Returns False
        when the last pull was not the sync-free kind (then use ``push``)."""
        ctx = self._ctx
        if ctx is None or not isinstance(ctx[0], str) or ctx[0] != "dev" or not self.use_hip:
            return False
        _, uniq, count = ctx
        _ext.load().segment_reduce_adagrad(rows, F, col0, self.dim, order, seg, count, uniq, self.table, self.accum,
                                           self.lr, self.eps, scale)
        return True

    def participate(self, scale: float = 1.0) -> None:
        """An owner without a batch of its own (PS rank) serves one pull+push round.
        ``scale``: the gradient scale the workers push with (the owner applies
        it to every received row), e.g. 1 / n_workers -- the same value on
        every rank of the job."""
        empty = torch.empty(0, dtype=torch.int64, device=self.device)
        self.pull(empty)
        self.push(torch.empty(0, self.dim, device=self.device), scale)


# ---------------------------------------------------------------- model
class CTRModel:
    """Embeddings (F fields x dim) + dense features -> MLP tower -> logit."""

    def __init__(self, n_fields: int, vocab_per_field: int, dim: int, n_dense: int, hidden, emb: ShardedEmbedding,
                 device, dtype=torch.bfloat16):
        self.F, self.V, self.D, self.nd = n_fields, vocab_per_field, dim, n_dense
        self.k_in = n_fields * dim + n_dense
        # padded to 64 columns: every tower layer's weight gradient then fits the
        # MFMA weight-gradient kernel's 64-wide tiles (no hipBLASLt in the step)
        self.k_pad = (self.k_in + 63) // 64 * 64
        self.emb = emb
        self.device = torch.device(device)
        self.dtype = dtype
        self.tower = DenseTower(self.k_pad, hidden).to(self.device)
        with torch.no_grad():
            for p in self.tower.parameters():
                p.data = p.data.to(dtype)
        self.field_off = (torch.arange(n_fields, device=self.device) * vocab_per_field)[None, :]

    def _csr_of(self, inv: torch.Tensor, count: torch.Tensor):
        # positions ascending per unique id: the argsort path's summation order;
        # live count on the device
        dd = self.emb.dedup
        n = inv.numel()
        ws = dd._buffers(n)
        seg = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        order = torch.empty(n, dtype=torch.int64, device=self.device)
        _ext.load().csr_from_inverse_only(inv, ws["sizes"], count, ws["bsum"], ws["cursor"], seg, order)
        return seg, order

    def build_input(self, ids: torch.Tensor, dense: torch.Tensor):
        B = ids.shape[0]
        gids = (ids + self.field_off).reshape(-1)
        x = torch.empty(B, self.k_pad, dtype=self.dtype, device=self.device)
        tail = self.k_pad - self.F * self.D
        fuse_tail = (dense.dtype == torch.float32 and dense.is_contiguous() and dense.dim() == 2
                     and dense.shape[1] == self.nd and tail % 8 == 0)
        # fused one-owner pull: table rows -> bf16 input directly; with the dense
        # features and the zero pad written by the same launch
        inv = self.emb.pull_into(gids, x, self.F, 0, dense if fuse_tail else None,
                                 tail if fuse_tail else 0) if self.device.type == "cuda" else None
        if inv is not None and fuse_tail:
            return x, inv, gids.numel()
        # every column is written below except the pad [k_in, k_pad): zero only that
        if self.k_pad > self.k_in:
            x[:, self.k_in:].zero_()
        if inv is not None:
            U = gids.numel()
        else:
            emb_u, inv = self.emb.pull(gids)
            U = emb_u.shape[0]
            emb_u_c = emb_u.to(self.dtype).contiguous()
            if self.device.type == "cuda" and _ext.available():
                _ext.load().embed_gather(emb_u_c, inv.contiguous(), self.F, x, 0)
            else:
                x[:, : self.F * self.D] = emb_u_c[inv].reshape(B, self.F * self.D)
        x[:, self.F * self.D: self.k_in].copy_(dense)  # cast + strided write in one launch
        return x, inv, U

    def push_grads(self, xgrad: torch.Tensor, inv: torch.Tensor, U: int, scale: float) -> None:
        B = xgrad.shape[0]
        ctx = self.emb._ctx
        kind = ctx[0] if ctx is not None and isinstance(ctx[0], str) else None
        count = ctx[2] if kind == "dev" else ctx[3] if kind == "fixed" else None
        if kind is not None and self.emb.dedup is not None and inv.numel() > 0:
            seg, order = self._csr_of(inv, count)
            if kind == "fixed":
                # each unique id's summed gradient row lands in its exchange slot
                # (rslot) of the send buffer: no [U, D] intermediate, no scatter
                gsend = self.emb.fixed_send_buffer()
                _ext.load().segment_reduce(xgrad, self.F, 0, self.D, order, seg, count, ctx[1], gsend)
                self.emb.push_send(gsend, scale)
                return
            if kind == "dev" and self.emb.push_rows(xgrad, self.F, 0, order, seg, scale):
                return
            g_u = _ext.load().segment_reduce(xgrad, self.F, 0, self.D, order, seg, count)
            self.emb.push(g_u, scale)
            return
        order = torch.argsort(inv, stable=True)
        counts = torch.bincount(inv, minlength=U)
        seg = torch.zeros(U + 1, dtype=torch.int64, device=self.device)
        seg[1:] = torch.cumsum(counts, 0)
        if self.device.type == "cuda" and _ext.available():
            g_u = _ext.load().segment_reduce(xgrad, self.F, 0, self.D, order, seg, None)
        else:
            rows = xgrad[:, : self.F * self.D].reshape(B * self.F, self.D).float()
            g_u = torch.zeros(U, self.D, device=self.device).index_add_(0, inv, rows)
        self.emb.push(g_u, scale)
