"""Distributed histogram gradient-boosted trees (the XGBoostJob data plane).

XGBoost's ``hist`` algorithm, depth-wise, re-designed for one GPU per rank:

* features quantised once to <= 256 bins (uint8 [N, F]) with quantile cuts
  agreed on by all ranks (samples all-gathered, every rank computes the same
  cuts -- the role of XGBoost's distributed sketch);
* per level: gradient/hessian histograms of every active node built by the
  ``gbdt_hist`` HIP kernel (LDS atomics, lane = feature), ALL-REDUCED across
  ranks (RCCL over xGMI; the rabit tree-allreduce of the reference's image),
  best split per (node, feature) by the ``gbdt_split`` kernel (block scan over
  bins + XGBoost gain), rows routed by ``gbdt_route`` and regrouped by a
  stable sort on child id;
* histogram subtraction: below the root only the smaller child of each split
  is built; its sibling is ``parent - child`` (halves the histogram work);
* objectives ``reg:squarederror``, ``binary:logistic``, ``multi:softprob``
  (one tree per class per round, as XGBoost).

On the GPU a tree never leaves the device while it grows: the native
``GbdtGrower`` (csrc/gbdt_grower.cpp over csrc/gbdt.hip) keeps nodes in heap
order, rows grouped per node by a stable in-segment partition, and the split
decisions, child segments and smaller-child choice in device arrays; the host
only enqueues a fixed kernel sequence per level (plus the two all-reduces per
level with several ranks).  The trees' heap arrays are copied to the host once,
at the end of ``fit``.  Quantisation is one kernel (``gbdt_quantise``).

Every rank holds a row shard; all ranks grow identical trees because they
see identical all-reduced histograms.  On CPU (or without the extension)
the same algorithm runs on torch ops -- that path is the numerics reference
for the kernels in tests.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.distributed as dist

from kubedl_amd.ops import _ext


@dataclass
class GBDTParams:
    objective: str = "reg:squarederror"
    num_class: int = 1
    n_estimators: int = 10
    learning_rate: float = 0.3
    max_depth: int = 6
    max_bin: int = 256
    reg_lambda: float = 1.0
    gamma: float = 0.0
    min_child_weight: float = 1.0
    base_score: float = 0.5

    @classmethod
    def parse(cls, spec: str, **kw) -> "GBDTParams":
        """``objective:multi:softprob,num_class:3`` (the example's --xgboost_parameter)."""
        p = cls(**kw)
        if not spec:
            return p
        spec = spec.strip().strip('"')
        for part in spec.split(","):
            if ":" not in part:
                continue
            k, v = part.split(":", 1)
            k = k.strip()
            alias = {"eta": "learning_rate", "lambda": "reg_lambda", "num_round": "n_estimators",
                     "min_split_loss": "gamma"}
            k = alias.get(k, k)
            if not hasattr(p, k):
                continue
            cur = getattr(p, k)
            setattr(p, k, type(cur)(v) if not isinstance(cur, str) else v)
        return p


@dataclass
class Tree:
    feature: List[int] = field(default_factory=list)
    split_bin: List[int] = field(default_factory=list)
    threshold: List[float] = field(default_factory=list)
    left: List[int] = field(default_factory=list)
    right: List[int] = field(default_factory=list)
    value: List[float] = field(default_factory=list)

    def add(self) -> int:
        for a in (self.feature, self.split_bin, self.left, self.right):
            a.append(-1)
        self.threshold.append(0.0)
        self.value.append(0.0)
        return len(self.value) - 1


def _world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _allreduce_(t: torch.Tensor) -> torch.Tensor:
    if _world() > 1:
        dist.all_reduce(t)
    return t


class HistGBDT:
    def __init__(self, params: GBDTParams, device=None):
        self.p = params
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.cuts: Optional[torch.Tensor] = None  # [F, B-1]
        self.trees: List[List[Tree]] = []
        self.use_hip = self.device.type == "cuda"
        if self.use_hip and not _ext.available():
            _ext.require_on_gpu("HistGBDT")
            self.use_hip = False
        self.stats = {"hist_builds": 0, "hist_subtracted": 0}

    # ------------------------------------------------------------ quantisation
    def fit_cuts(self, X: torch.Tensor, sample: int = 65536, seed: int = 0) -> None:
        B = self.p.max_bin
        n = X.shape[0]
        # a systematic sample (every n/sample-th row from a seeded offset): the
        # same rows on every device, no host permutation of n ids (torch.randperm
        # of 2M ids was ~0.15 s of the fit's set-up on the CPU)
        k = min(sample, n)
        off = (seed * 7919 + 17) % max(n // k, 1)
        idx = (torch.arange(k, device=X.device, dtype=torch.int64) * n) // k + off
        samp = X[idx.clamp_(max=n - 1)].float()
        if _world() > 1:
            # every rank contributes the same number of rows
            k = torch.tensor([samp.shape[0]], device=X.device)
            dist.all_reduce(k, op=dist.ReduceOp.MIN)
            samp = samp[: int(k.item())].contiguous()
            parts = [torch.empty_like(samp) for _ in range(_world())]
            dist.all_gather(parts, samp)
            samp = torch.cat(parts)
        # torch.quantile's 'linear' rule as a sort + lerp: the same cuts (to fp32
        # rounding), but torch.quantile's first call on a GPU costs ~0.18 s of
        # kernel loading where one sort costs ~8 ms (scripts/quantile_probe.py)
        q = torch.linspace(0, 1, B + 1, device=samp.device, dtype=torch.float64)[1:-1]
        srt, _ = torch.sort(samp.T.contiguous(), dim=1)  # [F, m]
        pos = q * (srt.shape[1] - 1)
        lo, hi = pos.floor().long(), pos.ceil().long()
        w = (pos - lo.double()).float()
        self.cuts = (srt[:, lo] * (1 - w) + srt[:, hi] * w).contiguous()  # [F, B-1]

    def host_cuts(self, X: torch.Tensor, sample: int = 65536, seed: int = 0) -> torch.Tensor:
        """``fit_cuts`` on a host copy of X, bitwise the same cuts: the same
        systematic sample, the same order statistics (``numpy.partition`` puts each
        needed rank exactly where a full sort would), the same float32 lerp.  On a
        fresh GPU process the device version's first calls load torch's sort and
        elementwise code objects (0.1-0.6 s, ``scripts/cuts_probe.py``); this one
        loads nothing and runs beside the host->device copy (``fit``)."""
        import numpy as np
        B = self.p.max_bin
        n = X.shape[0]
        k = min(sample, n)
        off = (seed * 7919 + 17) % max(n // k, 1)
        idx = np.minimum((np.arange(k, dtype=np.int64) * n) // k + off, n - 1)
        samp = np.ascontiguousarray(X.detach().numpy()[idx].astype(np.float32, copy=False))  # [k, F]
        q = torch.linspace(0, 1, B + 1, dtype=torch.float64)[1:-1]
        pos = q * (k - 1)
        lo, hi = pos.floor().long(), pos.ceil().long()
        w = (pos - lo.double()).float()
        kth = np.unique(np.concatenate([lo.numpy(), hi.numpy()]))
        part = np.partition(samp, kth, axis=0)
        a = torch.from_numpy(np.ascontiguousarray(part[lo.numpy()].T))  # [F, B-1]
        b = torch.from_numpy(np.ascontiguousarray(part[hi.numpy()].T))
        return (a * (1 - w) + b * w).contiguous()

    def quantise(self, X: torch.Tensor) -> torch.Tensor:
        if self.use_hip and X.is_cuda:
            return _ext.load().gbdt_quantise(X, self.cuts, self.p.max_bin)
        F = X.shape[1]
        out = torch.empty(X.shape, dtype=torch.uint8, device=X.device)
        for f in range(F):
            out[:, f] = torch.bucketize(X[:, f].contiguous().float(), self.cuts[f].contiguous(), right=False).clamp_(
                max=self.p.max_bin - 1).to(torch.uint8)
        return out

    # ------------------------------------------------------------ objectives
    def _grad_hess(self, pred: torch.Tensor, y: torch.Tensor):
        obj = self.p.objective
        if self.use_hip and pred.is_cuda:
            # csrc/gbdt.hip grad_hess_kernel: one launch, the torch composition's expressions
            code = 0 if obj.startswith("reg:") else 1 if obj == "binary:logistic" else 2 if obj.startswith("multi:") else -1
            if code >= 0:
                c = getattr(self, "_yf", None)
                if c is None or c[0] is not y:  # the labels as fp32, converted once per fit
                    c = self._yf = (y, y if (y.dtype == torch.float32 and y.is_contiguous()) else y.float().contiguous())
                g, h = _ext.load().gbdt_grad_hess(pred.contiguous(), c[1].view(-1), code)
                return g, h
        if obj.startswith("reg:"):
            return pred - y.view_as(pred), torch.ones_like(pred)
        if obj == "binary:logistic":
            pr = torch.sigmoid(pred)
            return pr - y.view_as(pred), (pr * (1 - pr)).clamp_min(1e-16)
        if obj.startswith("multi:"):
            pr = torch.softmax(pred, dim=1)
            yy = torch.nn.functional.one_hot(y.long(), self.p.num_class).to(pr.dtype)
            return pr - yy, (2.0 * pr * (1 - pr)).clamp_min(1e-16)
        raise ValueError(f"unsupported objective {obj}")

    def _base(self, n: int) -> torch.Tensor:
        K = self.p.num_class if self.p.objective.startswith("multi:") else 1
        if self.p.objective == "binary:logistic":
            b = math.log(self.p.base_score / (1 - self.p.base_score))
        elif self.p.objective.startswith("multi:"):
            b = 0.0
        else:
            b = self.p.base_score
        return torch.full((n, K), b, dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------ kernels (HIP or torch)
    def _hist(self, bins, g, h, rows, seg_cpu, F, B):
        nodes = len(seg_cpu) - 1
        hist = torch.zeros(nodes, F, B, 2, dtype=torch.float32, device=self.device)
        if nodes == 0:
            return hist
        self.stats["hist_builds"] += nodes
        if self.use_hip:
            seg = torch.tensor(seg_cpu, dtype=torch.int32, device=self.device)
            maxr = max(seg_cpu[i + 1] - seg_cpu[i] for i in range(nodes))
            _ext.load().gbdt_hist(bins, g, h, 1, rows, seg, int(maxr), B, hist)
            return hist
        counts = torch.tensor([seg_cpu[i + 1] - seg_cpu[i] for i in range(nodes)], device=self.device)
        node_of = torch.repeat_interleave(torch.arange(nodes, device=self.device), counts)
        rb = bins[rows.long()].long()  # [n, F]
        base = (node_of[:, None] * F + torch.arange(F, device=self.device)[None, :]) * B + rb
        flat = hist.view(-1, 2)
        flat[:, 0].index_add_(0, base.reshape(-1), g[rows.long()].repeat_interleave(F))
        flat[:, 1].index_add_(0, base.reshape(-1), h[rows.long()].repeat_interleave(F))
        return hist

    def _split(self, hist):
        lam, mcw = self.p.reg_lambda, self.p.min_child_weight
        if self.use_hip:
            return _ext.load().gbdt_split(hist.contiguous(), lam, mcw)
        G = hist[..., 0].cumsum(-1)
        H = hist[..., 1].cumsum(-1)
        tg, th = G[..., -1:], H[..., -1:]
        gr, hr = tg - G, th - H
        gain = G * G / (H + lam) + gr * gr / (hr + lam) - tg * tg / (th + lam)
        ok = (H >= mcw) & (hr >= mcw)
        ok[..., -1] = False
        gain = torch.where(ok, gain, torch.full_like(gain, -math.inf))
        best, bin_ = gain.max(-1)
        gl = G.gather(-1, bin_[..., None])[..., 0]
        hl = H.gather(-1, bin_[..., None])[..., 0]
        bin_ = torch.where(torch.isinf(best), torch.full_like(bin_, -1), bin_)
        return best, bin_.int(), gl, hl

    def _route(self, bins, rows, row_node, sfeat, sbin):
        if self.use_hip:
            return _ext.load().gbdt_route(bins, rows, row_node, sfeat, sbin)
        f = sfeat[row_node.long()].long()
        b = bins[rows.long(), f.clamp_min(0)].int()
        return ((f >= 0) & (b > sbin[row_node.long()])).int()

    # ------------------------------------------------------------ one tree
    def _grow(self, bins, g, h, n_local: int) -> (Tree, torch.Tensor):
        """Depth-wise growth.  Per level the host does O(1) device syncs (one
        batched read of the split decisions, one of the child counts): every
        per-node quantity is gathered/scattered with one tensor op per level,
        and each row's node id is carried through the stable sort instead of
        being re-expanded from the segment counts."""
        p = self.p
        F, B = bins.shape[1], p.max_bin
        dev = self.device
        tree = Tree()
        root = tree.add()
        rows = torch.arange(n_local, dtype=torch.int32, device=dev)
        row_node = torch.zeros(n_local, dtype=torch.int32, device=dev)  # level-local node of each row in ``rows``
        seg = [0, n_local]
        level_nodes = [root]
        leaf_of_row = torch.zeros(n_local, dtype=torch.int32, device=dev)
        hist = _allreduce_(self._hist(bins, g, h, rows, seg, F, B))
        ncut = self.cuts.shape[1]
        for depth in range(p.max_depth + 1):
            nodes = len(level_nodes)
            tot = hist[:, 0].sum(1)  # [nodes, 2] (every feature sums to the node total)
            weight = -tot[:, 0] / (tot[:, 1] + p.reg_lambda) * p.learning_rate
            if depth < p.max_depth:
                gain, sbin, gl, hl = self._split(hist)
                best_gain, best_f = gain.max(1)
                do_split = (best_gain > p.gamma) & torch.isfinite(best_gain)
                best_b = sbin.gather(1, best_f[:, None])[:, 0].long()
                thr = self.cuts[best_f, best_b.clamp(0, ncut - 1)]
                thr = torch.where(best_b < ncut, thr, torch.full_like(thr, math.inf))
                # one device->host transfer for every per-node decision of this level
                host = torch.stack([do_split.double(), weight.double(), best_f.double(), best_b.double(),
                                    thr.double()]).tolist()
                ds, weights, bf, bb, th = host[0], host[1], [int(v) for v in host[2]], [int(v) for v in host[3]], \
                    host[4]
                ds = [v > 0.5 for v in ds]
            else:
                ds, weights = [False] * nodes, weight.tolist()
            # leaves of this level: every row of a non-split node ends here
            leaf_id = [-1 if ds[i] else level_nodes[i] for i in range(nodes)]
            if any(v >= 0 for v in leaf_id):
                lid = torch.tensor(leaf_id, dtype=torch.int32, device=dev)[row_node.long()]
                m = lid >= 0
                leaf_of_row[rows[m].long()] = lid[m]
            for i, nid in enumerate(level_nodes):
                if not ds[i]:
                    tree.value[nid] = weights[i]
            if not any(ds):
                break
            sfeat = torch.tensor([bf[i] if ds[i] else -1 for i in range(nodes)], dtype=torch.int32, device=dev)
            sb = torch.tensor([bb[i] if ds[i] else -1 for i in range(nodes)], dtype=torch.int32, device=dev)
            go_right = self._route(bins, rows, row_node, sfeat, sb)
            next_nodes, remap = [], []
            for i, nid in enumerate(level_nodes):
                if ds[i]:
                    l, r = tree.add(), tree.add()
                    tree.feature[nid], tree.split_bin[nid] = bf[i], bb[i]
                    tree.threshold[nid] = th[i]
                    tree.left[nid], tree.right[nid] = l, r
                    remap.append((len(next_nodes), len(next_nodes) + 1))
                    next_nodes += [l, r]
                else:
                    remap.append((-1, -1))
            # new child index per row (-1 = leaf reached); the stable sort keeps rows grouped by child
            child = torch.tensor(remap, dtype=torch.int32, device=dev)[row_node.long(), go_right.long()]
            keep = child >= 0
            child, rows_k = child[keep], rows[keep]
            child, order = torch.sort(child, stable=True)
            rows = rows_k[order].contiguous()
            row_node = child.contiguous()
            ccount = torch.bincount(child, minlength=len(next_nodes))
            # histogram subtraction: build the smaller child (by global count), derive the sibling
            glob = _allreduce_(ccount.clone().float())
            cc = torch.stack([torch.cumsum(ccount, 0).double(), glob.double()]).tolist()
            seg = [0] + [int(v) for v in cc[0]]
            gl_ = cc[1]
            small = [2 * j + (0 if gl_[2 * j] <= gl_[2 * j + 1] else 1) for j in range(len(next_nodes) // 2)]
            sub_seg = [0]
            sub_rows = []
            for c in small:
                sub_rows.append(rows[seg[c]:seg[c + 1]])
                sub_seg.append(sub_seg[-1] + seg[c + 1] - seg[c])
            srows = torch.cat(sub_rows) if sub_rows else rows[:0]
            h_small = _allreduce_(self._hist(bins, g, h, srows.contiguous(), sub_seg, F, B))
            parents = torch.tensor([i for i in range(nodes) if ds[i]], dtype=torch.long, device=dev)
            small_t = torch.tensor(small, dtype=torch.long, device=dev)
            parent_hist = hist
            hist = torch.empty(len(next_nodes), F, B, 2, dtype=torch.float32, device=dev)
            hist[small_t] = h_small
            hist[small_t ^ 1] = parent_hist[parents] - h_small
            self.stats["hist_subtracted"] += len(small)
            level_nodes = next_nodes
        return tree, leaf_of_row

    # ------------------------------------------------------------ device-resident tree
    def _device_grower(self, bins):
        p = self.p
        if not self.use_hip or p.max_depth > 10 or (bins.shape[1] * p.max_bin) % 2:
            return None
        return _ext.load().GbdtGrower(bins, self.cuts, p.max_bin, p.max_depth, p.reg_lambda, p.gamma,
                                      p.learning_rate, p.min_child_weight)

    def _grow_device(self, gr, g, h):
        """One tree on the GPU; returns its [4, heap] arrays (feature, split bin,
        threshold, value)."""
        D = self.p.max_depth
        if _world() == 1:
            gr.grow_local(g, h)
        else:
            _allreduce_(gr.begin_tree(g, h))
            for d in range(D + 1):
                cnt = gr.level_a(d, False)
                if d < D:
                    _allreduce_(cnt)                    # global child counts -> same smaller child on all ranks
                    _allreduce_(gr.level_b(d, True))    # the built children's histograms
                    gr.level_c(d)
        return gr.heap_packed()  # [4, heap] in one launch (the leaf values go in by add_leaf)

    @staticmethod
    def _heap_tree(arr) -> Tree:
        feat, tbin, thr, val = arr
        t = Tree()
        t.feature = [int(v) for v in feat]
        t.split_bin = [int(v) for v in tbin]
        t.threshold = [float(v) for v in thr]
        t.value = [float(v) for v in val]
        t.left = [2 * i + 1 if f >= 0 else -1 for i, f in enumerate(t.feature)]
        t.right = [2 * i + 2 if f >= 0 else -1 for i, f in enumerate(t.feature)]
        return t

    # ------------------------------------------------------------ training
    def _sync_time(self) -> float:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return time.perf_counter()

    def fit(self, X: torch.Tensor, y: torch.Tensor, log_every: int = 0, callback=None):
        """``stats['setup_s']``: host->device copy, cut fitting, quantisation and the
        grower's workspaces; ``stats['boost_s']``: the boosting rounds alone (one
        synchronisation at each end, none inside)."""
        t0 = self._sync_time()
        host_cuts = {}
        th = None
        if (self.cuts is None and X.device.type == "cpu" and self.device.type == "cuda" and _world() == 1
                and X.dim() == 2 and X.dtype in (torch.float32, torch.float64)):
            # the cuts from the host copy, beside the host->device copy (numpy and
            # the copy release the GIL)
            import threading

            def run():
                try:
                    host_cuts["c"] = self.host_cuts(X)
                except BaseException as e:  # re-raised below
                    host_cuts["e"] = e
            th = threading.Thread(target=run, name="gbdt-cuts", daemon=True)
            th.start()
        X = X.to(self.device)
        y = y.to(self.device)
        ta = self._sync_time()
        if th is not None:
            th.join()
            if "e" in host_cuts:
                raise host_cuts["e"]
            self.cuts = host_cuts["c"].to(self.device)
        elif self.cuts is None:
            self.fit_cuts(X)
        if self.cuts.device != self.device:  # cuts fitted on a host copy (fit_cuts on a CPU X)
            self.cuts = self.cuts.to(self.device)
        tb = self._sync_time()
        bins = self.quantise(X).contiguous()
        n = X.shape[0]
        pred = self._base(n)
        K = pred.shape[1]
        tc = self._sync_time()
        grower = self._device_grower(bins)
        t1 = self._sync_time()
        for k, v in (("setup_h2d_s", ta - t0), ("setup_cuts_s", tb - ta), ("setup_quantise_s", tc - tb),
                     ("setup_grower_s", t1 - tc)):
            self.stats[k] = self.stats.get(k, 0.0) + v
        dev_trees = []
        for it in range(self.p.n_estimators):
            g_all, h_all = self._grad_hess(pred, y)
            round_trees = []
            for k in range(K):
                g = g_all[:, k].contiguous()
                h = h_all[:, k].contiguous()
                if grower is not None:
                    round_trees.append(self._grow_device(grower, g, h))
                    grower.add_leaf(pred, k)  # pred[:, k] += the rows' leaf values, one launch
                    continue
                tree, leaf = self._grow(bins, g, h, n)
                vals = torch.tensor(tree.value, dtype=torch.float32, device=self.device)
                pred[:, k] += vals[leaf.long()]
                round_trees.append(tree)
            if grower is not None:
                dev_trees.append(round_trees)
            else:
                self.trees.append(round_trees)
            if callback is not None:
                callback(it, pred)
        t2 = self._sync_time()
        self.stats["setup_s"] = self.stats.get("setup_s", 0.0) + (t1 - t0)
        self.stats["boost_s"] = self.stats.get("boost_s", 0.0) + (t2 - t1)
        if grower is not None:
            # the only device->host copy of training: every tree's heap arrays at once
            if dev_trees:
                host = torch.stack([torch.stack(r) for r in dev_trees]).cpu()
                self.trees += [[self._heap_tree(host[i, k]) for k in range(K)] for i in range(len(dev_trees))]
            b, s = grower.stats()
            self.stats["hist_builds"] += b
            self.stats["hist_subtracted"] += s
            # the fused route + scan's look-back never timed out (a timeout means
            # its partition was wrong: fail loudly rather than return bad trees)
            faults = grower.scan_faults()
            if faults:
                raise RuntimeError(f"GBDT route+scan: {faults} look-back timeouts (csrc/gbdt.hip route_scan_kernel)")
        return pred

    def predict_margin(self, X: torch.Tensor) -> torch.Tensor:
        X = X.to(self.device).float()
        pred = self._base(X.shape[0])
        for round_trees in self.trees:
            for k, t in enumerate(round_trees):
                feat = torch.tensor(t.feature, device=self.device)
                thr = torch.tensor(t.threshold, device=self.device, dtype=torch.float32)
                left = torch.tensor(t.left, device=self.device)
                right = torch.tensor(t.right, device=self.device)
                val = torch.tensor(t.value, device=self.device)
                node = torch.zeros(X.shape[0], dtype=torch.long, device=self.device)
                for _ in range(self.p.max_depth + 1):
                    f = feat[node]
                    leafm = f < 0
                    if bool(leafm.all()):
                        break
                    xv = X.gather(1, f.clamp_min(0)[:, None])[:, 0]
                    nxt = torch.where(xv <= thr[node], left[node], right[node])
                    node = torch.where(leafm, node, nxt)
                pred[:, k] += val[node]
        return pred

    def metric(self, pred: torch.Tensor, y: torch.Tensor) -> dict:
        obj = self.p.objective
        if obj.startswith("multi:"):
            pr = torch.softmax(pred, 1)
            ll = -torch.log(pr.gather(1, y.long()[:, None]).clamp_min(1e-15)).mean()
            return {"mlogloss": float(ll), "accuracy": float((pr.argmax(1) == y.long()).float().mean())}
        if obj == "binary:logistic":
            pr = torch.sigmoid(pred[:, 0])
            yy = y.float()
            ll = -(yy * torch.log(pr.clamp_min(1e-15)) + (1 - yy) * torch.log((1 - pr).clamp_min(1e-15))).mean()
            return {"logloss": float(ll), "accuracy": float(((pr > 0.5).float() == yy).float().mean())}
        return {"rmse": float(torch.sqrt(((pred[:, 0] - y.float()) ** 2).mean()))}
