"""Explicit forward/backward engine for ResNet-50 training on MI355X.

Autograd executes a network as a chain of independent ops, so every op pays
its own passes over HBM and every activation with two consumers (the
bottleneck input feeds conv1 AND the residual) gets an extra gradient-sum
kernel.  This engine runs the same ``models.resnet.ResNet`` parameters
through a hand-scheduled step instead, built around the fused 1x1-conv MFMA
GEMMs of ``csrc/conv1x1.hip``:

forward, per bottleneck (``B`` = BatchNorm, ``R`` = ReLU)::

    c1 = conv1(x)                [GEMM, epilogue: B1 statistics]
    a1 = R(B1(c1))               [apply pass; at 56x56 inside conv2 (halo prologue)]
    c2 = conv2(a1)               [3x3 implicit GEMM (csrc/igemm.hip), epilogue: B2 stats]
    c3 = conv3(R(B2(c2)))        [GEMM, prologue: B2+R while staging A -- the
                                  B2 output never reaches HBM; epilogue: B3 stats]
    cd = down(x)                 [GEMM, strided row gather, epilogue: Bd stats]
    out = R(B3(c3) + (Bd(cd) | x))  [one apply pass, 1-bit ReLU mask saved]

backward, per bottleneck (``g`` = gradient at the pre-ReLU block sum, already
masked; it and B3's reduction sums come out of the NEXT block's conv1 dgrad
epilogue)::

    dc3 (, dcd) = B3 (, Bd) apply-backward of g        [NOT a pass: computed in the A
                                                        staging of the dgrads below,
                                                        written through for the wgrads]
    g2 = conv3 dgrad (dc3), masked by R'(B2(c2)) + B2 reduction sums   [GEMM epilogue]
    dW3 = sum dc3^T R(B2(c2))                          [GEMM, B2+R recomputed in the prologue]
    dc2 = B2 apply-backward(g2) ; dW2 [3x3 implicit GEMM, csrc/wgrad_dma.hip] ;
          da1 [implicit GEMM with bn1's mask + sums fused; stride 2: four sub-pixel
          class GEMMs in one launch, kubedl_amd/ops/conv.py]
    dc1 = B1 apply-backward(da1)                       [in conv1 dgrad's A staging]
    g_prev = conv1 dgrad(dc1) + d(identity) (strided gather of the downsample dgrad),
             masked by the previous block's ReLU bits, + B3_prev (and Bd_prev)
             reduction sums                            [GEMM epilogue]
    dW1, dWd                                           [GEMM]

which deletes, per block, the B1/B3/Bd statistics passes, the B2 apply pass
(and its activation), the B2 and B3 reduction passes, the downsample BN
output, and autograd's residual-gradient add kernel.

Gradients are written straight into the ``FlatParamSpace`` gradient buffer
and each parameter is announced to ``FlatDDP.ready`` as soon as it is final,
so the bucketed RCCL all-reduce overlaps the rest of the backward exactly as
with autograd hooks.

Two kernel backends with identical semantics: ``HipKernels`` (the CDNA4
kernels; the only GPU path) and ``TorchKernels`` (plain fp32 PyTorch with the
same bf16 rounding points), which lets the CPU test-suite check the engine's
data flow against autograd on ``resnet_tiny``.

The reference has no model code; this is the data plane of
BASELINE.json's "PyTorchJob ResNet-50 DDP bf16" config.
"""
from __future__ import annotations

import contextlib
import math
import dataclasses
import os

import torch
import torch.nn.functional as F

from kubedl_amd.models.resnet import BNAct, Bottleneck, ResNet
from kubedl_amd.ops.conv import S2_TAPS, s2_dgrad_weights, stem_grad_from_k, stem_weights

REP = 32  # BN workspace replicas (csrc/bn_act.hip kReplicas)


def _nhwc_empty(n, c, h, w, like):
    # allocate channels_last directly (.contiguous(channels_last) on a fresh
    # NCHW tensor would launch a full-size copy kernel)
    return torch.empty((n, c, h, w), dtype=like.dtype, device=like.device, memory_format=torch.channels_last)


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels_last -> [N*H*W, C] view of the same memory."""
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _from_rows(r: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    c = r.shape[1]
    return r.view(n, h, w, c).permute(0, 3, 1, 2)


def _bfr(t: torch.Tensor) -> torch.Tensor:
    """Round an fp32 tensor through bf16 (the kernels' storage precision)."""
    return t.to(torch.bfloat16).float()


class BNState:
    """Per-layer BatchNorm bookkeeping of one step (module + saved statistics)."""

    def __init__(self, mod: BNAct, dev):
        self.mod = mod
        C = mod.channels
        self.C = C
        self.save_mean = torch.zeros(C, device=dev)
        self.save_invstd = torch.ones(C, device=dev)
        self.ws = None          # HIP workspace (replicas | coefs), self-cleaning
        self.xam = None         # stem: BN input at each max-pool window's argmax (native path)
        self.fin_done = False   # forward finalize already done by the producing GEMM (csrc/bn_fin.h)
        self.bfin_done = False  # backward finalize likewise
        # torch-backend state
        self.fsum = None        # (s1, s2, shift) forward sums
        self.fcoef = None       # (scale, shift)
        self.bsum = None        # (sa, sb) backward sums
        self.bcoef = None       # (k, c1, c0)


# ---------------------------------------------------------------------------- kernels
class HipKernels:
    """The CDNA4 path: csrc/conv1x1.hip GEMMs + csrc/bn_act.hip staged BN kernels."""

    name = "hip"

    def __init__(self, dev, fuse_fin: bool = True):
        from kubedl_amd.ops import _ext
        self.ext = _ext.load()
        self.dev = dev
        self._dw32 = {}
        self._ident = {}  # identity prologue coefficients [ones | zeros] per channel count
        # BN finalize folded into the producing conv GEMM's last arriving blocks
        # (csrc/bn_fin.h; EngineOptions.bn_fin = "kernel": separate finalize
        # launches).  Round 2 measured it neutral while its inlined tail made every
        # MASKX/STATS GEMM spill ~90 VGPRs; with the tail's replica sum chunked (no
        # spills) it is 19.33 / 19.37 vs 19.41 / 19.47 ms per step
        # (profiles/r03_knob_sweep.txt) and ~106 fewer launches
        self.fuse_fin = fuse_fin
        self._fin_ptrs = {}
        self.stem_path = None  # "kdl" | "miopen" once a forward ran (reported by bench / smoke)

    def fin_desc(self, st, dgamma, dbeta):
        """(Re)write st's finalize descriptor when a pointer it holds changed."""
        if not self.fuse_fin:
            return
        m = st.mod
        ptrs = (st.ws.data_ptr(), m.weight.data_ptr() if m.weight is not None else 0,
                m.running_mean.data_ptr(), st.save_mean.data_ptr(), st.save_invstd.data_ptr(),
                dgamma.data_ptr() if dgamma is not None else 0, dbeta.data_ptr() if dbeta is not None else 0)
        if self._fin_ptrs.get(id(st)) != ptrs:
            self.ext.bn_fin_desc(st.ws, m.weight, m.bias, m.running_mean, m.running_var, st.save_mean,
                                 st.save_invstd, dgamma, dbeta, float(m.momentum), float(m.eps))
            self._fin_ptrs[id(st)] = ptrs

    def _arm(self, st, M, st2=None, fwd=True):
        """The next conv GEMM finalizes st (and st2) itself."""
        if not self.fuse_fin or st.C > 2048 or st.C % 64:
            return
        self.ext.bn_fin_arm(st.ws, st2.ws if st2 is not None else None, st.C, M)
        for x in (st, st2):
            if x is not None:
                if fwd:
                    x.fin_done = True
                else:
                    x.bfin_done = True

    def init_bn(self, st: BNState):
        st.ws = torch.zeros(self.ext.bn_workspace_floats(st.C), device=self.dev)
        st.coef_off = self.ext.bn_coef_offset(st.C)

    def fcoef(self, st):  # [2C] scale | shift view of the workspace
        return st.ws[st.coef_off:st.coef_off + 2 * st.C]

    def bcoef(self, st):  # [3C] k | c1 | c0 backward coefficients (csrc/bn_act.hip ws_bcoef)
        return st.ws[st.coef_off + 2 * st.C:st.coef_off + 5 * st.C]

    def _fwd_acc(self, st):
        return st.ws[:REP * 2 * st.C]

    def _bwd_acc(self, st):
        return st.ws[REP * 2 * st.C:REP * 4 * st.C]

    # -- forward
    def conv1x1_fwd(self, x, w, stride, pro: BNState | None, out: BNState):
        n, cin, h, wd = x.shape
        cout = w.shape[0]
        ho, wo = (h - 1) // stride + 1, (wd - 1) // stride + 1
        y = _nhwc_empty(n, cout, ho, wo, x)
        M = n * ho * wo
        self._arm(out, M)
        self.ext.conv1x1_gemm(x, w, y, M, cout, cin, ho, wo, h, wd, stride,
                              self.fcoef(pro) if pro is not None else None, 1, out.mod.running_mean,
                              self._fwd_acc(out), None, None, None, None, 1, 0, 0, None, None, None, None)
        return y

    @staticmethod
    def relu_mask_like(x):  # bn_apply's packed ReLU mask: 1 bit per element
        return torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device)

    def conv1x1_fwd_res(self, c3, w, st3: BNState, res, xout, mbits, out: BNState, dual: BNState | None = None):
        """The next block's conv1 on x = relu(B3(c3) + res), the previous block's
        closing apply done in the GEMM's A staging (csrc/conv1x1.hip PRO_RES) and
        written through to ``xout`` with its packed ReLU mask ``mbits`` -- the
        same bits as bn_apply(c3, st3, res=res, want_mask=True); ``out``'s BN
        statistics in the epilogue; ``dual``: ``res`` is the downsample branch's
        BN input and the residual B_dual(res) (bn_apply's ``other``)."""
        n, cin, h, wd = c3.shape
        cout = w.shape[0]
        y = _nhwc_empty(n, cout, h, wd, c3)
        M = n * h * wd
        self._arm(out, M)
        self.ext.bn_res_pro_arm(res, self.fcoef(st3), cin, xout, mbits, self.fcoef(dual) if dual is not None else None)
        self.ext.conv1x1_gemm(c3, w, y, M, cout, cin, h, wd, h, wd, 1, None, 1, out.mod.running_mean,
                              self._fwd_acc(out), None, None, None, None, 1, 0, 0, None, None, None, None)
        return y

    def conv3x3_fwd(self, x, w, stride, out: BNState, pro: BNState | None = None, aout=None):
        """3x3 pad-1 conv as an implicit GEMM (LDS-DMA main loop, csrc/igemm.hip)
        with ``out``'s BN statistics in the epilogue (no separate stats pass);
        ``pro``: the input is relu(B_pro(x)), applied inside the conv (at 56x56 to
        the input halo in LDS, csrc/halo3x3.hip), written through to ``aout``."""
        n, cin, h, wd = x.shape
        cout = w.shape[0]
        ho, wo = (h - 1) // stride + 1, (wd - 1) // stride + 1
        y = _nhwc_empty(n, cout, ho, wo, x)
        self._arm(out, n * ho * wo)
        if aout is not None:
            self.ext.conv3x3_aout_arm(aout)
        self.ext.conv3x3_gemm(x, w, y, n, h, wd, cin, cout, stride, self.fcoef(pro) if pro is not None else None, 1,
                              out.mod.running_mean, self._fwd_acc(out), None, None, None)
        return y

    def _ws32(self, key, n):
        t = self._dw32.get(key)
        if t is None or t.numel() < n:
            t = self._dw32[key] = torch.empty(n, device=self.dev)
        return t

    def bn_stats(self, x, st):
        self.ext.bn_stage_fwd_stats(x, st.ws, x.numel() // st.C, st.C)

    def bn_finalize(self, st, M, x=None, gemm_shift=False):
        if st.fin_done:  # the producing GEMM did it
            st.fin_done = False
            return
        m = st.mod
        self.ext.bn_stage_fwd_finalize(None if gemm_shift else x, m.running_mean if gemm_shift else None, st.ws, M,
                                       st.C, m.weight, m.bias, m.running_mean, m.running_var, st.save_mean,
                                       st.save_invstd, True, float(m.momentum), float(m.eps))

    def bn_apply(self, x, st, relu=True, res=None, other=None, want_mask=False):
        M = x.numel() // st.C
        y = torch.empty_like(x)
        mb = torch.empty(M * st.C // 8, dtype=torch.uint8, device=x.device) if want_mask else None
        xd, std_ = other if other is not None else (None, None)
        self.ext.bn_stage_fwd_apply(x, st.ws, res, xd, std_.ws if std_ is not None else None, y, mb, M, st.C, relu)
        return y, mb

    def stem_conv(self, x, w, st):
        """7x7 / stride 2 stem conv on csrc/stem.hip (MFMA, the stem BN's
        statistics in the epilogue) at any input size.  Returns (c0, statistics
        already in st's workspace)."""
        if not (tuple(w.shape) == (64, 3, 7, 7) and x.shape[1] == 3 and x.dtype == torch.bfloat16
                and x.is_contiguous(memory_format=torch.channels_last)):
            raise ValueError(f"HIP engine stem: 3-channel bf16 NHWC input and a [64, 3, 7, 7] conv expected "
                             f"(got x {tuple(x.shape)} {x.dtype}, w {tuple(w.shape)})")
        oh, ow = (x.shape[2] - 1) // 2 + 1, (x.shape[3] - 1) // 2 + 1
        c0 = _nhwc_empty(x.shape[0], 64, oh, ow, x)
        # the channels_last [64, 3, 7, 7] parameter itself (the kernel reorders it
        # while staging); contiguous NCHW weights (tests) take the K-order copy
        wk = w if w.is_contiguous(memory_format=torch.channels_last) else stem_weights(w)
        self.ext.stem7x7_fwd(x, wk, c0, st.mod.running_mean, self._fwd_acc(st))
        self.stem_path = "kdl"
        return c0, True

    def stem_fwd(self, c0, st, gemm_stats=False):
        m = st.mod
        # native stem: also keep x at each window's argmax, so the backward's BN
        # sums run over the pooled cells (csrc/bn_act.hip bn_pool_fwd_kernel)
        y, mean, invstd, idx, xam = self.ext.bn_pool_fwd(c0, m.weight, m.bias, m.running_mean, m.running_var, True,
                                                         float(m.momentum), float(m.eps), st.ws, gemm_stats,
                                                         gemm_stats)
        st.save_mean, st.save_invstd = mean, invstd
        st.xam = xam if gemm_stats else None
        return y, idx

    # -- backward
    def head_mask_reduce(self, dfeat, hw, mbits, x, st, xd=None, std_=None):
        M = x.numel() // st.C
        g = torch.empty_like(x)
        self.ext.bn_stage_bwd_mask_reduce(dfeat.to(torch.bfloat16).contiguous(), hw, 1.0 / hw, mbits, x,
                                          st.save_mean, g, st.ws, M, st.C, xd,
                                          std_.save_mean if std_ is not None else None,
                                          std_.ws if std_ is not None else None)
        return g

    def bn_bwd_finalize(self, st, M, dgamma, dbeta):
        if st.bfin_done:  # the producing GEMM did it
            st.bfin_done = False
            return
        self.ext.bn_stage_bwd_finalize(st.ws, M, st.C, st.mod.weight, st.save_mean, st.save_invstd, dgamma, dbeta,
                                       True)

    def bn_bwd_apply(self, g, x, st, xd=None, std_=None):
        M = x.numel() // st.C
        dx = torch.empty_like(x)
        dxd = torch.empty_like(xd) if xd is not None else None
        self.ext.bn_stage_bwd_apply(g, x, st.ws, dx, xd, std_.ws if std_ is not None else None, dxd, M, st.C)
        return dx, dxd

    def bn_bwd_full(self, dy, x, st, dgamma, dbeta):
        """BN+ReLU backward with the mask recomputed from x: reduce pass, then the
        staged finalize (dgamma/dbeta straight into the gradient buffer) + apply."""
        m = st.mod
        M = x.numel() // st.C
        self.ext.bn_stage_bwd_reduce(dy, x, m.weight, m.bias, st.save_mean, st.save_invstd, st.ws, M, st.C, True)
        self.bn_bwd_finalize(st, M, dgamma, dbeta)
        dx = torch.empty_like(x)
        self.ext.bn_stage_bwd_apply_maskx(dy, x, m.weight, m.bias, st.save_mean, st.save_invstd, st.ws, dx, M, st.C)
        return dx

    def _arm_bpro(self, bpro, C):
        """Fuse a BN-backward apply into the next GEMM's A staging (csrc/conv1x1.hip
        PRO_BWD): bpro = (x, st, out) -- A' = k g + c1 x + c0 of BN ``st`` with
        input ``x``, written through to ``out`` (None: not materialised)."""
        if bpro is not None:
            x, st, out = bpro
            self.ext.bn_bwd_pro_arm(x, st.ws, C, out)

    def dgrad_maskx(self, g, wt, x2, st2, bpro=None):
        """g [.., K=cout] -> masked d(input) [.., cin] + st2 backward sums; wt = W^T [cin, cout]."""
        n, cout, h, w = g.shape
        cin = wt.shape[0]
        out = _nhwc_empty(n, cin, h, w, g)
        M = n * h * w
        self._arm(st2, M, fwd=False)
        self._arm_bpro(bpro, cout)
        self.ext.conv1x1_gemm(g, wt, out, M, cin, cout, 0, 0, 0, 0, 1, None, 2, None, self._bwd_acc(st2), x2,
                              st2.save_mean, self.fcoef(st2), None, 1, 0, 0, None, None, None, None)
        return out

    def dgrad3x3_maskx(self, g, wd, x1, st1):
        """Stride-1 3x3 dgrad (implicit GEMM, B = wd [Cin][3][3][Cout]) with the
        previous BN+ReLU's mask and backward sums fused into the epilogue."""
        n, cout, h, w = g.shape
        cin = wd.shape[0]
        out = _nhwc_empty(n, cin, h, w, g)
        self._arm(st1, n * h * w, fwd=False)
        self.ext.conv3x3_gemm(g, wd, out, n, h, w, cout, cin, 1, None, 2, None, self._bwd_acc(st1), x1,
                              st1.save_mean, self.fcoef(st1))
        return out

    def dgrad3x3s2_maskx(self, g, ball, x1, st1):
        """Stride-2 3x3 dgrad as four sub-pixel class GEMMs in one launch
        (csrc/igemm.hip G_DGRAD2; ball = class-major weights [Cin][9 Cout],
        kubedl_amd/ops/conv.py) with bn1's mask and backward sums fused.  The
        input x1 is 2h x 2w or, for an odd input size, 2h - 1 (2w - 1): the
        last sub-pixel row / column is masked in the epilogue."""
        n, cout, h, w = g.shape
        cin = ball.shape[0]
        hx, wx = x1.shape[-2:]
        out = _nhwc_empty(n, cin, hx, wx, g)
        self._arm(st1, n * hx * wx, fwd=False)
        self.ext.conv3x3_s2_dgrad(g, ball, out, n, h, w, cout, cin, 2, self._bwd_acc(st1), x1, st1.save_mean,
                                  self.fcoef(st1), hx, wx)
        return out

    def dgrad_plain(self, g, wt, bpro=None):
        n, cout, h, w = g.shape
        cin = wt.shape[0]
        out = _nhwc_empty(n, cin, h, w, g)
        self._arm_bpro(bpro, cout)
        self.ext.conv1x1_gemm(g, wt, out, n * h * w, cin, cout, 0, 0, 0, 0, 1, None, 0, None, None, None, None, None,
                              None, 1, 0, 0, None, None, None, None)
        return out

    def dgrad_res(self, g, wt, eres, res_stride, prev=None, bpro=None):
        """conv1 dgrad + d(identity); with ``prev`` = (mbits, c3, st3, cd, std) the
        previous block's ReLU mask is applied and its BN sums accumulated."""
        n, cout, h, w = g.shape
        cin = wt.shape[0]
        out = _nhwc_empty(n, cin, h, w, g)
        M = n * h * w
        if prev is None:
            self._arm_bpro(bpro, cout)
            self.ext.conv1x1_gemm(g, wt, out, M, cin, cout, 0, 0, 0, 0, 1, None, 4, None, None, None, None, None, eres,
                                  res_stride, h, w, None, None, None, None)
        else:
            mbits, c3, st3, cd, std_ = prev
            self._arm(st3, M, std_, fwd=False)
            self._arm_bpro(bpro, cout)
            self.ext.conv1x1_gemm(g, wt, out, M, cin, cout, 0, 0, 0, 0, 1, None, 3, None, self._bwd_acc(st3), c3,
                                  st3.save_mean, None, eres, res_stride, h, w, mbits, cd,
                                  std_.save_mean if std_ is not None else None,
                                  self._bwd_acc(std_) if std_ is not None else None)
        return out

    def wgrad(self, g, x, stride, pro: BNState | None, dW, gbpro=None):
        """1x1 weight gradient; ``gbpro`` = (gx, st): G is the BN-backward apply
        k g + c1 gx + c0 of BN ``st``, computed in the G fragments (BWDG)."""
        n, cout, ho, wo = g.shape
        _, cin, h, w = x.shape
        M = n * ho * wo
        key = (M, cout, cin)  # split-M slab workspace, shared by the layers of one shape (stream-ordered)
        need = self.ext.conv1x1_wgrad_splits(M, cout, cin) * cout * cin  # (tile mode may change: set_wgrad_big)
        dw32 = self._dw32.get(key)
        if dw32 is None or dw32.numel() < need:
            dw32 = self._dw32[key] = torch.empty(need, device=g.device)
        if gbpro is not None:
            self.ext.bn_bwd_pro_arm(gbpro[0], gbpro[1].ws, cout, None)
        self.ext.conv1x1_wgrad(g, x, self.fcoef(pro) if pro is not None else None, dw32, dW.view(cout, cin), 1.0,
                               M, cout, cin, ho, wo, h, w, stride)

    def wgrad_gram(self, g, x2, st2: BNState | None, st3: BNState, w3, dW):
        """A 1x1 conv's weight gradient with its output BN's backward apply folded in
        (csrc/conv1x1.hip Gram fold): dW = diag(k) g^T a + diag(c1) W (a^T a) + c0 (1^T a),
        a = relu(B2(x2)) (conv3) or x2 itself when ``st2`` is None (a stride-1
        downsample conv: its input is a block output, already >= 0) -- the BN's
        input gradient is never materialised.  G on the weight-gradient kernel
        (fp32, left in its slab workspace), Q | s on the Gram kernel, then the fold."""
        n, cout, ho, wo = g.shape
        _, cin, h, w = x2.shape
        M = n * ho * wo
        key = (M, cout, cin)
        need = self.ext.conv1x1_wgrad_splits(M, cout, cin) * cout * cin
        dw32 = self._dw32.get(key)
        if dw32 is None or dw32.numel() < need:
            dw32 = self._dw32[key] = torch.empty(need, device=g.device)
        pro = self.fcoef(st2) if st2 is not None else None
        self.ext.conv1x1_wgrad(g, x2, pro, dw32, None, 1.0, M, cout, cin, ho, wo, h, w, 1)
        if pro is None:  # relu(x * 1 + 0) = x for the non-negative block output
            pro = self._ident.get(cin)
            if pro is None:
                pro = self._ident[cin] = torch.cat([torch.ones(cin, device=g.device), torch.zeros(cin, device=g.device)])
        qs = self._ws32(("gram", M, cin), self.ext.conv1x1_gram_floats(M, cin))
        self.ext.conv1x1_gram(x2, pro, qs, M, cin)
        self.ext.gram_fold(dw32, qs, w3.view(cout, cin), self.bcoef(st3), dW.view(cout, cin), cout, cin)

    def wgrad3x3(self, g, x, stride, dW, pro: BNState | None = None):
        """3x3 pad-1 weight gradient straight into ``dW`` (channels_last = OHWI):
        the 56x56 stage's input halo kernel (csrc/halo3x3.hip) or the LDS-DMA
        implicit GEMM (csrc/wgrad_dma.hip), into fp32 slabs + fixed-order reduce;
        ``pro``: the conv input is relu(B_pro(x)), applied while staging."""
        n, cout, ho, wo = g.shape
        _, cin, h, w = x.shape
        M = n * ho * wo
        key = (M, cout, 9 * cin, h, stride)
        need = self.ext.conv3x3_wgrad_slabs(n, h, w, cin, cout, stride) * cout * 9 * cin
        dw32 = self._dw32.get(key)
        if dw32 is None or dw32.numel() < need:
            dw32 = self._dw32[key] = torch.empty(need, device=g.device)
        self.ext.conv3x3_wgrad(g, x, self.fcoef(pro) if pro is not None else None, dw32, dW, 1.0, n, h, w, cin, cout,
                               stride)

    def stem_wgrad(self, dc0, x, dw):
        """Stem conv weight gradient into ``dw`` ([64, 3, 7, 7]): csrc/stem.hip
        (both operands read pixel-major from LDS, no patch matrix), any input size."""
        ws = self._stem_ws(x.shape[0], x.device, x.shape[2], x.shape[3])
        if dw.is_contiguous(memory_format=torch.channels_last):  # written in place, raw layout
            self.ext.stem7x7_wgrad(dc0, x, ws[0], dw)
        else:
            self.ext.stem7x7_wgrad(dc0, x, ws[0], ws[1])
            dw.copy_(stem_grad_from_k(ws[1]))

    def stem_bwd(self, dp, idx, c0, st, dgamma, dbeta, with_dx=True):
        m = st.mod
        dx, dg, db = self.ext.bn_pool_bwd(dp, idx, c0, m.weight, m.bias, st.save_mean, st.save_invstd, True, st.ws,
                                          with_dx)
        dgamma.copy_(dg)
        dbeta.copy_(db)
        return dx

    def _stem_native_bwd(self, x, c0, dw):
        """The fused pool-backward + weight-gradient kernel serves 3x224x224 (its
        pooled-gradient gather is specialised to 112 -> 56); other sizes take the
        pooling backward pass + the general weight-gradient kernel."""
        return (tuple(x.shape[1:]) == (3, 224, 224) and tuple(dw.shape) == (64, 3, 7, 7)
                and x.is_contiguous(memory_format=torch.channels_last)
                and c0.is_contiguous(memory_format=torch.channels_last))

    def stem_backward(self, dp, idx, c0, x, st, dgamma, dbeta, dw):
        """Stem BN + ReLU + max-pool backward and the 7x7 weight gradient.  Native
        path: the BN sums pass only (no full-resolution apply), then
        csrc/stem.hip builds each tile's conv-output gradient in LDS from c0,
        the pooled gradient and the BN coefficients while it reduces dW."""
        xam = getattr(st, "xam", None)
        if xam is None or not self._stem_native_bwd(x, c0, dw):
            self.stem_wgrad(self.stem_bwd(dp, idx, c0, st, dgamma, dbeta), x, dw)
            return
        # BN sums over the pooled cells: sum(dp * mask(xam)), sum(dp * mask * (xam - mean))
        # == the per-pixel sums of the max-pool backward (each cell's gradient
        # lands on its argmax pixel); M of the finalize stays the pixel count
        m = st.mod
        self.ext.bn_stage_bwd_reduce(dp, xam, m.weight, m.bias, st.save_mean, st.save_invstd, st.ws,
                                     dp.numel() // st.C, st.C, True)
        self.bn_bwd_finalize(st, c0.numel() // st.C, dgamma, dbeta)
        st.xam = None
        nb = x.shape[0]
        ws = self._stem_ws(nb, x.device)
        if dw.is_contiguous(memory_format=torch.channels_last):  # written in place, raw layout
            self.ext.stem7x7_wgrad_bn(c0, dp, idx, st.ws, x, ws[0], dw)
        else:
            self.ext.stem7x7_wgrad_bn(c0, dp, idx, st.ws, x, ws[0], ws[1])
            dw.copy_(stem_grad_from_k(ws[1]))

    def head_ok(self, fmap, w, y) -> bool:
        n, c = fmap.shape[:2]
        L = w.shape[0]
        return (fmap.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.is_contiguous()
                and fmap.is_contiguous(memory_format=torch.channels_last) and n % 8 == 0 and c % 8 == 0
                and L <= 8192 and y.dtype == torch.int64)

    def head(self, fmap, w, b, y, dw, db):
        """Pool -> fc -> softmax CE -> backward on csrc/head.hip: (loss [1],
        dfeat [n, c] bf16); dW / db written into ``dw`` / ``db``."""
        n, c = fmap.shape[:2]
        L = w.shape[0]
        key = ("head", n, c, L)
        ws = self._dw32.get(key)
        if ws is None:
            s1, s2 = self.ext.head_splits(n, c, L)
            bf = dict(dtype=torch.bfloat16, device=fmap.device)
            f32 = dict(dtype=torch.float32, device=fmap.device)
            ws = self._dw32[key] = dict(feat=torch.empty(n, c, **bf), part1=torch.empty(s1 * n * L, **f32),
                                        lrow=torch.empty(n, **f32), dl=torch.empty(n, self.ext.head_lpad(L), **bf),
                                        dlT=torch.empty(L, n, **bf), part2=torch.empty(s2 * n * c, **f32),
                                        dfeat=torch.empty(n, c, **bf))
        yc = y if y.is_contiguous() else y.contiguous()
        self.ext.head_forward(fmap, w, b, yc, ws["feat"], ws["part1"], ws["lrow"], ws["dl"], ws["dlT"])
        loss = torch.empty(1, dtype=torch.float32, device=fmap.device)  # fresh per step (returned)
        self.ext.head_backward(ws["feat"], w, ws["dl"], ws["dlT"], ws["part2"], ws["dfeat"], dw, db, ws["lrow"],
                               loss)
        return loss.view(()), ws["dfeat"]

    def _stem_ws(self, nb, device, h=224, w=224):
        key = ("stem", nb, h, w)
        ws = self._dw32.get(key)
        if ws is None:
            ws = (torch.empty(self.ext.stem7x7_wgrad_slabs(nb, h, w) * 64 * 224, device=device),
                  torch.empty(64, 224, device=device, dtype=torch.bfloat16))
            self._dw32[key] = ws
        return ws


class TorchKernels:
    """Reference semantics of every HipKernels op in fp32 PyTorch (CPU tests)."""

    name = "torch"

    def __init__(self, dev):
        self.dev = dev

    def init_bn(self, st):
        pass

    @staticmethod
    def _pro(x, st):
        sc, sf = st.fcoef
        return _bfr(F.relu(x.float() * sc.view(1, -1, 1, 1) + sf.view(1, -1, 1, 1)))

    def conv1x1_fwd(self, x, w, stride, pro, out):
        a = self._pro(x, pro) if pro is not None else x.float()
        y = F.conv2d(a[:, :, ::stride, ::stride], w.float()[:, :, None, None])
        y = y.to(x.dtype)
        self._stats(y, out, out.mod.running_mean.clone())
        return y.contiguous(memory_format=torch.channels_last)

    @staticmethod
    def relu_mask_like(x):  # bn_apply's mask: a bool tensor here
        return torch.empty(x.shape, dtype=torch.bool, device=x.device)

    def conv1x1_fwd_res(self, c3, w, st3, res, xout, mbits, out, dual=None):
        if dual is not None:
            x, mb = self.bn_apply(c3, st3, relu=True, other=(res, dual), want_mask=True)
        else:
            x, mb = self.bn_apply(c3, st3, relu=True, res=res, want_mask=True)
        xout.copy_(x)
        mbits.copy_(mb)
        return self.conv1x1_fwd(xout, w, 1, None, out)

    def conv3x3_fwd(self, x, w, stride, out, pro=None, aout=None):
        a = self._pro(x, pro) if pro is not None else x.float()
        if aout is not None:
            aout.copy_(a)
        y = F.conv2d(a, w.float(), stride=stride, padding=1).to(x.dtype)
        self._stats(y, out, out.mod.running_mean.clone())
        return y.contiguous(memory_format=torch.channels_last)

    @staticmethod
    def bcoef(st):
        return st.bcoef

    def _stats(self, y, st, shift):
        d = _rows(y.float()) - shift
        st.fsum = (d.sum(0), (d * d).sum(0), shift)

    def bn_stats(self, x, st):
        self._stats(x, st, _rows(x.float())[0].clone())

    def bn_finalize(self, st, M, x=None, gemm_shift=False):
        s1, s2, K = st.fsum
        m = st.mod
        m1 = s1 / M
        var = (s2 / M - m1 * m1).clamp_min(0)
        mean = K + m1
        invstd = torch.rsqrt(var + m.eps)
        st.save_mean, st.save_invstd = mean, invstd
        with torch.no_grad():
            unb = var * M / (M - 1) if M > 1 else var
            m.running_mean.mul_(1 - m.momentum).add_(m.momentum * mean)
            m.running_var.mul_(1 - m.momentum).add_(m.momentum * unb)
        sc = m.weight.float() * invstd
        st.fcoef = (sc, m.bias.float() - mean * sc)

    def bn_apply(self, x, st, relu=True, res=None, other=None, want_mask=False):
        sc, sf = st.fcoef
        o = x.float() * sc.view(1, -1, 1, 1) + sf.view(1, -1, 1, 1)
        if other is not None:
            xd, sd = other
            o = o + (xd.float() * sd.fcoef[0].view(1, -1, 1, 1) + sd.fcoef[1].view(1, -1, 1, 1))
        elif res is not None:
            o = o + res.float()
        mask = o > 0 if want_mask else None
        if relu:
            o = F.relu(o)
        return o.to(x.dtype).contiguous(memory_format=torch.channels_last), mask

    @staticmethod
    def stem_conv(x, w, st):
        return F.conv2d(x, w, stride=2, padding=3).contiguous(memory_format=torch.channels_last), False

    def stem_fwd(self, c0, st, gemm_stats=False):
        self.bn_stats(c0, st)
        self.bn_finalize(st, c0.numel() // st.C)
        a, _ = self.bn_apply(c0, st, relu=True)
        y, idx = F.max_pool2d(a.float(), 3, 2, 1, return_indices=True)
        return y.to(c0.dtype).contiguous(memory_format=torch.channels_last), idx

    def head_mask_reduce(self, dfeat, hw, mask, x, st, xd=None, std_=None):
        n, c, h, w = x.shape
        dy = _bfr(_bfr(dfeat.float()) / hw).view(n, c, 1, 1).expand(n, c, h, w)
        g = torch.where(mask, dy, torch.zeros_like(dy))
        self._bsum(g, x, st)
        if xd is not None:
            self._bsum(g, xd, std_)
        return g.to(x.dtype).contiguous(memory_format=torch.channels_last)

    def _bsum(self, g, x, st):
        gr = _rows(g.float())
        st.bsum = (gr.sum(0), (gr * (_rows(x.float()) - st.save_mean)).sum(0))

    def bn_bwd_finalize(self, st, M, dgamma, dbeta):
        sa, sb = st.bsum
        inv = st.save_invstd
        db, dg = sa, sb * inv
        dgamma.copy_(dg)
        dbeta.copy_(db)
        k = st.mod.weight.float() * inv
        c1 = -k * inv * dg / M
        c0 = -k * db / M - c1 * st.save_mean
        st.bcoef = (k, c1, c0)

    @staticmethod
    def _bapply(g, x, st):
        k, c1, c0 = (t.view(1, -1, 1, 1) for t in st.bcoef)
        return (k * g.float() + c1 * x.float() + c0).to(x.dtype).contiguous(memory_format=torch.channels_last)

    def bn_bwd_apply(self, g, x, st, xd=None, std_=None):
        return self._bapply(g, x, st), (self._bapply(g, xd, std_) if xd is not None else None)

    def bn_bwd_full(self, dy, x, st, dgamma, dbeta):
        sc, sf = st.fcoef
        mask = (x.float() * sc.view(1, -1, 1, 1) + sf.view(1, -1, 1, 1)) > 0
        g = torch.where(mask, dy.float(), torch.zeros_like(dy.float()))
        self._bsum(g, x, st)
        self.bn_bwd_finalize(st, x.numel() // st.C, dgamma, dbeta)
        return self._bapply(g, x, st)

    def _bpro(self, g, bpro):
        """A operand of a GEMM with a fused BN-backward apply (HipKernels._arm_bpro)."""
        if bpro is None:
            return g
        x, st, out = bpro
        a = self._bapply(g, x, st)
        if out is not None:
            out.copy_(a)
        return a

    def dgrad_maskx(self, g, wt, x2, st2, bpro=None):
        g = self._bpro(g, bpro)
        d = _bfr(F.conv2d(g.float(), wt.float().unsqueeze(-1).unsqueeze(-1)))
        sc, sf = st2.fcoef
        mask = (x2.float() * sc.view(1, -1, 1, 1) + sf.view(1, -1, 1, 1)) > 0
        d = torch.where(mask, d, torch.zeros_like(d))
        self._bsum(d, x2, st2)
        return d.to(g.dtype).contiguous(memory_format=torch.channels_last)

    def dgrad3x3_maskx(self, g, wd, x1, st1):
        d = _bfr(F.conv2d(g.float(), wd.float(), padding=1))
        sc, sf = st1.fcoef
        mask = (x1.float() * sc.view(1, -1, 1, 1) + sf.view(1, -1, 1, 1)) > 0
        d = torch.where(mask, d, torch.zeros_like(d))
        self._bsum(d, x1, st1)
        return d.to(g.dtype).contiguous(memory_format=torch.channels_last)

    def dgrad3x3s2_maskx(self, g, w, x1, st1):
        d = _bfr(torch.nn.grad.conv2d_input(x1.shape, w.float(), g.float(), stride=2, padding=1))
        sc, sf = st1.fcoef
        mask = (x1.float() * sc.view(1, -1, 1, 1) + sf.view(1, -1, 1, 1)) > 0
        d = torch.where(mask, d, torch.zeros_like(d))
        self._bsum(d, x1, st1)
        return d.to(g.dtype).contiguous(memory_format=torch.channels_last)

    def dgrad_plain(self, g, wt, bpro=None):
        g = self._bpro(g, bpro)
        return F.conv2d(g.float(), wt.float().unsqueeze(-1).unsqueeze(-1)).to(g.dtype).contiguous(
            memory_format=torch.channels_last)

    def dgrad_res(self, g, wt, eres, res_stride, prev=None, bpro=None):
        g = self._bpro(g, bpro)
        d = _bfr(F.conv2d(g.float(), wt.float().unsqueeze(-1).unsqueeze(-1)))
        r = torch.zeros_like(d)
        r[:, :, ::res_stride, ::res_stride] = eres.float()
        d = _bfr(d + r)
        if prev is not None:
            mask, c3, st3, cd, std_ = prev
            d = torch.where(mask, d, torch.zeros_like(d))
            self._bsum(d, c3, st3)
            if cd is not None:
                self._bsum(d, cd, std_)
        return d.to(g.dtype).contiguous(memory_format=torch.channels_last)

    def wgrad(self, g, x, stride, pro, dW, gbpro=None):
        if gbpro is not None:
            g = self._bapply(g, gbpro[0], gbpro[1])
        a = self._pro(x, pro) if pro is not None else x.float()
        a = _rows(a[:, :, ::stride, ::stride].contiguous(memory_format=torch.channels_last))
        dW.copy_((_rows(g.float()).t() @ a).view_as(dW))

    def wgrad_gram(self, g, x2, st2, st3, w3, dW):
        """The Gram fold's algebra in fp32 (HipKernels.wgrad_gram)."""
        a = _rows((self._pro(x2, st2) if st2 is not None else x2.float()).contiguous(memory_format=torch.channels_last))
        G = _rows(g.float().contiguous(memory_format=torch.channels_last)).t() @ a
        Q = a.t() @ a
        k, c1, c0 = st3.bcoef
        W = w3.float().view(w3.shape[0], -1)
        dW.copy_((k[:, None] * G + c1[:, None] * (W @ Q) + c0[:, None] * a.sum(0)[None, :]).view_as(dW))

    def wgrad3x3(self, g, x, stride, dW, pro=None):
        a = self._pro(x, pro) if pro is not None else x.float()
        dW.copy_(torch.nn.grad.conv2d_weight(a, tuple(dW.shape), g.float(), stride=stride, padding=1))

    def stem_backward(self, dp, idx, c0, x, st, dgamma, dbeta, dw):
        self.stem_wgrad(self.stem_bwd(dp, idx, c0, st, dgamma, dbeta), x, dw)

    @staticmethod
    def stem_wgrad(dc0, x, dw):
        dw.copy_(torch.nn.grad.conv2d_weight(x.float(), dw.shape, dc0.float(), stride=2, padding=3))

    def stem_bwd(self, dp, idx, c0, st, dgamma, dbeta):
        sc, sf = st.fcoef
        n, c, h, w = c0.shape
        # overlapping 3x3/s2 windows: a pixel that is the max of several windows
        # receives the sum of their gradients (scatter-add, not unpool's overwrite)
        da = torch.zeros(n, c, h * w, dtype=torch.float32, device=c0.device)
        da.scatter_add_(2, idx.reshape(n, c, -1), dp.float().reshape(n, c, -1))
        da = da.view(n, c, h, w).to(c0.dtype).contiguous(memory_format=torch.channels_last)
        return self.bn_bwd_full(da, c0, st, dgamma, dbeta)


# ---------------------------------------------------------------------------- engine
@dataclasses.dataclass
class EngineOptions:
    """Schedule choices of the engine.  Every default is the measured winner
    (docs/perf_notes.md, profiles/r03*_ab.txt); A/B experiments override them
    through ONE variable, ``KDL_ENGINE="key=value,..."`` (e.g.
    ``KDL_ENGINE=side=0`` for the single-stream schedule)."""
    # weight gradients on a second HIP stream (0: single stream -- 10.7k vs
    # 11.3k img/s when introduced); side_prio: its HIP stream priority
    side: bool = True
    side_prio: int = 0
    # BN finalize in the producing GEMM's last blocks ("gemm") or own launches ("kernel")
    bn_fin: str = "gemm"
    # downsample conv of the forward on the side stream
    down_side: bool = True
    # closing BN3 + residual + ReLU in the successor's conv1 staging (up to this K;
    # 0 = apply pass), also before / after downsample blocks
    res_pro_kmax: int = 512
    res_pro_down: bool = True
    res_pro_dual: bool = True
    # bn1 + ReLU inside the 56x56 halo kernels: 1 forward + write-through, 0 apply
    # pass (the weight gradient transforming its own halo as well, a1 never
    # stored, measured slower -- 13,310-13,345 img/s, profiles/r03b_halo_pro_ab.txt
    # -- and is not an engine option)
    halo_pro: int = 1
    # BN-backward apply fused into 1x1 data-gradient GEMMs (1 write-through, 2 both
    # operands, 3 = bn3: dgrad prologue without write-through + the Gram-fold weight
    # gradient, dc3 never stored; 0 own pass) up to this many channels; bn1 too
    # (measured slower)
    bn_bwd_fuse: int = 3
    bn_bwd_fuse_kmax: int = 512
    bn_bwd_fuse_bn1: bool = False

    @classmethod
    def from_env(cls) -> "EngineOptions":
        o = cls()
        spec = os.environ.get("KDL_ENGINE", "")
        for item in filter(None, (x.strip() for x in spec.split(","))):
            key, _, val = item.partition("=")
            f = {x.name: x for x in dataclasses.fields(cls)}.get(key)
            if f is None:
                raise ValueError(f"KDL_ENGINE: unknown option {key!r} (known: {[x.name for x in dataclasses.fields(cls)]})")
            typ = type(getattr(o, key))
            setattr(o, key, (val.lower() in ("1", "true", "on")) if typ is bool else typ(val))
        return o


class ResNetEngine:
    """Hand-scheduled training step of a ``ResNet`` built from ``Bottleneck``s.

    ``grad_view(param)`` must return the tensor that receives ``param``'s
    gradient (a view of the flat gradient buffer); ``on_ready(param)`` is
    called once that gradient is final (DP bucket launch)."""

    def __init__(self, model: ResNet, backend: str = "auto", grad_view=None, on_ready=None,
                 options: EngineOptions | None = None, side=None):
        self.model = model
        p = next(model.parameters())
        self.dev = p.device
        if backend == "auto":
            backend = "hip" if self.dev.type == "cuda" else "torch"
        o = self.opts = options or EngineOptions.from_env()
        self.K = HipKernels(self.dev, fuse_fin=o.bn_fin != "kernel") if backend == "hip" else TorchKernels(self.dev)
        self.grad_view = grad_view or self._own_grad
        self.on_ready = on_ready or (lambda prm: None)
        self.bn = {}
        for m in model.modules():
            if isinstance(m, BNAct):
                st = BNState(m, self.dev)
                self.K.init_bn(st)
                self.bn[m] = st
        self.blocks = [b for b in model.layers if isinstance(b, Bottleneck)]
        assert len(self.blocks) == len(model.layers), "engine supports Bottleneck stacks only"
        self._wt_ptrs = None
        self._wt_buf = {}
        # 3x3 forward convs, data and weight gradients on the kdl implicit-GEMM /
        # halo / sub-pixel kernels (per-layer A/B vs MIOpen:
        # profiles/r02_igemm_v1_vs_reg_vs_miopen.jsonl, r02_wgrad_dma_vs_reg_vs_miopen.jsonl,
        # r02_dgrad_s2_vs_miopen.jsonl): their operand chunks are 64 channels wide
        if self.K.name == "hip" and not all(b.conv2.in_channels % 64 == 0 and b.conv2.out_channels % 64 == 0
                                            for b in self.blocks):
            raise ValueError("the HIP engine's 3x3 kernels need channel counts that are multiples of 64 "
                             "(use backend='torch' or the autograd model for other widths)")
        # Weight gradients on a second HIP stream (default; EngineOptions.side = False
        # turns it off -- 10.7k -> 11.3k img/s at batch 256, profiles/): a wgrad
        # depends only on its layer's output gradient and saved input, and nothing
        # in the rest of backward reads it, so it runs concurrently with the next
        # layers' BN-backward / data-gradient kernels on the main stream.  The
        # BN workspace keeps forward (prologue) and backward coefficients apart
        # (csrc/bn_act.hip ws_bcoef) so a wgrad's recomputed BN never races the
        # main stream's backward finalize of the same BN.
        # BN-backward apply passes of bn3 / downsample BN / bn1 fused into their
        # 1x1 data-gradient GEMMs (csrc/conv1x1.hip PRO_BWD); bn_bwd_fuse = 0: separate passes
        # (1: dgrad A prologue + write-through; 2: dgrad A prologue + weight-gradient G
        # prologue, never materialised), for BNs of at most bn_bwd_fuse_kmax channels.
        # Per-layer A/B (profiles/r03_bn_bwd_fuse_layers.jsonl, apply + dgrad vs fused
        # dgrad, uncontended): mode 1 wins where the dgrad has ONE output-channel tile
        # -- bn3 / downsample BN into conv3 / downsample dgrads at K = 4C <= 512
        # (stage 1: 390 -> 287 us, down 371 -> 258; stage 2: 192 -> 157); it loses on
        # conv1's dgrad (N = 4C output tiles each re-transform the A tile) and at
        # K >= 1024 (the register-staged loop vs the LDS-DMA one: 88 -> 138 us); the
        # G prologue (mode 2) loses to reading the written-through tensor (106 -> 354 us).
        # Mode 3 (default): mode 1 for every BN except a block's bn3, whose conv3
        # weight gradient is the Gram fold diag(k) g^T a2 + diag(c1) W3 (a2^T a2) +
        # c0 1^T a2 (HipKernels.wgrad_gram) -- dc3, a 4C-channel tensor, is neither
        # written by the dgrad nor read by the wgrad: 13,841 -> 13,900-13,960 img/s,
        # main-stream busy 18.21 -> 17.80 ms/step (profiles/r05_gram_fold_ab.txt).
        # downsample branch conv of the forward on the side stream (down_side = False: in
        # line): 13,333-13,347 vs 13,252-13,279 img/s, profiles/r03b_fwd_down_side_ab.txt
        self.down_side = o.down_side
        # the closing BN3 + residual + ReLU of a block whose successor has no
        # downsample branch, applied in the successor's conv1 A staging and written
        # through (csrc/conv1x1.hip PRO_RES) instead of its own pass, up to
        # res_pro_kmax channels (the register-staged loop; beyond, the LDS-DMA
        # GEMM + apply pass); 0: apply pass
        self.res_pro_kmax = o.res_pro_kmax
        # ... also before a downsample block (its conv1 then runs before the side-stream
        # downsample conv, which reads the written-through block output)
        self.res_pro_down = o.res_pro_down
        # ... and after a downsample block: the residual is the downsample branch's BN
        # output, applied in the same prologue (PRO_RES2)
        self.res_pro_dual = o.res_pro_dual
        # bn1 + ReLU of the stride-1 56x56 3x3 convs applied inside the halo kernels,
        # which stage the input halo in LDS and transform it there (halo_pro):
        # 1 = the forward conv does, writing a1 = relu(B1(c1)) through for the weight
        # gradient (no apply pass); 0 = apply pass
        if o.halo_pro not in (0, 1):
            raise ValueError(f"KDL_ENGINE halo_pro={o.halo_pro}: 0 (apply pass) or 1 (halo prologue)")
        self.halo_pro = o.halo_pro
        self.fuse_bwd = o.bn_bwd_fuse
        self.fuse_kmax = o.bn_bwd_fuse_kmax
        self.fuse_bn1 = o.bn_bwd_fuse_bn1
        self.side = None
        if self.K.name == "hip" and o.side:
            from kubedl_amd.ops.streams import side_stream
            # (``side``: a stream the caller created -- and ran a kernel on -- before
            # anything else claimed the hardware queues; ResNetTrainer does)
            self.side = side if side is not None else side_stream(self.dev, o.side_prio)  # (ops/streams.py)
            # overlapped with the main stream, the 1x1 weight gradients gain from 256x256
            # tiles too (fewer, heavier side-stream blocks; csrc/conv1x1.hip wgrad_tiles)
            self.K.ext.set_wgrad_big(2)

    def _refresh_wt(self) -> None:
        """HIP path: the data-gradient GEMMs' B operands -- W^T of every 1x1 conv
        and the tap-reversed per-tap transpose Wd[Cin][3][3][Cout] of every
        stride-1 3x3 conv -- in ONE batched-transpose launch per step
        (csrc/multi_tensor.hip), instead of a copy kernel per conv.  The tile
        table is static while the parameter storage is."""
        if self.K.name != "hip":
            return
        convs = [c for b in self.blocks for c in (b.conv1, b.conv3, b.down_conv) if c is not None]
        c3s = [b.conv2 for b in self.blocks if b.conv2.stride[0] == 1]
        c3s2 = [b.conv2 for b in self.blocks if b.conv2.stride[0] == 2]
        ptrs = tuple(c.weight.data_ptr() for c in convs + c3s + c3s2)
        if ptrs != self._wt_ptrs:
            rows = []
            self._wt_buf = {}
            for c in convs:
                w = c.weight.view(c.out_channels, -1)
                co, ci = w.shape
                wt = torch.empty(ci, co, dtype=w.dtype, device=w.device)
                self._wt_buf[c] = wt
                for r0 in range(0, co, 64):
                    for c0 in range(0, ci, 64):
                        rows.append((w.data_ptr(), wt.data_ptr(), co | (ci << 32), r0 | (c0 << 32), ci | (co << 32)))
            for c in c3s:
                w = c.weight  # [Cout, Cin, 3, 3] channels_last = OHWI in memory
                co, ci = w.shape[:2]
                assert w.is_contiguous(memory_format=torch.channels_last)
                wd = torch.empty(ci, co, 3, 3, dtype=w.dtype, device=w.device).contiguous(
                    memory_format=torch.channels_last)
                self._wt_buf[c] = wd
                esz = w.element_size()
                for tap in range(9):
                    for r0 in range(0, co, 64):
                        for c0 in range(0, ci, 64):
                            rows.append((w.data_ptr() + tap * ci * esz, wd.data_ptr() + (8 - tap) * co * esz,
                                         co | (ci << 32), r0 | (c0 << 32), (9 * ci) | ((9 * co) << 32)))
            for c in c3s2:  # class-major [Cin][9 Cout] of the stride-2 dgrad (ops/conv.py CLASS_TAPS)
                w = c.weight
                co, ci = w.shape[:2]
                assert w.is_contiguous(memory_format=torch.channels_last)
                ball = torch.empty(ci, 9 * co, dtype=w.dtype, device=w.device)
                self._wt_buf[c] = ball
                esz = w.element_size()
                for pos, (r, s) in enumerate(S2_TAPS):
                    for r0 in range(0, co, 64):
                        for c0 in range(0, ci, 64):
                            rows.append((w.data_ptr() + (3 * r + s) * ci * esz, ball.data_ptr() + pos * co * esz,
                                         co | (ci << 32), r0 | (c0 << 32), (9 * ci) | ((9 * co) << 32)))
            self._wt_table = torch.tensor(rows, dtype=torch.int64).to(self.dev)
            self._wt_ptrs = ptrs
        self.K.ext.transpose_tiles(self._wt_table)

    def _ball(self, conv):
        """B operand of the stride-2 3x3 data gradient: the class-major
        [Cin][9 Cout] regrouping (HIP path) or the weight itself (torch path)."""
        if self.K.name != "hip":
            return conv.weight
        ball = self._wt_buf.get(conv)
        return ball if ball is not None else s2_dgrad_weights(conv.weight)

    def _wd(self, conv):
        """Data-gradient weight of a stride-1 3x3 conv: flip(W, taps) with Cin/Cout swapped."""
        wd = self._wt_buf.get(conv)
        if wd is not None:
            return wd
        return conv.weight.flip(2, 3).transpose(0, 1)

    @staticmethod
    def _own_grad(prm):
        if prm.grad is None:
            prm.grad = torch.zeros_like(prm)
        return prm.grad

    def _g(self, prm):
        return self.grad_view(prm)

    def _on_side(self, *tensors):
        """Context for a weight-gradient launch: on the side stream (ordered after
        everything the main stream has issued so far) when enabled.  Operands
        produced on the main stream are marked as in use by the side stream so
        the caching allocator does not hand their memory to the main stream
        before the side stream is done with them."""
        if self.side is None:
            return contextlib.nullcontext()
        self.side.wait_stream(torch.cuda.current_stream(self.dev))
        for t in tensors:
            t.record_stream(self.side)
        return torch.cuda.stream(self.side)

    def _fin_descs(self) -> None:
        """HIP path: every conv BN's finalize descriptor (csrc/bn_fin.h) -- written
        once, and again only if the gradient buffer moved."""
        if self.K.name != "hip" or not self.K.fuse_fin:
            return
        sts = [st for mod, st in self.bn.items() if mod is not self.model.bn1]
        sig = tuple(t.data_ptr() for t in self._bn_grads(sts[0])) + (sts[0].ws.data_ptr(),)
        if sig != getattr(self, "_fin_sig", None):
            for st in sts:
                self.K.fin_desc(st, *self._bn_grads(st))
            self._fin_sig = sig

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def forward(self, x: torch.Tensor):
        K, m = self.K, self.model
        self._fin_descs()
        self._wt_evt = None
        if self.side is not None and K.name == "hip":
            # the data-gradient weight transposes (~0.1 ms, one launch) run on the
            # side stream under the forward pass instead of heading the backward;
            # ordered after everything issued so far (last step's optimizer update)
            self.side.wait_stream(torch.cuda.current_stream(self.dev))
            with torch.cuda.stream(self.side):
                self._refresh_wt()
                self._wt_evt = torch.cuda.Event()
                self._wt_evt.record(self.side)
        st0 = self.bn[m.bn1]
        c0, gemm_stats = K.stem_conv(x, m.conv1.weight, st0)
        x1, idx = K.stem_fwd(c0, st0, gemm_stats)
        saved = []
        cur = x1
        pend = None  # (c3, st3, residual, mbits) of a closing apply deferred into this block's conv1
        nb = len(self.blocks)
        for bi, blk in enumerate(self.blocks):
            s = blk.conv2.stride[0]
            st1, st2, st3 = self.bn[blk.bn1], self.bn[blk.bn2], self.bn[blk.bn3]
            n, _, h, w = cur.shape
            down_evt = None
            c1 = None
            if pend is not None:
                # cur is written by this conv1 (the previous block's closing apply), so
                # it runs before the downsample branch that reads cur is issued
                c1 = K.conv1x1_fwd_res(pend[0], blk.conv1.weight.view(blk.conv1.out_channels, -1), pend[1], pend[2],
                                       cur, pend[3], st1, dual=pend[4])
                pend = None
            if blk.down_conv is not None and self.down_side and self.side is not None:
                # the downsample branch needs only the block input: on the side stream
                # (idle in the forward but for the weight transposes), concurrent with
                # conv1 -> conv2 -> conv3; the BN-apply that joins the branches waits on it
                std_ = self.bn[blk.down_bn]
                main = torch.cuda.current_stream(self.dev)
                with self._on_side(cur):
                    hd = (h - 1) // blk.down_conv.stride[0] + 1
                    wd_ = (w - 1) // blk.down_conv.stride[0] + 1
                    cd = K.conv1x1_fwd(cur, blk.down_conv.weight.view(blk.down_conv.out_channels, -1),
                                       blk.down_conv.stride[0], None, std_)
                    K.bn_finalize(std_, n * hd * wd_, gemm_shift=True)
                    down_evt = torch.cuda.Event()
                    down_evt.record(self.side)
                cd.record_stream(main)
            if c1 is None:
                c1 = K.conv1x1_fwd(cur, blk.conv1.weight.view(blk.conv1.out_channels, -1), 1, None, st1)
            K.bn_finalize(st1, n * h * w, gemm_shift=True)
            if self._halo_pro_ok(c1, s):
                # the conv applies B1 + ReLU to its input halo (csrc/halo3x3.hip) and
                # writes a1 through for the weight gradient
                a1 = torch.empty_like(c1)
                c2 = K.conv3x3_fwd(c1, blk.conv2.weight, s, st2, pro=st1, aout=a1)
                ho, wo = c2.shape[-2:]
                K.bn_finalize(st2, n * ho * wo, gemm_shift=True)
            else:
                a1, _ = K.bn_apply(c1, st1, relu=True)
                # implicit GEMM + B2 statistics in the epilogue (shift = running mean)
                c2 = K.conv3x3_fwd(a1, blk.conv2.weight, s, st2)
                ho, wo = c2.shape[-2:]
                K.bn_finalize(st2, n * ho * wo, gemm_shift=True)
            c3 = K.conv1x1_fwd(c2, blk.conv3.weight.view(blk.conv3.out_channels, -1), 1, st2, st3)
            K.bn_finalize(st3, n * ho * wo, gemm_shift=True)
            # the closing apply deferred into the successor's conv1 (which writes out / mbits)?
            defer = bi + 1 < nb and c3.shape[1] <= self.res_pro_kmax and \
                (self.res_pro_down or self.blocks[bi + 1].down_conv is None) and \
                (blk.down_conv is None or self.res_pro_dual)
            if down_evt is not None:
                torch.cuda.current_stream(self.dev).wait_event(down_evt)
            elif blk.down_conv is not None:
                std_ = self.bn[blk.down_bn]
                cd = K.conv1x1_fwd(cur, blk.down_conv.weight.view(blk.down_conv.out_channels, -1),
                                   blk.down_conv.stride[0], None, std_)
                K.bn_finalize(std_, n * ho * wo, gemm_shift=True)
            else:
                cd = None
            if defer:
                out = torch.empty_like(c3)
                mbits = K.relu_mask_like(c3)
                # (residual: the block input, or the downsample branch's BN input + its BN)
                pend = (c3, st3, cur, mbits, None) if cd is None else (c3, st3, cd, mbits, std_)
            elif cd is not None:
                out, mbits = K.bn_apply(c3, st3, relu=True, other=(cd, std_), want_mask=True)
            else:
                out, mbits = K.bn_apply(c3, st3, relu=True, res=cur, want_mask=True)
            saved.append((cur, c1, a1, c2, c3, cd, mbits))
            cur = out
        self._saved = (x, c0, idx, saved, cur)
        return cur

    # ------------------------------------------------------------------ step
    def forward_backward(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """One training forward + backward; returns the (detached) loss."""
        m = self.model
        feat_map = self.forward(x)
        n, c, h, w = feat_map.shape
        head = getattr(self.K, "head", None)
        if head is not None and self.K.head_ok(feat_map, m.fc.weight, y):
            # csrc/head.hip: pool + fc + softmax CE + their backward, dW / db straight
            # into the gradient buffer (no autograd, no vendor GEMM)
            loss, dfeat = head(feat_map, m.fc.weight, m.fc.bias, y, self._g(m.fc.weight), self._g(m.fc.bias))
            self.on_ready(m.fc.weight)
            self.on_ready(m.fc.bias)
            self.backward(dfeat, h * w)
            return loss
        with torch.enable_grad():  # torch backend / unsupported shapes: the head under autograd
            feat = feat_map.mean((2, 3), dtype=torch.float32).detach().requires_grad_(True)
            fcw = m.fc.weight.detach().requires_grad_(True)
            fcb = m.fc.bias.detach().requires_grad_(True)
            logits = F.linear(feat.to(fcw.dtype), fcw, fcb)
            loss = F.cross_entropy(logits.float(), y)
            dfeat, dfcw, dfcb = torch.autograd.grad(loss, (feat, fcw, fcb))
        with torch.no_grad():
            self._g(m.fc.weight).copy_(dfcw)
            self._g(m.fc.bias).copy_(dfcb)
        self.on_ready(m.fc.weight)
        self.on_ready(m.fc.bias)
        self.backward(dfeat, h * w)
        return loss.detach()

    def _wt(self, conv):
        wt = self._wt_buf.get(conv)
        if wt is not None:
            return wt
        return conv.weight.view(conv.out_channels, -1).t().contiguous()

    def _halo_pro_ok(self, c1, stride) -> bool:
        """B1 + ReLU inside conv2 (forward and weight gradient): the stride-1
        56x56 / 64-channel geometry of the halo kernels (csrc/halo3x3.hip), HIP path."""
        n, c, h, w = c1.shape
        return self.halo_pro > 0 and self.K.name == "hip" and stride == 1 and c == 64 and h == 56 and w == 56

    def _wgrad3x3(self, g, a, stride, weight, pro=None):
        """conv2's weight gradient: the implicit-GEMM / halo kernel writing straight
        into the gradient buffer; ``pro``: ``a`` is the BN input and the operand
        relu(B_pro(a)) (halo kernel prologue)."""
        self.K.wgrad3x3(g, a, stride, self._g(weight), pro=pro)

    def _fuse_mode(self, C: int, bn1: bool = False) -> int:
        """How the BN-backward apply of a C-channel BN reaches its 1x1 consumers:
        0 its own pass; 1 inside the data-gradient GEMM's A staging, written
        through for the weight gradient; 2 inside both GEMMs' operand staging
        (never materialised)."""
        if bn1 and not self.fuse_bn1:
            return 0
        return self.fuse_bwd if C <= self.fuse_kmax else 0

    def _bn_bwd_operand(self, g, x, st, bn1: bool = False, gram: bool = False):
        """(dgrad A, dgrad bpro, wgrad G, wgrad gbpro) for the BN-backward apply
        dc = k g + c1 x + c0 of BN ``st`` (input ``x``) per ``_fuse_mode``; wgrad
        gbpro "gram": the weight gradient folds the apply in (``gram``: a block's
        bn3, whose conv3 input is B2's prologued c2 -- HipKernels.wgrad_gram)."""
        mode = self._fuse_mode(x.shape[1], bn1)
        if mode == 3 and gram:
            return g, (x, st, None), g, "gram"
        if mode == 3:
            mode = 1
        if mode == 0:
            dc, _ = self.K.bn_bwd_apply(g, x, st)
            return dc, None, dc, None
        if mode == 1:
            dc = torch.empty_like(x)
            return g, (x, st, dc), dc, None
        return g, (x, st, None), g, (x, st)

    @staticmethod
    def _side_of(op):
        """Tensors a weight gradient on ``op`` reads (side-stream lifetime)."""
        return (op[2],) if op[3] is None or isinstance(op[3], str) else (op[2], op[3][0])

    def _bn_grads(self, st):
        return self._g(st.mod.weight), self._g(st.mod.bias)

    def _bn_ready(self, st):
        self.on_ready(st.mod.weight)
        self.on_ready(st.mod.bias)

    @torch.no_grad()
    def backward(self, dfeat: torch.Tensor, hw: int) -> None:
        K, m = self.K, self.model
        if getattr(self, "_wt_evt", None) is not None:
            torch.cuda.current_stream(self.dev).wait_event(self._wt_evt)
            self._wt_evt = None
        else:
            self._refresh_wt()
        x, c0, idx, saved, last = self._saved
        nb = len(self.blocks)
        # gradient at the last block's pre-ReLU sum, plus its bn3 sums
        cur_in, c1, a1, c2, c3, cd, mbits = saved[-1]
        lblk = self.blocks[-1]
        g = K.head_mask_reduce(dfeat, hw, mbits, c3, self.bn[lblk.bn3], cd,
                               self.bn[lblk.down_bn] if cd is not None else None)
        for i in range(nb - 1, -1, -1):
            blk = self.blocks[i]
            cur_in, c1, a1, c2, c3, cd, mbits = saved[i]
            st1, st2, st3 = self.bn[blk.bn1], self.bn[blk.bn2], self.bn[blk.bn3]
            n, _, ho, wo = g.shape
            Mo = n * ho * wo
            # bn3 (+ downsample BN) backward: one apply pass over g for both branches
            K.bn_bwd_finalize(st3, Mo, *self._bn_grads(st3))
            self._bn_ready(st3)
            std_ = self.bn[blk.down_bn] if blk.down_bn is not None else None
            if std_ is not None:
                K.bn_bwd_finalize(std_, Mo, *self._bn_grads(std_))
                self._bn_ready(std_)
            if std_ is not None and self._fuse_mode(c3.shape[1]) == 0:
                dc3, dcd = K.bn_bwd_apply(g, c3, st3, cd, std_)  # one pass for both branches
                op3, opd = (dc3, None, dc3, None), (dcd, None, dcd, None)
            else:
                op3 = self._bn_bwd_operand(g, c3, st3, gram=True)
                # a stride-1 downsample conv's input is dense: its weight gradient
                # takes the Gram fold too (the dedicated Gram kernel: 64 / 128 channels)
                # (13,910-13,933 vs 13,848-13,872 img/s, profiles/r05_gram_fold_ab.txt)
                dgram = (std_ is not None and blk.down_conv.stride[0] == 1
                         and (blk.down_conv.in_channels in (64, 128) or K.name != "hip"))
                opd = self._bn_bwd_operand(g, cd, std_, gram=dgram) if std_ is not None else None
            # conv3: dgrad with B2+ReLU mask and B2 sums fused; wgrad with B2+ReLU recomputed
            g2 = K.dgrad_maskx(op3[0], self._wt(blk.conv3), c2, st2, bpro=op3[1])
            with self._on_side(*self._side_of(op3)):
                if op3[3] == "gram":
                    K.wgrad_gram(g, c2, st2, st3, blk.conv3.weight, self._g(blk.conv3.weight))
                else:
                    K.wgrad(op3[2], c2, 1, st2, self._g(blk.conv3.weight), gbpro=op3[3])
            self.on_ready(blk.conv3.weight)
            K.bn_bwd_finalize(st2, Mo, *self._bn_grads(st2))
            self._bn_ready(st2)
            dc2, _ = K.bn_bwd_apply(g2, c2, st2)
            # conv2 (3x3): weight gradient on the kdl kernels (halo / LDS-DMA implicit
            # GEMM, side stream); stride-1 data gradient on the implicit-GEMM or halo
            # kernel with bn1's ReLU mask + backward sums fused
            s = blk.conv2.stride[0]
            if s == 1:
                with self._on_side(dc2):
                    self._wgrad3x3(dc2, a1, 1, blk.conv2.weight)
                self.on_ready(blk.conv2.weight)
                g1 = K.dgrad3x3_maskx(dc2, self._wd(blk.conv2), c1, st1)
                n1, _, h1, w1 = c1.shape
                K.bn_bwd_finalize(st1, n1 * h1 * w1, *self._bn_grads(st1))
            elif s == 2:
                # stride 2: four sub-pixel class GEMMs with bn1's mask + sums fused
                # (no MIOpen, no zero-filled dx, no separate BN-backward reduce pass;
                # an odd input size masks the last sub-pixel row / column)
                with self._on_side(dc2):
                    self._wgrad3x3(dc2, a1, s, blk.conv2.weight)
                self.on_ready(blk.conv2.weight)
                g1 = K.dgrad3x3s2_maskx(dc2, self._ball(blk.conv2), c1, st1)
                n1, _, h1, w1 = c1.shape
                K.bn_bwd_finalize(st1, n1 * h1 * w1, *self._bn_grads(st1))
            else:
                raise NotImplementedError(f"engine: 3x3 stride {s} (Bottleneck strides are 1 or 2)")
            self._bn_ready(st1)
            # bn1 backward apply: its own pass, or (fused) inside conv1's dgrad below
            op1 = self._bn_bwd_operand(g1, c1, st1, bn1=True)
            # conv1 dgrad + identity gradient (+ previous block's mask and BN sums)
            if blk.down_conv is not None:
                ds = blk.down_conv.stride[0]
                eres = K.dgrad_plain(opd[0], self._wt(blk.down_conv), bpro=opd[1])
                res_stride = ds
            else:
                eres, res_stride = g, 1
            if i > 0:
                p_in, p_c1, p_a1, p_c2, p_c3, p_cd, p_mbits = saved[i - 1]
                pblk = self.blocks[i - 1]
                p_std = self.bn[pblk.down_bn] if pblk.down_bn is not None else None
                g_prev = K.dgrad_res(op1[0], self._wt(blk.conv1), eres, res_stride,
                                     (p_mbits, p_c3, self.bn[pblk.bn3], p_cd, p_std), bpro=op1[1])
            else:
                g_prev = K.dgrad_res(op1[0], self._wt(blk.conv1), eres, res_stride, None, bpro=op1[1])
            with self._on_side(*self._side_of(op1), *(self._side_of(opd) if opd is not None else ())):
                K.wgrad(op1[2], cur_in, 1, None, self._g(blk.conv1.weight), gbpro=op1[3])
                if blk.down_conv is not None and opd[3] == "gram":
                    K.wgrad_gram(g, cur_in, None, std_, blk.down_conv.weight, self._g(blk.down_conv.weight))
                elif blk.down_conv is not None:
                    K.wgrad(opd[2], cur_in, blk.down_conv.stride[0], None, self._g(blk.down_conv.weight),
                            gbpro=opd[3])
            self.on_ready(blk.conv1.weight)
            if blk.down_conv is not None:
                self.on_ready(blk.down_conv.weight)
            g = g_prev
        # stem: fused BN + ReLU + max-pool backward, then the 7x7 conv weight gradient
        st0 = self.bn[m.bn1]
        K.stem_backward(g, idx, c0, x, st0, *self._bn_grads(st0), self._g(m.conv1.weight))
        self._bn_ready(st0)
        if self.side is not None:  # the optimizer (and the next forward) read every weight gradient
            torch.cuda.current_stream(self.dev).wait_stream(self.side)
        self.on_ready(m.conv1.weight)
        self._saved = None
