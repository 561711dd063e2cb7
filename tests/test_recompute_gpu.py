"""Recompute blocks (csrc/bnfold.hip, csrc/conv1x1.hip PRO_SEG / PRO_RECOMP,
csrc/gemm_epi.h APPLY): a bottleneck whose conv3 output c3 is never stored.

Each fused op is checked against the path it replaces (the engine's own
kernels with c3 materialised) and the fold kernels against fp32 PyTorch:

- statistics-only conv3 + APPLY epilogue == conv3 (STATS) + bn_apply, bit for
  bit (same GEMM accumulation, same fmaf / add / compare sequence);
- RESBITS recomputing c3 in a second accumulator == RESBITS reading the stored
  c3: identical output, BN3 sums equal up to atomic order;
- the BN-folded conv3 data / weight gradients == bn_bwd_apply + dgrad_maskx /
  wgrad within bf16 rounding (the fold moves rounding points, none of them a
  systematic one: k scales g per element, S travels as a bf16 hi + lo pair);
- the fold kernels == their fp32 definitions.
"""
import pytest
import torch

from kubedl_amd.models.resnet import BNAct
from kubedl_amd.models.resnet_engine import BNState, HipKernels, _nhwc_empty

pytestmark = pytest.mark.gpu

SHAPES = [(4, 14, 14, 64), (2, 28, 28, 128), (3, 10, 9, 64)]  # (n, h, w, C); 4C = conv3 outputs


def _kern():
    K = HipKernels(torch.device("cuda"))
    K.fuse_fin = False  # separate finalize launches: no descriptors needed
    return K


def _st(K, C, seed):
    g = torch.Generator().manual_seed(seed)
    m = BNAct(C)
    with torch.no_grad():
        m.weight.copy_(torch.rand(C, generator=g) + 0.5)
        m.bias.copy_(torch.rand(C, generator=g) * 0.4 - 0.2)
        m.running_mean.copy_(torch.randn(C, generator=g) * 0.1)
    m = m.cuda()
    st = BNState(m, torch.device("cuda"))
    K.init_bn(st)
    return st


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _inputs(n, h, w, C, seed=0):
    torch.manual_seed(seed)
    K = _kern()
    st2 = _st(K, C, seed + 1)
    sc = torch.rand(C, device="cuda") + 0.5
    sh = torch.randn(C, device="cuda") * 0.5
    K.fcoef(st2).copy_(torch.cat([sc, sh]))
    st2.save_mean = torch.randn(C, device="cuda") * 0.2
    c2 = _nhwc(torch.randn(n, C, h, w, device="cuda").bfloat16())
    w3 = (torch.randn(4 * C, C, device="cuda") / C ** 0.5).bfloat16()
    res = _nhwc(torch.randn(n, 4 * C, h, w, device="cuda").bfloat16())
    return K, st2, c2, w3, res


@pytest.mark.parametrize("n,h,w,C", SHAPES)
def test_stats_pass_and_apply_epilogue_match_stored_path(n, h, w, C):
    K, st2, c2, w3, res = _inputs(n, h, w, C)
    M = n * h * w
    sta, stb = _st(K, 4 * C, 7), _st(K, 4 * C, 7)
    c3 = K.conv1x1_fwd(c2, w3, 1, st2, sta)
    K.bn_finalize(sta, M, gemm_shift=True)
    out_a, mb_a = K.bn_apply(c3, sta, relu=True, res=res, want_mask=True)
    K.conv1x1_stats(c2, w3, st2, stb)
    K.bn_finalize(stb, M, gemm_shift=True)
    torch.cuda.synchronize()
    torch.testing.assert_close(stb.save_mean, sta.save_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(stb.save_invstd, sta.save_invstd, rtol=1e-5, atol=1e-6)
    K.fcoef(stb).copy_(K.fcoef(sta))  # same coefficients: the apply must be bit-identical
    out_b, mb_b = K.conv1x1_apply(c2, w3, st2, stb, res)
    torch.cuda.synchronize()
    assert torch.equal(out_b, out_a)
    assert torch.equal(mb_b, mb_a)


@pytest.mark.parametrize("n,h,w,C", SHAPES)
def test_resbits_recompute_matches_stored_c3(n, h, w, C):
    K, st2, c2, w3, res = _inputs(n, h, w, C, seed=3)
    M = n * h * w
    st3 = _st(K, 4 * C, 11)
    c3 = K.conv1x1_fwd(c2, w3, 1, st2, st3)
    K.bn_finalize(st3, M, gemm_shift=True)
    _, mbits = K.bn_apply(c3, st3, relu=True, res=res, want_mask=True)
    C1 = 2 * C  # the next block's conv1 width (any multiple of 64)
    dc1 = _nhwc(torch.randn(n, C1, h, w, device="cuda").bfloat16())
    wt = (torch.randn(4 * C, C1, device="cuda") / C1 ** 0.5).bfloat16()  # W1^T [Cin = 4C, C1]
    eres = _nhwc(torch.randn(n, 4 * C, h, w, device="cuda").bfloat16())
    outs, sums = [], []
    for rc in (None, (c2, w3, st2)):
        st = _st(K, 4 * C, 11)
        st.save_mean, st.save_invstd = st3.save_mean.clone(), st3.save_invstd.clone()
        prev = (mbits, None if rc else c3, st, None, None)
        outs.append(K.dgrad_res(dc1, wt, eres, 1, prev, recomp=rc))
        dg, db = torch.empty(4 * C, device="cuda"), torch.empty(4 * C, device="cuda")
        K.bn_bwd_finalize(st, M, dg, db)
        sums.append((dg, db))
    torch.cuda.synchronize()
    assert torch.equal(outs[1], outs[0])
    for a, b in zip(sums[1], sums[0]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4 * (b.abs().max().item() + 1e-6))


def _bwd_setup(n, h, w, C, seed):
    K, st2, c2, w3, res = _inputs(n, h, w, C, seed=seed)
    M = n * h * w
    st3 = _st(K, 4 * C, 13)
    c3 = K.conv1x1_fwd(c2, w3, 1, st2, st3)
    K.bn_finalize(st3, M, gemm_shift=True)
    g = _nhwc(torch.randn(n, 4 * C, h, w, device="cuda").bfloat16())
    # BN3 backward sums and coefficients as the RESBITS epilogue + finalize leave them
    K.bn_bwd_full(g, c3, st3, torch.empty(4 * C, device="cuda"), torch.empty(4 * C, device="cuda"))
    return K, st2, st3, c2, c3, w3, g, M


@pytest.mark.parametrize("n,h,w,C", SHAPES)
def test_fold_kernels_match_fp32_definitions(n, h, w, C):
    K, st2, st3, c2, c3, w3, g, M = _bwd_setup(n, h, w, C, 5)
    N4 = 4 * C
    s2 = torch.empty(C, 2 * C, device="cuda", dtype=torch.bfloat16)
    bias = torch.empty(C, device="cuda")
    K.ext.bn_fold_dgrad(w3, K.bcoef(st3), s2, bias)
    k, c1, c0 = K.bcoef(st3).view(3, N4)
    W = w3.float()
    torch.cuda.synchronize()
    S = W.t() @ (c1[:, None] * W)  # symmetric: S2's row j holds column j
    hi, lo = s2[:, :C].float(), s2[:, C:].float()
    torch.testing.assert_close(hi, S.t().bfloat16().float(), rtol=1e-2, atol=1e-2 * S.abs().max().item())
    # the hi + lo pair carries ~16 significant bits
    assert ((hi + lo) - S.t()).abs().max().item() <= 1e-4 * S.abs().max().item() + 1e-9
    torch.testing.assert_close(bias, W.t() @ c0, rtol=1e-4, atol=1e-5 * (c0.abs().max().item() + 1e-9))
    parts = K.ext.relu_colsum_parts(M)
    part = torch.empty(parts * C, device="cuda")
    pro = K.fcoef(st2)
    K.ext.relu_colsum(c2, pro, C, part)
    K.ext.slab_reduce_f32(part, C, parts)
    a2 = torch.relu(c2.float() * pro[:C].view(1, -1, 1, 1) + pro[C:].view(1, -1, 1, 1))
    torch.cuda.synchronize()
    torch.testing.assert_close(part[:C], a2.sum((0, 2, 3)), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("n,h,w,C", SHAPES)
def test_folded_dgrad_and_wgrad_match_materialised_dc3(n, h, w, C):
    K, st2, st3, c2, c3, w3, g, M = _bwd_setup(n, h, w, C, 9)
    N4 = 4 * C
    # materialised path: dc3 = BN3 backward apply, then the masked dgrad and the wgrad
    sta, stb = _st(K, C, 21), _st(K, C, 21)
    for s in (sta, stb):
        K.fcoef(s).copy_(K.fcoef(st2))
        s.save_mean = st2.save_mean
    dc3, _ = K.bn_bwd_apply(g, c3, st3)
    w3t = w3.t().contiguous()
    g2a = K.dgrad_maskx(dc3, w3t, c2, sta)
    g2b = K.dgrad_folded(g, c2, stb, st3, w3, w3t)
    dWa = torch.empty(N4, C, device="cuda", dtype=torch.bfloat16)
    dWb = torch.empty_like(dWa)
    K.wgrad(dc3, c2, 1, sta, dWa)
    K.wgrad_folded(g, c2, stb, st3, w3, dWb, K.fold_moments(c2, stb))
    sums = []
    for s in (sta, stb):
        dg, db = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
        K.bn_bwd_finalize(s, M, dg, db)
        sums.append((dg, db))
    torch.cuda.synchronize()

    def rel(a, b):
        return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()

    assert rel(g2b, g2a) < 2e-2, rel(g2b, g2a)
    assert rel(dWb, dWa) < 2e-2, rel(dWb, dWa)
    for a, b in zip(sums[1], sums[0]):
        assert rel(a, b) < 3e-2, rel(a, b)
    assert torch.isfinite(g2b.float()).all() and torch.isfinite(dWb.float()).all()
