"""BN-apply prologues fused into their conv consumers.

BN + ReLU prologue of the 56x56 halo kernels (csrc/halo3x3.hip PRO): the
forward 3x3 conv and its weight gradient read the BN input c1 and transform
the landed input halo in LDS, relu(c1 * scale + shift), instead of reading a
materialised a1 = bn_apply(c1).  Same fmaf / ReLU / bf16 rounding as the apply
pass, padding pixels stay zero: the outputs match the two-pass path bit for bit
(forward) and up to the fixed-order fp32 slab sums (weight gradient, exact
too since both paths stage identical operands).  Checked against fp32 PyTorch
as well.
"""
import pytest
import torch
import torch.nn.functional as F

from kubedl_amd.models.resnet import BNAct
from kubedl_amd.models.resnet_engine import BNState, HipKernels

pytestmark = pytest.mark.gpu

BATCHES = [2, 5]


def _kern():
    K = HipKernels(torch.device("cuda"))
    K.fuse_fin = False
    return K


def _st(K, C, seed, coef=None):
    g = torch.Generator().manual_seed(seed)
    m = BNAct(C)
    with torch.no_grad():
        m.weight.copy_(torch.rand(C, generator=g) + 0.5)
        m.bias.copy_(torch.rand(C, generator=g) * 0.4 - 0.2)
        m.running_mean.copy_(torch.randn(C, generator=g) * 0.1)
    st = BNState(m.cuda(), torch.device("cuda"))
    K.init_bn(st)
    if coef is not None:
        K.fcoef(st).copy_(coef)
    return st


def _setup(n, seed=0):
    torch.manual_seed(seed)
    K = _kern()
    C = 64
    coef = torch.cat([torch.rand(C) + 0.5, torch.randn(C) * 0.5]).cuda()
    st1 = _st(K, C, seed + 1, coef)
    c1 = torch.randn(n, C, 56, 56, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, C, 3, 3, device="cuda") / 24).bfloat16().contiguous(memory_format=torch.channels_last)
    return K, st1, c1, w, coef


def _a1_ref(c1, coef):
    C = c1.shape[1]
    return torch.relu(c1.float() * coef[:C].view(1, -1, 1, 1) + coef[C:].view(1, -1, 1, 1))


@pytest.mark.parametrize("n", BATCHES)
def test_halo_forward_prologue_matches_apply_pass(n):
    K, st1, c1, w, coef = _setup(n)
    M = n * 56 * 56
    sta, stb = _st(K, 64, 7), _st(K, 64, 7)
    a1, _ = K.bn_apply(c1, st1, relu=True)
    ya = K.conv3x3_fwd(a1, w, 1, sta)
    K.bn_finalize(sta, M, gemm_shift=True)
    a1b = torch.full_like(c1, float("nan"))
    yb = K.conv3x3_fwd(c1, w, 1, stb, pro=st1, aout=a1b)
    K.bn_finalize(stb, M, gemm_shift=True)
    torch.cuda.synchronize()
    assert torch.equal(yb, ya)
    assert torch.equal(a1b, a1)  # the write-through covers every pixel once
    torch.testing.assert_close(stb.save_mean, sta.save_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(stb.save_invstd, sta.save_invstd, rtol=1e-5, atol=1e-6)
    ref = F.conv2d(_a1_ref(c1, coef), w.float(), padding=1)
    err = ((yb.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("n", BATCHES)
def test_halo_wgrad_prologue_matches_apply_pass(n):
    K, st1, c1, w, coef = _setup(n, seed=3)
    g = torch.randn(n, 64, 56, 56, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    a1, _ = K.bn_apply(c1, st1, relu=True)
    dWa = torch.empty_like(w)
    dWb = torch.empty_like(w)
    K.wgrad3x3(g, a1, 1, dWa)
    K.wgrad3x3(g, c1, 1, dWb, pro=st1)
    torch.cuda.synchronize()
    assert torch.equal(dWb, dWa)
    ref = torch.nn.grad.conv2d_weight(_a1_ref(c1, coef), tuple(w.shape), g.float(), padding=1)
    err = ((dWb.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


# ---- the closing BN + residual + ReLU of a block in the next conv1's A staging
# (csrc/conv1x1.hip PRO_RES): conv output, written-through block output and its
# packed ReLU mask are bit-identical to bn_apply(..., want_mask=True) + conv1x1_fwd

RES_SHAPES = [(3, 10, 9, 256, 64), (2, 14, 14, 512, 128), (2, 7, 7, 1024, 256), (4, 8, 8, 256, 128)]


@pytest.mark.parametrize("n,h,w,K4,N1", RES_SHAPES)
def test_residual_prologue_matches_apply_pass(n, h, w, K4, N1):
    torch.manual_seed(11)
    K = _kern()
    coef = torch.cat([torch.rand(K4) + 0.5, torch.randn(K4) * 0.5]).cuda()
    st3 = _st(K, K4, 2, coef)
    nhwc = dict(memory_format=torch.channels_last)
    c3 = torch.randn(n, K4, h, w, device="cuda").bfloat16().contiguous(**nhwc)
    res = torch.randn(n, K4, h, w, device="cuda").bfloat16().contiguous(**nhwc)
    w1 = (torch.randn(N1, K4, device="cuda") / K4 ** 0.5).bfloat16()
    M = n * h * w
    sta, stb = _st(K, N1, 5), _st(K, N1, 5)
    xa, mba = K.bn_apply(c3, st3, relu=True, res=res, want_mask=True)
    ya = K.conv1x1_fwd(xa, w1, 1, None, sta)
    K.bn_finalize(sta, M, gemm_shift=True)
    xb = torch.full_like(c3, float("nan"))
    mbb = torch.full_like(mba, 0x5A)
    yb = K.conv1x1_fwd_res(c3, w1, st3, res, xb, mbb, stb)
    K.bn_finalize(stb, M, gemm_shift=True)
    torch.cuda.synchronize()
    assert torch.equal(xb, xa)
    assert torch.equal(mbb, mba)
    assert torch.equal(yb, ya)
    torch.testing.assert_close(stb.save_mean, sta.save_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(stb.save_invstd, sta.save_invstd, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("n,h,w,K4,N1", [(3, 10, 9, 256, 64), (2, 14, 14, 512, 128), (2, 8, 8, 384, 128)])
def test_dual_residual_prologue_matches_apply_pass(n, h, w, K4, N1):
    """After a downsample block: residual = the downsample branch's BN (PRO_RES2)."""
    torch.manual_seed(12)
    K = _kern()
    st3 = _st(K, K4, 2, torch.cat([torch.rand(K4) + 0.5, torch.randn(K4) * 0.5]).cuda())
    std_ = _st(K, K4, 3, torch.cat([torch.rand(K4) + 0.5, torch.randn(K4) * 0.5]).cuda())
    nhwc = dict(memory_format=torch.channels_last)
    c3 = torch.randn(n, K4, h, w, device="cuda").bfloat16().contiguous(**nhwc)
    cd = torch.randn(n, K4, h, w, device="cuda").bfloat16().contiguous(**nhwc)
    w1 = (torch.randn(N1, K4, device="cuda") / K4 ** 0.5).bfloat16()
    M = n * h * w
    sta, stb = _st(K, N1, 5), _st(K, N1, 5)
    xa, mba = K.bn_apply(c3, st3, relu=True, other=(cd, std_), want_mask=True)
    ya = K.conv1x1_fwd(xa, w1, 1, None, sta)
    K.bn_finalize(sta, M, gemm_shift=True)
    xb = torch.full_like(c3, float("nan"))
    mbb = torch.full_like(mba, 0x5A)
    yb = K.conv1x1_fwd_res(c3, w1, st3, cd, xb, mbb, stb, dual=std_)
    K.bn_finalize(stb, M, gemm_shift=True)
    torch.cuda.synchronize()
    assert torch.equal(xb, xa)
    assert torch.equal(mbb, mba)
    assert torch.equal(yb, ya)
    torch.testing.assert_close(stb.save_mean, sta.save_mean, rtol=1e-5, atol=1e-6)
