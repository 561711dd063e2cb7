"""LDS-DMA GEMM main loop (csrc/igemm.hip) vs plain PyTorch fp32 references.

The core is forced on (``set_gemm_core(1)``) for every call here, so each
epilogue, each A-row gather mode and every tile config is exercised on it --
including M tails, N = 64..512, the 3x3 implicit GEMM with padding taps
served by out-of-bounds buffer loads, and stride 2.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

REP = 32


def _ext():
    from kubedl_amd.ops import _ext
    return _ext.load()


@pytest.fixture(autouse=True, params=[0, 1, 2, 3, 4])
def dma_core(request):
    ext = _ext()
    old = ext.get_gemm_core()
    ext.set_gemm_core(1)
    ext.set_igemm_cfg(request.param)  # a config whose BN does not divide N falls back to the by-shape pick
    yield request.param
    ext.set_igemm_cfg(-1)
    ext.set_gemm_core(old)


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _rows(t):
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _gemm(A, W, C, M, N, K, **kw):
    args = dict(Hout=0, Wout=0, Hin=0, Win=0, stride=1, pro_coef=None, epi=0, shift=None, acc=None, ex=None,
                emean=None, ecoef=None, eres=None, res_stride=1, res_H=0, res_W=0, ebits=None, ex2=None,
                emean2=None, acc2=None)
    args.update(kw)
    _ext().conv1x1_gemm(A, W, C, M, N, K, args["Hout"], args["Wout"], args["Hin"], args["Win"], args["stride"],
                        args["pro_coef"], args["epi"], args["shift"], args["acc"], args["ex"], args["emean"],
                        args["ecoef"], args["eres"], args["res_stride"], args["res_H"], args["res_W"], args["ebits"],
                        args["ex2"], args["emean2"], args["acc2"])


@pytest.mark.parametrize("M,N,K", [(1000, 64, 64), (777, 128, 512), (4096, 256, 1024), (300, 512, 2048),
                                   (2500, 256, 2304)])
def test_dma_plain(M, N, K):
    torch.manual_seed(0)
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    C = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    _gemm(A, W, C, M, N, K)
    ref = A.float() @ W.float().t()
    torch.testing.assert_close(C.float(), ref, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("stride", [1, 2])
def test_dma_strided_stats(stride):
    torch.manual_seed(1)
    nb, H, Wd, N, K = 3, 14, 10, 256, 512
    x = _nhwc(torch.randn(nb, K, H, Wd, device="cuda").bfloat16())
    w = (torch.randn(N, K, 1, 1, device="cuda") / K ** 0.5).bfloat16()
    shift = torch.randn(N, device="cuda")
    Ho, Wo = (H - 1) // stride + 1, (Wd - 1) // stride + 1
    M = nb * Ho * Wo
    y = _nhwc(torch.empty(nb, N, Ho, Wo, device="cuda", dtype=torch.bfloat16))
    ws = torch.zeros(_ext().bn_workspace_floats(N), device="cuda")
    _gemm(x, w, y, M, N, K, Hout=Ho, Wout=Wo, Hin=H, Win=Wd, stride=stride, epi=1, shift=shift, acc=ws)
    ref = F.conv2d(x.float(), w.float(), stride=stride)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)
    acc = ws[:REP * 2 * N].view(REP, 2, N).sum(0).double()
    yr = _rows(y).double() - shift.double()
    torch.testing.assert_close(acc[0], yr.sum(0), atol=1e-2 * M ** 0.5, rtol=1e-3)
    torch.testing.assert_close(acc[1], (yr * yr).sum(0), atol=1e-2 * M ** 0.5, rtol=1e-3)


def test_dma_dgrad_maskx():
    torch.manual_seed(2)
    M, N, K = 3000, 256, 1024
    dy = torch.randn(M, K, device="cuda").bfloat16()
    wt = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    x = torch.randn(M, N, device="cuda").bfloat16()
    coef = torch.cat([torch.rand(N, device="cuda") + 0.5, torch.randn(N, device="cuda")]).float()
    mean = torch.randn(N, device="cuda")
    ws = torch.zeros(_ext().bn_workspace_floats(N), device="cuda")
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    _gemm(dy, wt, out, M, N, K, epi=2, ex=x, emean=mean, ecoef=coef, acc=ws)
    g = (dy.float() @ wt.float().t()).bfloat16().float()
    g = torch.where((x.float() * coef[:N] + coef[N:]) > 0, g, torch.zeros_like(g))
    torch.testing.assert_close(out.float(), g, atol=3e-2, rtol=3e-2)
    acc = ws[:REP * 2 * N].view(REP, 2, N).sum(0).double()
    torch.testing.assert_close(acc[0], g.double().sum(0), atol=0.5, rtol=1e-2)
    torch.testing.assert_close(acc[1], (g.double() * (x.double() - mean.double())).sum(0), atol=0.5, rtol=1e-2)


@pytest.mark.parametrize("res_stride,with_x2", [(1, False), (2, True)])
def test_dma_dgrad_resbits(res_stride, with_x2):
    torch.manual_seed(3)
    nb, H, Wd, N, K = 2, 8, 6, 256, 512
    M = nb * H * Wd
    dy = torch.randn(M, K, device="cuda").bfloat16()
    wt = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    Ho, Wo = (H - 1) // res_stride + 1, (Wd - 1) // res_stride + 1
    res = torch.randn(nb * Ho * Wo, N, device="cuda").bfloat16()
    x = torch.randn(M, N, device="cuda").bfloat16()
    x2 = torch.randn(M, N, device="cuda").bfloat16() if with_x2 else None
    bits = torch.randint(0, 256, (M, N // 8), device="cuda", dtype=torch.uint8)
    mean, mean2 = torch.randn(N, device="cuda"), torch.randn(N, device="cuda")
    nws = _ext().bn_workspace_floats(N)
    ws, ws2 = torch.zeros(nws, device="cuda"), torch.zeros(nws, device="cuda")
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    _gemm(dy, wt, out, M, N, K, epi=3, ex=x, emean=mean, acc=ws, eres=res, res_stride=res_stride, res_H=H, res_W=Wd,
          ebits=bits, ex2=x2, emean2=mean2 if with_x2 else None, acc2=ws2 if with_x2 else None)
    g = (dy.float() @ wt.float().t()).bfloat16().float()
    r = torch.zeros(nb, H, Wd, N, device="cuda")
    r[:, ::res_stride, ::res_stride, :] = res.float().view(nb, Ho, Wo, N)
    g = (g + r.view(M, N)).bfloat16().float()
    m = ((bits.unsqueeze(-1) >> torch.arange(8, device="cuda", dtype=torch.uint8)) & 1).view(M, N).bool()
    g = torch.where(m, g, torch.zeros_like(g))
    torch.testing.assert_close(out.float(), g, atol=3e-2, rtol=3e-2)
    acc = ws[:REP * 2 * N].view(REP, 2, N).sum(0).double()
    torch.testing.assert_close(acc[0], g.double().sum(0), atol=0.3, rtol=1e-2)
    torch.testing.assert_close(acc[1], (g.double() * (x.double() - mean.double())).sum(0), atol=0.3, rtol=1e-2)
    if with_x2:
        acc2 = ws2[:REP * 2 * N].view(REP, 2, N).sum(0).double()
        torch.testing.assert_close(acc2[1], (g.double() * (x2.double() - mean2.double())).sum(0), atol=0.3,
                                   rtol=1e-2)


@pytest.mark.parametrize("Cin,Cout,H,W,stride", [(64, 64, 12, 10, 1), (128, 128, 9, 9, 2), (64, 256, 7, 11, 2),
                                                 (256, 256, 6, 6, 1), (128, 512, 7, 7, 1)])
def test_dma_conv3x3_forward_stats(Cin, Cout, H, W, stride):
    torch.manual_seed(4)
    ext = _ext()
    nb = 3
    x = _nhwc(torch.randn(nb, Cin, H, W, device="cuda").bfloat16())
    w = _nhwc((torch.randn(Cout, Cin, 3, 3, device="cuda") / (3 * Cin ** 0.5)).bfloat16())
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    y = _nhwc(torch.empty(nb, Cout, Ho, Wo, device="cuda", dtype=torch.bfloat16))
    shift = torch.randn(Cout, device="cuda") * 0.1
    acc = torch.zeros(REP * 2 * Cout, device="cuda")
    ext.conv3x3_gemm(x, w, y, nb, H, W, Cin, Cout, stride, None, 1, shift, acc, None, None, None)
    ref = F.conv2d(x.float(), w.float(), stride=stride, padding=1)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)
    yr = _rows(y.float()) - shift
    s = acc.view(REP, 2, Cout).sum(0)
    torch.testing.assert_close(s[0], yr.sum(0), atol=5e-2, rtol=1e-3)
    torch.testing.assert_close(s[1], (yr * yr).sum(0), atol=5e-2, rtol=1e-3)


@pytest.mark.parametrize("Cin,Cout,H,W", [(64, 64, 12, 10), (256, 128, 7, 9)])
def test_dma_conv3x3_dgrad_maskx(Cin, Cout, H, W):
    torch.manual_seed(5)
    ext = _ext()
    nb = 2
    dy = _nhwc(torch.randn(nb, Cout, H, W, device="cuda").bfloat16())
    w = _nhwc((torch.randn(Cout, Cin, 3, 3, device="cuda") / (3 * Cin ** 0.5)).bfloat16())
    wd = _nhwc(w.flip(2, 3).transpose(0, 1))
    xbn = _nhwc(torch.randn(nb, Cin, H, W, device="cuda").bfloat16())
    coef = torch.cat([torch.rand(Cin, device="cuda") + 0.5, torch.randn(Cin, device="cuda") * 0.5]).float()
    mean = torch.randn(Cin, device="cuda") * 0.1
    acc = torch.zeros(REP * 2 * Cin, device="cuda")
    out = _nhwc(torch.empty(nb, Cin, H, W, device="cuda", dtype=torch.bfloat16))
    ext.conv3x3_gemm(dy, wd, out, nb, H, W, Cout, Cin, 1, None, 2, None, acc, xbn, mean, coef)
    dx = torch.nn.grad.conv2d_input(xbn.shape, w.float(), dy.float(), padding=1)
    mask = (xbn.float() * coef[:Cin].view(1, Cin, 1, 1) + coef[Cin:].view(1, Cin, 1, 1)) > 0
    ref = torch.where(mask, dx.bfloat16().float(), torch.zeros_like(dx))
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2)
