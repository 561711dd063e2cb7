"""csrc/halo3x3.hip (3x3 stride-1 conv with an LDS-resident input halo) at the
geometry it serves -- 56x56 with Cin 64 (Cout 64 or 128) -- vs plain
PyTorch fp32: forward with the BN-statistics epilogue and the stride-1 data
gradient with the ReLU-mask + BN-backward-sums epilogue; and bitwise agreement
of the halo path with the implicit-GEMM path it replaces where both are exact
(same fp32 accumulation order is not guaranteed, so the agreement is within
bf16 rounding)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

REP = 32


def _ext():
    from kubedl_amd.ops import _ext
    return _ext.load()


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _rows(t):
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


@pytest.fixture(params=[1, 0], ids=["halo", "igemm"])
def halo(request):
    ext = _ext()
    ext.set_halo3x3(request.param)
    yield request.param
    ext.set_halo3x3(1)


@pytest.mark.parametrize("Cin,Cout,H,nb", [(64, 64, 56, 3), (64, 128, 56, 2), (128, 128, 28, 2)])
def test_halo_forward_stats(Cin, Cout, H, nb, halo):
    torch.manual_seed(11)
    ext = _ext()
    x = _nhwc(torch.randn(nb, Cin, H, H, device="cuda").bfloat16())
    w = _nhwc((torch.randn(Cout, Cin, 3, 3, device="cuda") / (3 * Cin ** 0.5)).bfloat16())
    y = _nhwc(torch.empty(nb, Cout, H, H, device="cuda", dtype=torch.bfloat16))
    shift = torch.randn(Cout, device="cuda") * 0.1
    acc = torch.zeros(REP * 2 * Cout, device="cuda")
    ext.conv3x3_gemm(x, w, y, nb, H, H, Cin, Cout, 1, None, 1, shift, acc, None, None, None)
    ref = F.conv2d(x.float(), w.float(), padding=1)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)
    yr = _rows(y.float()) - shift
    s = acc.view(REP, 2, Cout).sum(0)
    torch.testing.assert_close(s[0], yr.sum(0), atol=0.2, rtol=1e-3)
    torch.testing.assert_close(s[1], (yr * yr).sum(0), atol=0.2, rtol=1e-3)


@pytest.mark.parametrize("C,H,nb", [(64, 56, 2), (128, 28, 3)])
def test_halo_dgrad_maskx(C, H, nb, halo):
    torch.manual_seed(12)
    ext = _ext()
    dy = _nhwc(torch.randn(nb, C, H, H, device="cuda").bfloat16())
    w = _nhwc((torch.randn(C, C, 3, 3, device="cuda") / (3 * C ** 0.5)).bfloat16())
    wd = _nhwc(w.flip(2, 3).transpose(0, 1))
    xbn = _nhwc(torch.randn(nb, C, H, H, device="cuda").bfloat16())
    coef = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.5]).float()
    mean = torch.randn(C, device="cuda") * 0.1
    acc = torch.zeros(REP * 2 * C, device="cuda")
    out = _nhwc(torch.empty(nb, C, H, H, device="cuda", dtype=torch.bfloat16))
    ext.conv3x3_gemm(dy, wd, out, nb, H, H, C, C, 1, None, 2, None, acc, xbn, mean, coef)
    dx = torch.nn.grad.conv2d_input(xbn.shape, w.float(), dy.float(), padding=1)
    mask = (xbn.float() * coef[:C].view(1, C, 1, 1) + coef[C:].view(1, C, 1, 1)) > 0
    ref = torch.where(mask, dx.bfloat16().float(), torch.zeros_like(dx))
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2)
    g = _rows(out.float()).double()
    s = acc.view(REP, 2, C).sum(0).double()
    torch.testing.assert_close(s[0], g.sum(0), atol=0.3, rtol=1e-2)
    torch.testing.assert_close(s[1], (g * (_rows(xbn.float()).double() - mean.double())).sum(0), atol=0.3,
                               rtol=1e-2)


def test_halo_matches_implicit_gemm():
    torch.manual_seed(13)
    ext = _ext()
    nb, C, H = 2, 64, 56
    x = _nhwc(torch.randn(nb, C, H, H, device="cuda").bfloat16())
    w = _nhwc((torch.randn(C, C, 3, 3, device="cuda") / (3 * C ** 0.5)).bfloat16())
    outs = []
    for on in (1, 0):
        ext.set_halo3x3(on)
        y = _nhwc(torch.empty(nb, C, H, H, device="cuda", dtype=torch.bfloat16))
        ext.conv3x3_gemm(x, w, y, nb, H, H, C, C, 1, None, 0, None, None, None, None, None)
        outs.append(y.float())
    ext.set_halo3x3(1)
    torch.testing.assert_close(outs[0], outs[1], atol=2e-2, rtol=1e-2)
