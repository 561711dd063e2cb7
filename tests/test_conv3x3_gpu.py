"""3x3 pad-1 convolutions as implicit MFMA GEMMs (csrc/conv1x1.hip, G_CONV3 mode)
vs plain PyTorch fp32 references: forward with the BN+ReLU prologue and the
BN-statistics epilogue, stride-1 data gradient with the mask+BN-sums epilogue,
and the weight gradient with the BN+ReLU prologue recomputed."""
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


def _coef(C):
    return torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.5]).float()


def _pro(x, coef):
    C = x.shape[1]
    return F.relu(x.float() * coef[:C].view(1, C, 1, 1) + coef[C:].view(1, C, 1, 1)).bfloat16().float()


@pytest.mark.parametrize("Cin,Cout,H,W,stride", [(64, 64, 12, 10, 1), (128, 64, 9, 9, 2), (64, 128, 7, 11, 2),
                                                 (256, 256, 6, 6, 1)])
@pytest.mark.parametrize("pro", [False, True])
def test_conv3x3_forward_stats(Cin, Cout, H, W, stride, pro):
    torch.manual_seed(0)
    ext = _ext()
    nb = 3
    x = _nhwc(torch.randn(nb, Cin, H, W, device="cuda").bfloat16())
    w = _nhwc((torch.randn(Cout, Cin, 3, 3, device="cuda") / (3 * Cin ** 0.5)).bfloat16())
    coef = _coef(Cin) if pro else None
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    y = _nhwc(torch.empty(nb, Cout, Ho, Wo, device="cuda", dtype=torch.bfloat16))
    shift = torch.randn(Cout, device="cuda") * 0.1
    acc = torch.zeros(REP * 2 * Cout, device="cuda")
    ext.conv3x3_gemm(x, w, y, nb, H, W, Cin, Cout, stride, coef, 1, shift, acc, None, None, None)
    a = _pro(x, coef) if pro else x.float()
    ref = F.conv2d(a, w.float(), stride=stride, padding=1)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)
    # statistics epilogue: shifted sums of the bf16 output
    yr = _rows(y.float()) - shift
    s = acc.view(REP, 2, Cout).sum(0)
    torch.testing.assert_close(s[0], yr.sum(0), atol=5e-2, rtol=1e-3)
    torch.testing.assert_close(s[1], (yr * yr).sum(0), atol=5e-2, rtol=1e-3)


@pytest.mark.parametrize("Cin,Cout,H,W", [(64, 64, 12, 10), (128, 64, 7, 9), (64, 256, 8, 8)])
def test_conv3x3_dgrad_maskx(Cin, Cout, H, W):
    """dx of a stride-1 3x3 conv = 3x3 conv of dy with the flipped, transposed
    weight; epilogue = the previous BN+ReLU's mask and backward sums."""
    torch.manual_seed(1)
    ext = _ext()
    nb = 2
    dy = _nhwc(torch.randn(nb, Cout, H, W, device="cuda").bfloat16())
    w = _nhwc((torch.randn(Cout, Cin, 3, 3, device="cuda") / (3 * Cin ** 0.5)).bfloat16())
    wd = _nhwc(w.flip(2, 3).transpose(0, 1))  # [Cin][3][3][Cout]
    xbn = _nhwc(torch.randn(nb, Cin, H, W, device="cuda").bfloat16())  # the BN input whose ReLU masks dx
    coef = _coef(Cin)
    mean = torch.randn(Cin, device="cuda") * 0.1
    acc = torch.zeros(REP * 2 * Cin, device="cuda")
    out = _nhwc(torch.empty(nb, Cin, H, W, device="cuda", dtype=torch.bfloat16))
    ext.conv3x3_gemm(dy, wd, out, nb, H, W, Cout, Cin, 1, None, 2, None, acc, xbn, mean, coef)
    dx = torch.nn.grad.conv2d_input(xbn.shape, w.float(), dy.float(), padding=1)
    mask = (xbn.float() * coef[:Cin].view(1, Cin, 1, 1) + coef[Cin:].view(1, Cin, 1, 1)) > 0
    ref = torch.where(mask, dx.bfloat16().float(), torch.zeros_like(dx))
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2)
    g = _rows(out.float())
    s = acc.view(REP, 2, Cin).sum(0)
    torch.testing.assert_close(s[0], g.sum(0), atol=5e-2, rtol=1e-3)
    torch.testing.assert_close(s[1], (g * (_rows(xbn.float()) - mean)).sum(0), atol=5e-2, rtol=1e-3)


@pytest.mark.parametrize("Cin,Cout,H,W,stride", [(64, 64, 12, 10, 1), (128, 64, 9, 9, 2), (64, 128, 28, 27, 1),
                                                 (256, 128, 7, 7, 1)])
@pytest.mark.parametrize("pro", [False, True])
def test_conv3x3_wgrad(Cin, Cout, H, W, stride, pro):
    torch.manual_seed(2)
    ext = _ext()
    nb = 4
    x = _nhwc(torch.randn(nb, Cin, H, W, device="cuda").bfloat16())
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    dy = _nhwc(torch.randn(nb, Cout, Ho, Wo, device="cuda").bfloat16())
    coef = _coef(Cin) if pro else None
    M = nb * Ho * Wo
    ws = torch.empty(ext.conv1x1_wgrad_splits(M, Cout, 9 * Cin) * Cout * 9 * Cin, device="cuda")
    dW = _nhwc(torch.empty(Cout, Cin, 3, 3, device="cuda", dtype=torch.bfloat16))
    ext.conv3x3_wgrad(dy, x, coef, ws, dW, 1.0, nb, H, W, Cin, Cout, stride)
    a = _pro(x, coef) if pro else x.float()
    ref = torch.nn.grad.conv2d_weight(a, (Cout, Cin, 3, 3), dy.float(), stride=stride, padding=1)
    scale = ref.abs().max().item()
    torch.testing.assert_close(dW.float() / scale, ref / scale, atol=2e-2, rtol=2e-2)
