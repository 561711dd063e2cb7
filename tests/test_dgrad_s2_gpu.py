"""Stride-2 3x3 data gradient as four sub-pixel class GEMMs (csrc/igemm.hip
G_DGRAD2, kubedl_amd/ops/conv.py) vs plain PyTorch fp32
``conv2d_input(stride=2, padding=1)``: the PLAIN epilogue, the MASKX epilogue
(bn1's ReLU mask recomputed from its input + the BN backward sums), every
LDS-DMA tile config, and a row count that leaves partial tiles in each class."""
import pytest
import torch
import torch.nn.functional as F

from kubedl_amd.ops.conv import s2_dgrad_weights

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


@pytest.fixture(params=[-1, 0, 1, 2, 3], ids=["pick", "256x256", "256x128", "128x128", "256x64"])
def cfg(request):
    ext = _ext()
    ext.set_igemm_cfg(request.param)
    yield request.param
    ext.set_igemm_cfg(-1)


@pytest.mark.parametrize("Cd,N,Hd,nb", [(128, 128, 28, 2), (256, 256, 14, 2), (512, 512, 7, 3), (128, 64, 5, 3)])
def test_s2_dgrad_plain(Cd, N, Hd, nb, cfg):
    if cfg == 0 and N % 256:
        pytest.skip("256-wide tile needs N % 256 == 0")
    if cfg in (1, 2) and N % 128:
        pytest.skip("128-wide tile needs N % 128 == 0")
    torch.manual_seed(21)
    ext = _ext()
    dy = _nhwc(torch.randn(nb, Cd, Hd, Hd, device="cuda").bfloat16())
    w = _nhwc((torch.randn(Cd, N, 3, 3, device="cuda") / (3 * Cd ** 0.5)).bfloat16())
    dx = _nhwc(torch.full((nb, N, 2 * Hd, 2 * Hd), float("nan"), device="cuda", dtype=torch.bfloat16))
    ext.conv3x3_s2_dgrad(dy, s2_dgrad_weights(w), dx, nb, Hd, Hd, Cd, N, 0, None, None, None, None)
    ref = torch.nn.grad.conv2d_input(dx.shape, w.float(), dy.float(), stride=2, padding=1)
    assert torch.isfinite(dx.float()).all(), "dx pixels left unwritten"
    torch.testing.assert_close(dx.float(), ref, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("C,Hd,nb", [(128, 28, 2), (256, 14, 2), (512, 7, 2)])
def test_s2_dgrad_maskx(C, Hd, nb):
    torch.manual_seed(22)
    ext = _ext()
    dy = _nhwc(torch.randn(nb, C, Hd, Hd, device="cuda").bfloat16())
    w = _nhwc((torch.randn(C, C, 3, 3, device="cuda") / (3 * C ** 0.5)).bfloat16())
    xbn = _nhwc(torch.randn(nb, C, 2 * Hd, 2 * Hd, device="cuda").bfloat16())
    coef = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.5]).float()
    mean = torch.randn(C, device="cuda") * 0.1
    acc = torch.zeros(REP * 2 * C, device="cuda")
    out = _nhwc(torch.empty(nb, C, 2 * Hd, 2 * Hd, device="cuda", dtype=torch.bfloat16))
    ext.conv3x3_s2_dgrad(dy, s2_dgrad_weights(w), out, nb, Hd, Hd, C, C, 2, acc, xbn, mean, coef)
    dx = torch.nn.grad.conv2d_input(xbn.shape, w.float(), dy.float(), stride=2, padding=1)
    mask = (xbn.float() * coef[:C].view(1, C, 1, 1) + coef[C:].view(1, C, 1, 1)) > 0
    ref = torch.where(mask, dx.bfloat16().float(), torch.zeros_like(dx))
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2)
    g = _rows(out.float()).double()
    s = acc.view(REP, 2, C).sum(0).double()
    torch.testing.assert_close(s[0], g.sum(0), atol=0.3, rtol=1e-2)
    torch.testing.assert_close(s[1], (g * (_rows(xbn.float()).double() - mean.double())).sum(0), atol=0.3,
                               rtol=1e-2)


def test_s2_dgrad_weights_match_engine_table():
    """The engine's batched-transpose regrouping equals ops.conv.s2_dgrad_weights."""
    from kubedl_amd.models.resnet import ResNet
    from kubedl_amd.models.resnet_engine import ResNetEngine
    torch.manual_seed(23)
    model = ResNet((1, 1, 1, 1), num_classes=10, width=64).cuda().bfloat16().to(memory_format=torch.channels_last)
    eng = ResNetEngine(model, backend="hip")
    eng._refresh_wt()
    for blk in eng.blocks:
        if blk.conv2.stride[0] == 2:
            torch.testing.assert_close(eng._ball(blk.conv2), s2_dgrad_weights(blk.conv2.weight), atol=0, rtol=0)


@pytest.mark.parametrize("C,Hd", [(128, 28), (256, 14), (512, 7)])
def test_s2_dgrad_maskx_full_batch_writes_every_pixel(C, Hd):
    """ResNet-50 b256 shapes with the output pre-filled with NaN: every pixel is
    written (a zero dy gives exact zeros), and a random dy matches the reference."""
    ext = _ext()
    nb = 256
    torch.manual_seed(24)
    w = _nhwc((torch.randn(C, C, 3, 3, device="cuda") / (3 * C ** 0.5)).bfloat16())
    xbn = _nhwc(torch.randn(nb, C, 2 * Hd, 2 * Hd, device="cuda").bfloat16())
    coef = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.5]).float()
    mean = torch.randn(C, device="cuda") * 0.1
    for zero in (True, False):
        dy = _nhwc(torch.randn(nb, C, Hd, Hd, device="cuda").bfloat16())
        if zero:
            dy.zero_()
        acc = torch.zeros(REP * 2 * C, device="cuda")
        out = _nhwc(torch.full((nb, C, 2 * Hd, 2 * Hd), float("nan"), device="cuda", dtype=torch.bfloat16))
        ext.conv3x3_s2_dgrad(dy, s2_dgrad_weights(w), out, nb, Hd, Hd, C, C, 2, acc, xbn, mean, coef)
        torch.cuda.synchronize()
        assert torch.isfinite(out.float()).all(), "dx pixels left unwritten"
        if zero:
            assert float(out.float().abs().max()) == 0.0
            continue
        dx = torch.nn.grad.conv2d_input(xbn.shape, w.float(), dy.float(), stride=2, padding=1)
        mask = (xbn.float() * coef[:C].view(1, C, 1, 1) + coef[C:].view(1, C, 1, 1)) > 0
        ref = torch.where(mask, dx.bfloat16().float(), torch.zeros_like(dx))
        torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("C,Hx,Wx,nb", [(128, 27, 27, 2), (256, 13, 14, 2), (64, 7, 7, 3), (128, 55, 56, 1)])
def test_s2_dgrad_maskx_odd_input(C, Hx, Wx, nb):
    """Odd conv input (dx = 2 Hd - 1 rows / columns): the last sub-pixel row /
    column is masked in the epilogue -- every dx pixel written once, nothing past
    the tensor (a NaN guard region behind it stays NaN), BN sums over dx only."""
    torch.manual_seed(25)
    ext = _ext()
    Hd, Wd = (Hx - 1) // 2 + 1, (Wx - 1) // 2 + 1
    dy = _nhwc(torch.randn(nb, C, Hd, Wd, device="cuda").bfloat16())
    w = _nhwc((torch.randn(C, C, 3, 3, device="cuda") / (3 * C ** 0.5)).bfloat16())
    xbn = _nhwc(torch.randn(nb, C, Hx, Wx, device="cuda").bfloat16())
    coef = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.5]).float()
    mean = torch.randn(C, device="cuda") * 0.1
    acc = torch.zeros(REP * 2 * C, device="cuda")
    n_out = nb * C * Hx * Wx
    buf = torch.full((n_out + 4096 * C,), float("nan"), device="cuda", dtype=torch.bfloat16)
    out = buf[:n_out].view(nb, Hx, Wx, C).permute(0, 3, 1, 2)  # channels_last view of the buffer head
    ext.conv3x3_s2_dgrad(dy, s2_dgrad_weights(w), out, nb, Hd, Wd, C, C, 2, acc, xbn, mean, coef, Hx, Wx)
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all(), "dx pixels left unwritten"
    assert torch.isnan(buf[n_out:].float()).all(), "write past the end of dx"
    dx = torch.nn.grad.conv2d_input(xbn.shape, w.float(), dy.float(), stride=2, padding=1)
    mask = (xbn.float() * coef[:C].view(1, C, 1, 1) + coef[C:].view(1, C, 1, 1)) > 0
    ref = torch.where(mask, dx.bfloat16().float(), torch.zeros_like(dx))
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2)
    g = _rows(out.float()).double()
    s = acc.view(REP, 2, C).sum(0).double()
    torch.testing.assert_close(s[0], g.sum(0), atol=0.3, rtol=1e-2)
    torch.testing.assert_close(s[1], (g * (_rows(xbn.float()).double() - mean.double())).sum(0), atol=0.3,
                               rtol=1e-2)
