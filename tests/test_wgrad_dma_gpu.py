"""Weight gradients on the LDS-DMA pipeline (csrc/wgrad_dma.hip) vs plain
PyTorch fp32 references, with the core forced on; and the DMA and
register-staged kernels against each other on the same inputs.

Covers dense / strided-gather / 3x3 (padding taps as out-of-range loads, stride
1 and 2) operands, the BN+ReLU prologue applied to the transposed fragments
(with rows past the M range re-zeroed), ragged last splits and many splits."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ext():
    from kubedl_amd.ops import _ext
    return _ext.load()


@pytest.fixture(autouse=True)
def dma_core():
    ext = _ext()
    old = ext.get_gemm_core()
    ext.set_gemm_core(1)
    yield
    ext.set_gemm_core(old)


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _rows(t):
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _wgrad1x1(g, x, coef, N, K, Ho, Wo, H, Wd, stride, scale=1.0):
    ext = _ext()
    M = g.shape[0]
    ws = torch.full((ext.conv1x1_wgrad_splits(M, N, K) * N * K,), float("nan"), device="cuda")
    dwb = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    ext.conv1x1_wgrad(g, x, coef, ws, dwb, scale, M, N, K, Ho, Wo, H, Wd, stride)
    return dwb


@pytest.mark.parametrize("N,K", [(64, 64), (128, 256), (256, 64), (64, 128), (512, 2048), (256, 256), (1024, 512)])
@pytest.mark.parametrize("stride,pro", [(1, False), (2, True), (1, True), (2, False)])
def test_dma_wgrad_1x1(N, K, stride, pro):
    torch.manual_seed(4)
    nb, H, Wd = 3, 12, 9
    Ho, Wo = (H - 1) // stride + 1, (Wd - 1) // stride + 1
    M = nb * Ho * Wo  # not a multiple of 64: ragged last split
    x = _nhwc(torch.randn(nb, K, H, Wd, device="cuda").bfloat16())
    g = torch.randn(M, N, device="cuda").bfloat16()
    coef = torch.cat([torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda")]).float() if pro else None
    dw = _wgrad1x1(g, x, coef, N, K, Ho, Wo, H, Wd, stride)
    a = x.float()
    if pro:
        a = F.relu(a * coef[:K].view(1, K, 1, 1) + coef[K:].view(1, K, 1, 1)).bfloat16().float()
    a = _rows(a[:, :, ::stride, ::stride].contiguous(memory_format=torch.channels_last))
    ref = g.float().t() @ a
    scale = ref.abs().max().item()
    torch.testing.assert_close(dw.float() / scale, ref / scale, atol=1e-2, rtol=1e-2)
    assert torch.equal(dw, _wgrad1x1(g, x, coef, N, K, Ho, Wo, H, Wd, stride))  # deterministic


@pytest.mark.parametrize("N,K", [(64, 64), (256, 128), (256, 512)])
def test_dma_wgrad_many_splits_matches_register_kernel(N, K):
    torch.manual_seed(5)
    ext = _ext()
    nb, H, Wd = 8, 28, 27
    M = nb * H * Wd
    assert ext.conv1x1_wgrad_splits(M, N, K) > 16
    x = _nhwc(torch.randn(nb, K, H, Wd, device="cuda").bfloat16())
    g = torch.randn(M, N, device="cuda").bfloat16()
    coef = torch.cat([torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda")]).float()
    dma = _wgrad1x1(g, x, coef, N, K, H, Wd, H, Wd, 1)
    ext.set_gemm_core(0)
    reg = _wgrad1x1(g, x, coef, N, K, H, Wd, H, Wd, 1)
    ext.set_gemm_core(1)
    a = F.relu(x.float() * coef[:K].view(1, K, 1, 1) + coef[K:].view(1, K, 1, 1)).bfloat16().float()
    ref = g.float().t() @ _rows(a)
    scale = ref.abs().max().item()
    torch.testing.assert_close(dma.float() / scale, ref / scale, atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(dma.float() / scale, reg.float() / scale, atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("Cin,Cout,H,W,stride", [(64, 64, 12, 10, 1), (128, 64, 9, 9, 2), (64, 128, 28, 27, 1),
                                                 (256, 128, 7, 7, 1), (128, 256, 14, 14, 2),
                                                 (256, 256, 14, 14, 1), (256, 512, 13, 13, 2), (512, 512, 7, 7, 1)])
def test_dma_wgrad_3x3(Cin, Cout, H, W, stride):
    torch.manual_seed(2)
    ext = _ext()
    nb = 4
    x = _nhwc(torch.randn(nb, Cin, H, W, device="cuda").bfloat16())
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    dy = _nhwc(torch.randn(nb, Cout, Ho, Wo, device="cuda").bfloat16())
    M = nb * Ho * Wo
    ref = torch.nn.grad.conv2d_weight(x.float(), (Cout, Cin, 3, 3), dy.float(), stride=stride, padding=1)
    scale = ref.abs().max().item()
    # a conv1x1_wgrad_splits-sized workspace (128 x 128 tiles) and the engine's
    # conv3x3_wgrad_slabs-sized one (256 x 256 tiles where Cin, Cout % 256 == 0)
    for slabs in (ext.conv1x1_wgrad_splits(M, Cout, 9 * Cin), ext.conv3x3_wgrad_slabs(nb, H, W, Cin, Cout, stride)):
        ws = torch.full((slabs * Cout * 9 * Cin,), float("nan"), device="cuda")
        dW = _nhwc(torch.empty(Cout, Cin, 3, 3, device="cuda", dtype=torch.bfloat16))
        ext.conv3x3_wgrad(dy, x, None, ws, dW, 1.0, nb, H, W, Cin, Cout, stride)
        torch.testing.assert_close(dW.float() / scale, ref / scale, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("nb", [1, 3, 20])
def test_halo_wgrad_3x3_stage1(nb):
    """The 56x56 / 64-channel weight gradient on the input-halo kernel (csrc/halo3x3.hip:
    dy and the input halo staged once per 4-row tile, nine shifted transposed reads)
    against fp32 truth; bitwise equal to itself on a rerun (fixed-order slabs), and the
    small conv1x1_wgrad_splits workspace still takes the implicit-GEMM path."""
    torch.manual_seed(5)
    ext = _ext()
    Cin = Cout = 64
    H = W = 56
    x = _nhwc(torch.randn(nb, Cin, H, W, device="cuda").bfloat16())
    dy = _nhwc(torch.randn(nb, Cout, H, W, device="cuda").bfloat16())
    slabs = ext.conv3x3_wgrad_slabs(nb, H, W, Cin, Cout, 1)
    assert slabs >= min(nb * 14, 128)  # one slab per halo block (<= 256 blocks)
    ref = torch.nn.grad.conv2d_weight(x.float(), (Cout, Cin, 3, 3), dy.float(), stride=1, padding=1)
    scale = ref.abs().max().item()
    outs = []
    for n_slabs in (slabs, slabs, ext.conv1x1_wgrad_splits(nb * H * W, Cout, 9 * Cin)):
        ws = torch.full((n_slabs * Cout * 9 * Cin,), float("nan"), device="cuda")
        dW = _nhwc(torch.empty(Cout, Cin, 3, 3, device="cuda", dtype=torch.bfloat16))
        ext.conv3x3_wgrad(dy, x, None, ws, dW, 1.0, nb, H, W, Cin, Cout, 1)
        torch.testing.assert_close(dW.float() / scale, ref / scale, atol=2e-2, rtol=2e-2)
        outs.append(dW)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("N,K", [(64, 64), (256, 64), (64, 256), (128, 128), (512, 2048), (2048, 512), (64, 128)])
@pytest.mark.parametrize("stride,pro", [(1, False), (1, True), (2, False)])
def test_dma_wgrad_bwd_apply_g_prologue(N, K, stride, pro):
    """BWDG: the weight gradient on (g, gx) with the BN-backward apply
    G' = k g + c1 gx + c0 computed in the G fragments equals the weight
    gradient of the materialised G' (bn_stage_bwd_apply's output, bit-identical
    operand) within reduction-order rounding, ragged last split included."""
    ext = _ext()
    torch.manual_seed(9)
    nb, H, Wd = 3, 12, 9
    Ho, Wo = (H - 1) // stride + 1, (Wd - 1) // stride + 1
    M = nb * Ho * Wo
    x = _nhwc(torch.randn(nb, K, H, Wd, device="cuda").bfloat16())
    g = torch.randn(M, N, device="cuda").bfloat16()
    gx = (torch.randn(M, N, device="cuda") * 2 + 1).bfloat16()
    ws = torch.zeros(ext.bn_workspace_floats(N), device="cuda")
    off = ext.bn_coef_offset(N) + 2 * N
    ws[off:off + 3 * N] = torch.randn(3 * N, device="cuda")
    gp = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ext.bn_stage_bwd_apply(g, gx, ws, gp, None, None, None, M, N)
    coef = torch.cat([torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda")]).float() if pro else None
    ref = _wgrad1x1(gp, x, coef, N, K, Ho, Wo, H, Wd, stride)
    wsl = torch.full((ext.conv1x1_wgrad_splits(M, N, K) * N * K,), float("nan"), device="cuda")
    dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    ext.bn_bwd_pro_arm(gx, ws, N, None)
    ext.conv1x1_wgrad(g, x, coef, wsl, dw, 1.0, M, N, K, Ho, Wo, H, Wd, stride)
    a = x.float()
    if pro:
        a = F.relu(a * coef[:K].view(1, K, 1, 1) + coef[K:].view(1, K, 1, 1)).bfloat16().float()
    a = _rows(_nhwc(a[:, :, ::stride, ::stride]))
    truth = gp.float().t() @ a
    scale = truth.abs().max().item()
    torch.testing.assert_close(dw.float(), truth, atol=2e-2 * scale, rtol=2e-2)
    torch.testing.assert_close(dw.float(), ref.float(), atol=1e-2 * scale, rtol=1e-2)
