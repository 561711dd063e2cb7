"""ResNet stem conv on MFMA (csrc/stem.hip, 7x7 / stride 2 / pad 3, 224 -> 112,
3 -> 64 channels) vs plain PyTorch fp32 conv2d: plain store, the BN-statistics
epilogue, and the stem BN + ReLU + max-pool forward fed by those statistics
(``bn_pool_fwd(gemm_stats=True)``) vs the same op computing its own."""
import pytest
import torch
import torch.nn.functional as F

from kubedl_amd.ops.conv import stem_weights

pytestmark = pytest.mark.gpu

REP = 32


def _ext():
    from kubedl_amd.ops import _ext
    return _ext.load()


def _inputs(nb, seed):
    torch.manual_seed(seed)
    x = torch.randn(nb, 224, 224, 3, device="cuda").bfloat16().permute(0, 3, 1, 2)  # NHWC storage
    w = (torch.randn(64, 3, 7, 7, device="cuda") / 12).bfloat16().contiguous(memory_format=torch.channels_last)
    return x, w


@pytest.mark.parametrize("nb", [1, 3])
def test_stem_plain_matches_fp32(nb):
    ext = _ext()
    x, w = _inputs(nb, 31)
    y = torch.full((nb, 64, 112, 112), float("nan"), device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ext.stem7x7_fwd(x, stem_weights(w), y, None, None)
    ref = F.conv2d(x.float(), w.float(), stride=2, padding=3)
    assert torch.isfinite(y.float()).all()
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)


def test_stem_stats_and_bn_pool():
    ext = _ext()
    nb = 2
    x, w = _inputs(nb, 32)
    y = torch.empty(nb, 64, 112, 112, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    rm = torch.randn(64, device="cuda") * 0.1
    rv = torch.rand(64, device="cuda") + 0.5
    ws = torch.zeros(ext.bn_workspace_floats(64), device="cuda")
    ext.stem7x7_fwd(x, stem_weights(w), y, rm, ws[:REP * 2 * 64])
    yr = y.float().permute(0, 2, 3, 1).reshape(-1, 64) - rm
    s = ws[:REP * 2 * 64].view(REP, 2, 64).sum(0)
    torch.testing.assert_close(s[0], yr.sum(0), atol=0.5, rtol=1e-3)
    torch.testing.assert_close(s[1], (yr * yr).sum(0), atol=0.5, rtol=1e-3)
    # the BN + ReLU + max-pool forward from the epilogue's sums == computing its own
    gamma = (torch.rand(64, device="cuda") + 0.5).bfloat16()
    beta = (torch.randn(64, device="cuda") * 0.1).bfloat16()
    rm2, rv2 = rm.clone(), rv.clone()
    ws2 = torch.zeros_like(ws)
    out = ext.bn_pool_fwd(y, gamma, beta, rm, rv, True, 0.1, 1e-5, ws, True, False)
    ref = ext.bn_pool_fwd(y, gamma, beta, rm2, rv2, True, 0.1, 1e-5, ws2, False, False)
    torch.testing.assert_close(out[1], ref[1], atol=1e-4, rtol=1e-4)  # mean
    torch.testing.assert_close(out[2], ref[2], atol=1e-3, rtol=1e-3)  # invstd
    torch.testing.assert_close(out[0].float(), ref[0].float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(rm, rm2, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(rv, rv2, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("nb", [1, 3, 10])
def test_stem_wgrad_matches_fp32(nb):
    """Weight gradient (both operands read pixel-major from LDS, fp32 slabs,
    fixed-order reduce) vs torch.nn.grad.conv2d_weight in fp32; nb = 3 and 10
    leave a partial last round of tiles for some blocks."""
    from kubedl_amd.ops.conv import stem_grad_from_k
    ext = _ext()
    x, _ = _inputs(nb, 33)
    dy = torch.randn(nb, 112, 112, 64, device="cuda").bfloat16().permute(0, 3, 1, 2)
    ws = torch.empty(ext.stem7x7_wgrad_slabs(nb) * 64 * 224, device="cuda")
    dwk = torch.empty(64, 224, device="cuda", dtype=torch.bfloat16)
    ext.stem7x7_wgrad(dy, x, ws, dwk)
    ref = torch.nn.grad.conv2d_weight(x.float(), (64, 3, 7, 7), dy.float(), stride=2, padding=3)
    got = stem_grad_from_k(dwk).float()
    scale = ref.abs().max().item()
    torch.testing.assert_close(got, ref, atol=1e-2 * scale, rtol=1e-2)
    again = torch.empty_like(dwk)
    ext.stem7x7_wgrad(dy, x, ws, again)
    assert torch.equal(again, dwk), "stem weight gradient must be deterministic"


def _pool_setup(nb, seed):
    ext = _ext()
    x, w = _inputs(nb, seed)
    c0 = torch.empty(nb, 64, 112, 112, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ext.stem7x7_fwd(x, stem_weights(w), c0, None, None)
    gamma = (torch.rand(64, device="cuda") + 0.5).bfloat16()
    beta = (torch.randn(64, device="cuda") * 0.3).bfloat16()
    rm, rv = torch.zeros(64, device="cuda"), torch.ones(64, device="cuda")
    ws = torch.zeros(ext.bn_workspace_floats(64), device="cuda")
    y, mean, invstd, idx, xam = ext.bn_pool_fwd(c0, gamma, beta, rm, rv, True, 0.1, 1e-5, ws, False, True)
    dp = torch.randn_like(y.float()).bfloat16().contiguous(memory_format=torch.channels_last)
    return ext, x, c0, gamma, beta, mean, invstd, idx, dp, ws, xam


@pytest.mark.parametrize("nb", [2, 5])
def test_stem_wgrad_bn_fused_matches_unfused(nb):
    """BN + ReLU + max-pool backward folded into the weight gradient == the
    separate apply pass followed by the plain stem weight gradient."""
    ext, x, c0, gamma, beta, mean, invstd, idx, dp, ws, xam = _pool_setup(nb, 34)
    slabs = torch.empty(ext.stem7x7_wgrad_slabs(nb) * 64 * 224, device="cuda")
    dx, dg, db = ext.bn_pool_bwd(dp, idx, c0, gamma, beta, mean, invstd, True, ws, True)
    ref = torch.empty(64, 224, device="cuda", dtype=torch.bfloat16)
    ext.stem7x7_wgrad(dx, x, slabs, ref)
    ws2 = ws.clone()
    nodx, dg2, db2 = ext.bn_pool_bwd(dp, idx, c0, gamma, beta, mean, invstd, True, ws2, False)
    assert nodx is None
    torch.testing.assert_close(dg2.float(), dg.float(), atol=0, rtol=0)
    torch.testing.assert_close(db2.float(), db.float(), atol=0, rtol=0)
    # the engine's sums over pooled cells (x at the argmax) == the per-pixel gather sums
    ws3 = ws.clone()
    dg3 = torch.empty_like(dg)
    db3 = torch.empty_like(db)
    ext.bn_stage_bwd_reduce(dp, xam, gamma, beta, mean, invstd, ws3, dp.numel() // 64, 64, True)
    ext.bn_stage_bwd_finalize(ws3, c0.numel() // 64, 64, gamma, mean, invstd, dg3, db3, True)
    torch.testing.assert_close(dg3.float(), dg.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(db3.float(), db.float(), atol=2e-2, rtol=2e-2)
    got = torch.empty_like(ref)
    ext.stem7x7_wgrad_bn(c0, dp, idx, ws2, x, slabs, got)
    scale = ref.float().abs().max().item()
    torch.testing.assert_close(got.float(), ref.float(), atol=2e-3 * scale, rtol=1e-2)


@pytest.mark.parametrize("nb", [2, 3])
def test_stem_raw_weight_layout_bit_exact(nb):
    """The channels_last [64, 3, 7, 7] parameter passed as is: the forward
    reorders it while staging (no per-step stem_weights launch) and the weight
    gradient lands directly in the parameter's layout -- both bit-identical to
    the K-order path (the same sums, only the index map differs)."""
    from kubedl_amd.ops.conv import stem_grad_from_k
    ext = _ext()
    x, w = _inputs(nb, 35)
    assert w.is_contiguous(memory_format=torch.channels_last)
    ya = torch.empty(nb, 64, 112, 112, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    yb = torch.empty_like(ya)
    ext.stem7x7_fwd(x, stem_weights(w), ya, None, None)
    ext.stem7x7_fwd(x, w, yb, None, None)
    bad = (ya.float() != yb.float()).nonzero()
    assert bad.numel() == 0, (f"{bad.shape[0]} differing outputs, first {bad[:8].tolist()}; "
                              f"ya {ya[tuple(bad[0])].item()} yb {yb[tuple(bad[0])].item()}")
    dy = torch.randn(nb, 112, 112, 64, device="cuda").bfloat16().permute(0, 3, 1, 2)
    ws = torch.empty(ext.stem7x7_wgrad_slabs(nb) * 64 * 224, device="cuda")
    dwk = torch.empty(64, 224, device="cuda", dtype=torch.bfloat16)
    ext.stem7x7_wgrad(dy, x, ws, dwk)
    raw = torch.full((64, 3, 7, 7), float("nan"), device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ext.stem7x7_wgrad(dy, x, ws, raw)
    assert torch.equal(raw, stem_grad_from_k(dwk))


@pytest.mark.parametrize("nb,h,w", [(2, 64, 64), (1, 97, 250), (3, 33, 17)])
def test_stem_any_geometry_matches_fp32(nb, h, w):
    """the stem kernel at sizes other than 224 (2-row x
    112-column tiles, masked edges, odd heights / widths, more than one column
    chunk) -- forward with the BN-statistics epilogue and the weight gradient vs
    fp32 PyTorch; no MIOpen fallback remains."""
    ext = _ext()
    torch.manual_seed(h * 1000 + w)
    x = torch.randn(nb, h, w, 3, device="cuda").bfloat16().permute(0, 3, 1, 2)
    wt = (torch.randn(64, 3, 7, 7, device="cuda") / 12).bfloat16().contiguous(memory_format=torch.channels_last)
    oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    y = torch.full((nb, 64, oh, ow), float("nan"), device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    rm = torch.randn(64, device="cuda") * 0.1
    ws = torch.zeros(ext.bn_workspace_floats(64), device="cuda")
    ext.stem7x7_fwd(x, wt, y, rm, ws[:REP * 2 * 64])
    ref = F.conv2d(x.float(), wt.float(), stride=2, padding=3)
    assert torch.isfinite(y.float()).all()
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)
    yr = y.float().permute(0, 2, 3, 1).reshape(-1, 64) - rm
    s = ws[:REP * 2 * 64].view(REP, 2, 64).sum(0)
    torch.testing.assert_close(s[0], yr.sum(0), atol=0.5, rtol=1e-3)  # masked slots add nothing
    dy = torch.randn(nb, oh, ow, 64, device="cuda").bfloat16().permute(0, 3, 1, 2)
    slabs = torch.empty(ext.stem7x7_wgrad_slabs(nb, h, w) * 64 * 224, device="cuda")
    dw = torch.full((64, 3, 7, 7), float("nan"), device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ext.stem7x7_wgrad(dy, x, slabs, dw)
    gref = torch.nn.grad.conv2d_weight(x.float(), (64, 3, 7, 7), dy.float(), stride=2, padding=3)
    torch.testing.assert_close(dw.float(), gref, atol=1e-2 * gref.abs().max().item(), rtol=1e-2)
