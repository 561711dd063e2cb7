"""Fused 1x1-conv MFMA GEMMs (csrc/conv1x1.hip) vs plain PyTorch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

REP = 32  # BN workspace replicas


def _ext():
    from kubedl_amd.ops import _ext
    return _ext.load()


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _ws(C, dev):
    return torch.zeros(_ext().bn_workspace_floats(C), device=dev)


def _rows(t):  # NHWC 4-D -> [rows, C] view of the same memory
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _gemm(A, W, C, M, N, K, **kw):
    ext = _ext()
    args = dict(Hout=0, Wout=0, Hin=0, Win=0, stride=1, pro_coef=None, epi=0, shift=None, acc=None, ex=None,
                emean=None, ecoef=None, eres=None, res_stride=1, res_H=0, res_W=0, ebits=None, ex2=None,
                emean2=None, acc2=None)
    args.update(kw)
    ext.conv1x1_gemm(A, W, C, M, N, K, args["Hout"], args["Wout"], args["Hin"], args["Win"], args["stride"],
                     args["pro_coef"], args["epi"], args["shift"], args["acc"], args["ex"], args["emean"],
                     args["ecoef"], args["eres"], args["res_stride"], args["res_H"], args["res_W"], args["ebits"],
                     args["ex2"], args["emean2"], args["acc2"])


@pytest.mark.parametrize("N,K,M", [(64, 64, 1000), (256, 64, 4096), (64, 256, 777), (512, 128, 2048),
                                   (128, 1024, 300)])
def test_gemm_plain_matches_conv(N, K, M):
    torch.manual_seed(0)
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    _gemm(A, W, C, M, N, K)
    ref = A.float() @ W.float().t()
    torch.testing.assert_close(C.float(), ref, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("N,K", [(128, 64), (64, 128)])
def test_gemm_prologue_gather_stats(stride, N, K):
    torch.manual_seed(1)
    nb, H, Wd = 3, 14, 10
    x = _nhwc(torch.randn(nb, K, H, Wd, device="cuda").bfloat16())
    w = (torch.randn(N, K, 1, 1, device="cuda") / K ** 0.5).bfloat16()
    coef = torch.cat([torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda")]).float()
    shift = torch.randn(N, device="cuda")
    Ho, Wo = (H - 1) // stride + 1, (Wd - 1) // stride + 1
    M = nb * Ho * Wo
    y = _nhwc(torch.empty(nb, N, Ho, Wo, device="cuda", dtype=torch.bfloat16))
    ws = _ws(N, "cuda")
    _gemm(x, w, y, M, N, K, Hout=Ho, Wout=Wo, Hin=H, Win=Wd, stride=stride, pro_coef=coef, epi=1, shift=shift,
          acc=ws)
    a = F.relu(x.float() * coef[:K].view(1, K, 1, 1) + coef[K:].view(1, K, 1, 1)).bfloat16().float()
    ref = F.conv2d(a, w.float(), stride=stride)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)
    acc = ws[:REP * 2 * N].view(REP, 2, N).sum(0).double()
    yr = _rows(y).double() - shift.double()
    torch.testing.assert_close(acc[0], yr.sum(0), atol=1e-2 * M ** 0.5, rtol=1e-3)
    torch.testing.assert_close(acc[1], (yr * yr).sum(0), atol=1e-2 * M ** 0.5, rtol=1e-3)


def test_gemm_dgrad_maskx():
    torch.manual_seed(2)
    M, N, K = 3000, 128, 256  # dgrad: A = dy [M, K=Cout], B = W^T [N=Cin, K=Cout]
    dy = torch.randn(M, K, device="cuda").bfloat16()
    wt = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    x = torch.randn(M, N, device="cuda").bfloat16()
    coef = torch.cat([torch.rand(N, device="cuda") + 0.5, torch.randn(N, device="cuda")]).float()
    mean = torch.randn(N, device="cuda")
    ws = _ws(N, "cuda")
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    _gemm(dy, wt, out, M, N, K, epi=2, ex=x, emean=mean, ecoef=coef, acc=ws)
    g = (dy.float() @ wt.float().t()).bfloat16().float()
    mask = (x.float() * coef[:N] + coef[N:]) > 0
    g = torch.where(mask, g, torch.zeros_like(g))
    torch.testing.assert_close(out.float(), g, atol=3e-2, rtol=3e-2)
    acc = ws[:REP * 2 * N].view(REP, 2, N).sum(0).double()
    torch.testing.assert_close(acc[0], g.double().sum(0), atol=0.5, rtol=1e-2)
    torch.testing.assert_close(acc[1], (g.double() * (x.double() - mean.double())).sum(0), atol=0.5, rtol=1e-2)


@pytest.mark.parametrize("res_stride", [1, 2])
@pytest.mark.parametrize("with_x2", [False, True])
def test_gemm_dgrad_resbits(res_stride, with_x2):
    torch.manual_seed(3)
    nb, H, Wd, N, K = 2, 8, 6, 64, 128
    M = nb * H * Wd
    dy = torch.randn(M, K, device="cuda").bfloat16()
    wt = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    Ho, Wo = (H - 1) // res_stride + 1, (Wd - 1) // res_stride + 1
    res = torch.randn(nb * Ho * Wo, N, device="cuda").bfloat16()
    x = torch.randn(M, N, device="cuda").bfloat16()
    x2 = torch.randn(M, N, device="cuda").bfloat16() if with_x2 else None
    bits = torch.randint(0, 256, (M, N // 8), device="cuda", dtype=torch.uint8)
    mean, mean2 = torch.randn(N, device="cuda"), torch.randn(N, device="cuda")
    ws, ws2 = _ws(N, "cuda"), _ws(N, "cuda")
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
        torch.testing.assert_close(acc2[0], g.double().sum(0), atol=0.3, rtol=1e-2)
        torch.testing.assert_close(acc2[1], (g.double() * (x2.double() - mean2.double())).sum(0), atol=0.3,
                                   rtol=1e-2)


@pytest.mark.parametrize("N,K", [(64, 64), (128, 256), (256, 64), (64, 128)])
@pytest.mark.parametrize("stride,pro", [(1, False), (2, True), (1, True)])
def test_wgrad(N, K, stride, pro):
    torch.manual_seed(4)
    ext = _ext()
    nb, H, Wd = 3, 12, 9
    Ho, Wo = (H - 1) // stride + 1, (Wd - 1) // stride + 1
    M = nb * Ho * Wo
    x = _nhwc(torch.randn(nb, K, H, Wd, device="cuda").bfloat16())
    g = torch.randn(M, N, device="cuda").bfloat16()
    coef = torch.cat([torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda")]).float() if pro else None
    slabs = ext.conv1x1_wgrad_splits(M, N, K)
    ws = torch.full((slabs * N * K,), float("nan"), device="cuda")  # no initialisation required
    ext.conv1x1_wgrad(g, x, coef, ws, None, 1.0, M, N, K, Ho, Wo, H, Wd, stride)
    dw = ws[:N * K].view(N, K)
    a = x.float()
    if pro:
        a = F.relu(a * coef[:K].view(1, K, 1, 1) + coef[K:].view(1, K, 1, 1)).bfloat16().float()
    a = _rows(a[:, :, ::stride, ::stride].contiguous(memory_format=torch.channels_last))
    ref = g.float().t() @ a
    torch.testing.assert_close(dw, ref, atol=5e-2, rtol=1e-2)
    dwb = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    ext.conv1x1_wgrad(g, x, coef, ws, dwb, 0.5, M, N, K, Ho, Wo, H, Wd, stride)
    torch.testing.assert_close(dwb.float(), 0.5 * ref, atol=5e-2, rtol=2e-2)
    dwb2 = torch.empty_like(dwb)
    ext.conv1x1_wgrad(g, x, coef, ws, dwb2, 0.5, M, N, K, Ho, Wo, H, Wd, stride)
    assert torch.equal(dwb, dwb2)  # fixed-order slab reduction: bitwise deterministic


@pytest.mark.parametrize("N,K", [(64, 64), (256, 128)])
def test_wgrad_many_splits(N, K):
    """Large M: tens of split-M slabs, folded by all 16 reduce groups (and a ragged last split)."""
    torch.manual_seed(5)
    ext = _ext()
    nb, H, Wd = 8, 28, 27
    M = nb * H * Wd
    assert ext.conv1x1_wgrad_splits(M, N, K) > 16
    x = _nhwc(torch.randn(nb, K, H, Wd, device="cuda").bfloat16())
    g = torch.randn(M, N, device="cuda").bfloat16()
    ws = torch.empty(ext.conv1x1_wgrad_splits(M, N, K) * N * K, device="cuda")
    dwb = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    ext.conv1x1_wgrad(g, x, None, ws, dwb, 1.0, M, N, K, H, Wd, H, Wd, 1)
    ref = g.float().t() @ _rows(x.float())
    torch.testing.assert_close(dwb.float(), ref, atol=0.25, rtol=2e-2)


def _bwd_ws(C, dev, seed):
    """BN workspace with random backward coefficients k | c1 | c0 (ws_bcoef)."""
    g = torch.Generator(device=dev).manual_seed(seed)
    ws = _ws(C, dev)
    off = _ext().bn_coef_offset(C) + 2 * C
    ws[off:off + 3 * C] = torch.randn(3 * C, device=dev, generator=g)
    return ws


@pytest.mark.parametrize("epi", [0, 2, 3])
@pytest.mark.parametrize("M,N,K", [(3000, 64, 256), (700, 512, 2048), (1100, 256, 64), (513, 128, 512)])
def test_gemm_bwd_apply_prologue_bit_exact(epi, M, N, K):
    """csrc/conv1x1.hip PRO_BWD: the armed dgrad GEMM on (g, x) equals the
    separate bn_stage_bwd_apply pass + the same GEMM on its output bit for bit
    (register-staged main loop in both arms), and writes that output through."""
    ext = _ext()
    torch.manual_seed(7)
    dev = "cuda"
    g = torch.randn(M, K, device=dev).bfloat16()
    x = (torch.randn(M, K, device=dev) * 2 + 0.5).bfloat16()
    wt = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    wsb = _bwd_ws(K, dev, 11)
    dc = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    ext.bn_stage_bwd_apply(g, x, wsb, dc, None, None, None, M, K)
    kw = {}
    if epi == 2:
        kw = dict(ex=torch.randn(M, N, device=dev).bfloat16(), emean=torch.randn(N, device=dev),
                  ecoef=torch.randn(2 * N, device=dev))
    elif epi == 3:
        kw = dict(ex=torch.randn(M, N, device=dev).bfloat16(), emean=torch.randn(N, device=dev),
                  eres=torch.randn(M, N, device=dev).bfloat16(),
                  ebits=torch.randint(0, 256, (M, N // 8), device=dev, dtype=torch.uint8))
    old = ext.get_gemm_core()
    ext.set_gemm_core(0)
    try:
        ref = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ws_r = _ws(N, dev)
        _gemm(dc, wt, ref, M, N, K, epi=epi, acc=ws_r if epi else None, **kw)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        thru = torch.full((M, K), float("nan"), device=dev, dtype=torch.bfloat16)
        ws_f = _ws(N, dev)
        ext.bn_bwd_pro_arm(x, wsb, K, thru)
        _gemm(g, wt, out, M, N, K, epi=epi, acc=ws_f if epi else None, **kw)
    finally:
        ext.set_gemm_core(old)
    torch.cuda.synchronize()
    assert torch.equal(thru.view(torch.int16), dc.view(torch.int16))
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))
    if epi:
        a, b = (w[:REP * 2 * N].view(REP, 2, N).sum(0) for w in (ws_f, ws_r))
        torch.testing.assert_close(a, b, atol=1e-2, rtol=1e-4)
    # and against an fp32 reference of the whole op (apply, then the plain GEMM)
    off = ext.bn_coef_offset(K) + 2 * K
    k, c1, c0 = wsb[off:off + K], wsb[off + K:off + 2 * K], wsb[off + 2 * K:off + 3 * K]
    a32 = (k * g.float() + c1 * x.float() + c0).bfloat16().float()
    if epi == 0:
        torch.testing.assert_close(out.float(), a32 @ wt.float().t(), atol=5e-2, rtol=3e-2)


def test_gemm_bwd_apply_arm_is_consumed_and_checked():
    ext = _ext()
    M, N, K = 256, 64, 128
    g = torch.randn(M, K, device="cuda").bfloat16()
    wsb = _bwd_ws(K, "cuda", 3)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    wt = torch.randn(N, K, device="cuda").bfloat16()
    ext.bn_bwd_pro_arm(torch.randn(2 * M, K, device="cuda").bfloat16(), wsb, K, None)
    with pytest.raises(RuntimeError, match="armed for"):
        _gemm(g, wt, out, M, N, K)
    _gemm(g, wt, out, M, N, K)  # the failed launch disarmed it
    torch.testing.assert_close(out.float(), g.float() @ wt.float().t(), atol=5e-2, rtol=3e-2)
