"""The BN + ReLU A prologue on the LDS-DMA GEMM loop (csrc/igemm.hip PRO,
``set_igemm_pro(1)``) vs the register-staged loop's PRO_FWD (csrc/conv1x1.hip):
the same forward 1x1 conv with the statistics epilogue.  A' = bf16(relu(A *
scale + shift)) is built with the same fmaf / ReLU / rounding in both, and both
accumulate K in 16-deep MFMA steps, so the outputs must agree bit for bit; the
BN sums to fp32 rounding.  Also checked against a plain PyTorch fp32 reference.
M tails exercise the rows past M (transformed garbage, never stored or summed)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

REP = 32


def _ext():
    from kubedl_amd.ops import _ext
    return _ext.load()


def _run(ext, a, b, coef, M, N, K, pro_on):
    ext.set_igemm_pro(1 if pro_on else 0)
    try:
        c = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        shift = torch.randn(N, device="cuda", generator=torch.Generator("cuda").manual_seed(5)) * 0.1
        acc = torch.zeros(REP * 2 * N, device="cuda")
        ext.conv1x1_gemm(a, b, c, M, N, K, 0, 0, 0, 0, 1, coef, 1, shift, acc, None, None, None, None, 1, 0, 0,
                         None, None, None, None)
        torch.cuda.synchronize()
        return c, acc.view(REP, 2, N).sum(0), shift
    finally:
        ext.set_igemm_pro(0)


@pytest.mark.parametrize("M,K,N", [(4100, 64, 256), (3000, 128, 512), (2000, 256, 1024), (1000, 512, 256),
                                   (777, 1024, 128), (50176, 256, 1024)])
def test_igemm_pro_matches_register_prologue(M, K, N):
    ext = _ext()
    torch.manual_seed(M + K)
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    coef = torch.cat([torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.5]).float()
    y0, s0, shift = _run(ext, a, b, coef, M, N, K, False)
    y1, s1, _ = _run(ext, a, b, coef, M, N, K, True)
    assert torch.isfinite(y1.float()).all(), "rows left unwritten"
    assert torch.equal(y0, y1), (y0.float() - y1.float()).abs().max()
    torch.testing.assert_close(s1, s0, atol=1e-2, rtol=1e-4)
    ap = torch.relu(a.float() * coef[:K] + coef[K:]).bfloat16().float()
    ref = ap @ b.float().t()
    torch.testing.assert_close(y1.float(), ref, atol=3e-2, rtol=3e-2)
    d = y1.float() - shift
    torch.testing.assert_close(s1[0], d.sum(0), atol=0.5, rtol=1e-3)
    torch.testing.assert_close(s1[1], (d * d).sum(0), atol=0.5, rtol=1e-3)
