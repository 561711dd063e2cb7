"""Classifier head kernels (csrc/head.hip: mean pool -> fc on MFMA -> softmax
cross-entropy -> dfeat / dW / db) vs a plain PyTorch fp32 reference of the same
op, at the ResNet-50 shape (2048 features, 1000 classes, 7x7 maps) and at an
odd one (masked tiles, K splits that do not divide evenly)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ext():
    from kubedl_amd.ops import _ext
    return _ext.load()


def _run(n, c, L, hw, seed, bad_label=None):
    ext = _ext()
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(n, hw, hw, c, device="cuda", generator=g).relu().bfloat16().permute(0, 3, 1, 2)
    w = (torch.randn(L, c, device="cuda", generator=g) * 0.05).bfloat16()
    b = (torch.randn(L, device="cuda", generator=g) * 0.1).bfloat16()
    y = torch.randint(0, L, (n,), device="cuda", generator=g)
    if bad_label is not None:
        y[1] = bad_label
        return _bad(ext, n, c, L, x, w, b, y)
    s1, s2 = ext.head_splits(n, c, L)
    bf = dict(dtype=torch.bfloat16, device="cuda")
    feat, dl, dlT = torch.empty(n, c, **bf), torch.empty(n, ext.head_lpad(L), **bf), torch.empty(L, n, **bf)
    part1, part2 = torch.empty(s1 * n * L, device="cuda"), torch.empty(s2 * n * c, device="cuda")
    lrow, loss = torch.empty(n, device="cuda"), torch.empty(1, device="cuda")
    dfeat, dw, db = torch.empty(n, c, **bf), torch.full((L, c), float("nan"), **bf), torch.empty(L, **bf)
    ext.head_forward(x, w, b, y, feat, part1, lrow, dl, dlT)
    ext.head_backward(feat, w, dl, dlT, part2, dfeat, dw, db, lrow, loss)
    torch.cuda.synchronize()
    # fp32 reference of the same op (features rounded to bf16 as the fc input, as the kernel)
    f32 = x.float().mean((2, 3))
    fr = f32.bfloat16().float().requires_grad_(True)
    wr, br = w.float().requires_grad_(True), b.float().requires_grad_(True)
    lr = F.cross_entropy(F.linear(fr, wr, br), y)
    lr.backward()
    return dict(feat=(feat, f32), loss=(loss[0], lr.detach()), dfeat=(dfeat, fr.grad), dw=(dw, wr.grad),
                db=(db, br.grad), dl=(dl, dlT))


@pytest.mark.parametrize("n,c,L,hw", [(256, 2048, 1000, 7), (24, 136, 40, 3), (8, 64, 10, 2)])
def test_head_matches_fp32(n, c, L, hw):
    r = _run(n, c, L, hw, 7)
    torch.testing.assert_close(r["feat"][0].float(), r["feat"][1], atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(r["loss"][0], r["loss"][1], atol=2e-3, rtol=2e-3)
    for k in ("dfeat", "dw", "db"):
        got, ref = r[k][0].float(), r[k][1]
        scale = ref.abs().max().item()
        torch.testing.assert_close(got, ref, atol=1e-2 * scale, rtol=2e-2, msg=k)
        cos = F.cosine_similarity(got.flatten(), ref.flatten(), dim=0).item()
        assert cos > 0.9999, (k, cos)
    dl, dlT = r["dl"]
    assert torch.equal(dl[:, :L].t(), dlT)  # both layouts of the same rounded values
    assert not dl[:, L:].any()  # row padding is zero


def test_head_deterministic():
    a, b = _run(256, 2048, 1000, 7, 3), _run(256, 2048, 1000, 7, 3)
    for k in ("loss", "dfeat", "dw", "db"):
        assert torch.equal(a[k][0], b[k][0]), k


def _bad(ext, n, c, L, x, w, b, y):
    s1, s2 = ext.head_splits(n, c, L)
    bf = dict(dtype=torch.bfloat16, device="cuda")
    feat, dl, dlT = torch.empty(n, c, **bf), torch.empty(n, ext.head_lpad(L), **bf), torch.empty(L, n, **bf)
    part1, part2 = torch.empty(s1 * n * L, device="cuda"), torch.empty(s2 * n * c, device="cuda")
    lrow, loss = torch.empty(n, device="cuda"), torch.empty(1, device="cuda")
    dfeat, dw, db = torch.empty(n, c, **bf), torch.empty(L, c, **bf), torch.empty(L, **bf)
    ext.head_forward(x, w, b, y, feat, part1, lrow, dl, dlT)
    ext.head_backward(feat, w, dl, dlT, part2, dfeat, dw, db, lrow, loss)
    torch.cuda.synchronize()
    return lrow, loss, dl


@pytest.mark.parametrize("bad", [-100, 10, 1 << 40])
def test_head_out_of_range_label_is_nan_not_a_wild_read(bad):
    """a label outside [0, L) (the ignore_index -100, or L itself)
    never indexes past the logits: that row's loss is NaN (the step's loss turns
    NaN, loudly) and its gradient row is zero; the other rows are untouched."""
    lrow, loss, dl = _run(8, 64, 10, 2, 5, bad_label=bad)
    assert torch.isnan(lrow[1]) and torch.isnan(loss[0])
    assert not torch.isnan(lrow[torch.arange(8, device="cuda") != 1]).any()
    assert not dl[1].float().any()
