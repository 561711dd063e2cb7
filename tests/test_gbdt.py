"""Histogram GBDT: torch path (CPU), distributed equivalence (gloo, 2 ranks),
and the HIP kernels against the torch reference (GPU)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from kubedl_amd.models.gbdt import GBDTParams, HistGBDT


def _data(n=4000, f=8, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, f, generator=g)
    y = ((X[:, 0] - X[:, 1] * X[:, 2] + 0.2 * torch.randn(n, generator=g)) > 0).long()
    return X, y


def test_params_parse():
    p = GBDTParams.parse('"objective:multi:softprob,num_class:3"', n_estimators=10, learning_rate=0.1)
    assert p.objective == "multi:softprob" and p.num_class == 3 and p.n_estimators == 10
    assert p.learning_rate == 0.1
    p = GBDTParams.parse("eta:0.05,max_depth:3,lambda:2")
    assert p.learning_rate == 0.05 and p.max_depth == 3 and p.reg_lambda == 2.0


def test_cpu_binary_learns_and_predict_consistent():
    X, y = _data()
    m = HistGBDT(GBDTParams(objective="binary:logistic", n_estimators=15, max_depth=5, max_bin=64), "cpu")
    pred = m.fit(X, y)
    met = m.metric(pred, y)
    assert met["accuracy"] > 0.9
    assert m.stats["hist_subtracted"] > 0
    torch.testing.assert_close(m.predict_margin(X), pred, atol=1e-5, rtol=1e-5)


def test_histogram_subtraction_exact():
    """Sibling histogram = parent - child equals a directly built one."""
    X, y = _data(2000, 5)
    m = HistGBDT(GBDTParams(max_bin=32), "cpu")
    m.fit_cuts(X)
    bins = m.quantise(X)
    g, h = torch.randn(2000), torch.rand(2000) + 0.5
    rows = torch.arange(2000, dtype=torch.int32)
    parent = m._hist(bins, g, h, rows, [0, 2000], 5, 32)
    left = rows[X[:, 0] <= 0]
    right = rows[X[:, 0] > 0]
    hl = m._hist(bins, g, h, left, [0, len(left)], 5, 32)
    hr = m._hist(bins, g, h, right, [0, len(right)], 5, 32)
    torch.testing.assert_close(parent - hl, hr, atol=1e-4, rtol=1e-4)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dist_worker(rank, world, port, X, y, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    m = HistGBDT(GBDTParams(objective="binary:logistic", n_estimators=4, max_depth=4, max_bin=32), "cpu")
    # cuts from the full data so both runs quantise identically
    m.fit_cuts(X, sample=len(X))
    Xs, ys = X[rank::world], y[rank::world]
    m.fit(Xs, ys)
    out[rank] = [[(t.feature, t.split_bin, [round(v, 5) for v in t.value]) for t in r] for r in m.trees]
    dist.destroy_process_group()


def test_distributed_trees_match_single_process():
    X, y = _data(1200, 6, seed=3)
    single = HistGBDT(GBDTParams(objective="binary:logistic", n_estimators=4, max_depth=4, max_bin=32), "cpu")
    single.fit_cuts(X, sample=len(X))
    single.fit(X, y)
    ref = [[(t.feature, t.split_bin, [round(v, 5) for v in t.value]) for t in r] for r in single.trees]
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, X, y, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert out[0] == out[1], "ranks grew different trees"
    # same model as one process on all rows, up to float-summation near-ties
    # (a different reduction order can flip a split between two equal-gain bins)
    assert ref[0][0][0][0] == out[0][0][0][0][0] and ref[0][0][1][0] == out[0][0][0][1][0]  # root split
    same = tot = 0
    for r_single, r_dist in zip(ref, out[0]):
        for (f1, b1, _), (f2, b2, _) in zip(r_single, r_dist):
            same += sum(int(a == b and c == d) for a, b, c, d in zip(f1, f2, b1, b2))
            tot += len(f1)
    assert same / tot > 0.8


@pytest.mark.gpu
def test_hip_kernels_match_torch_reference():
    from kubedl_amd.ops import _ext
    ext = _ext.load()
    torch.manual_seed(0)
    N, F, B = 50000, 70, 256  # F > 64 exercises two feature tiles
    bins = torch.randint(0, B, (N, F), dtype=torch.uint8)
    g, h = torch.randn(N), torch.rand(N) + 0.1
    perm = torch.randperm(N).int()
    seg = [0, 17000, 17001, 50000]
    cpu = HistGBDT(GBDTParams(max_bin=B), "cpu")
    ref = cpu._hist(bins, g, h, perm, seg, F, B)
    hist = torch.zeros(3, F, B, 2, device="cuda")
    ext.gbdt_hist(bins.cuda(), g.cuda(), h.cuda(), 1, perm.cuda(), torch.tensor(seg, dtype=torch.int32).cuda(),
                  33000, B, hist)
    torch.testing.assert_close(hist.cpu(), ref, atol=2e-3, rtol=1e-4)
    gain, bb, gl, hl = ext.gbdt_split(hist, 1.0, 1.0)
    rgain, rbin, rgl, rhl = cpu._split(hist.cpu())
    ok = torch.isfinite(rgain)
    assert torch.equal(ok, torch.isfinite(gain.cpu()))
    torch.testing.assert_close(gain.cpu()[ok], rgain[ok], atol=1e-2, rtol=1e-3)
    # bins agree except on numerical near-ties
    agree = (bb.cpu() == rbin).float().mean()
    assert agree > 0.97
    node = torch.randint(0, 3, (N,), dtype=torch.int32)
    sf = torch.tensor([5, -1, 69], dtype=torch.int32)
    sbn = torch.tensor([100, -1, 3], dtype=torch.int32)
    gr = ext.gbdt_route(bins.cuda(), perm.cuda(), node.cuda(), sf.cuda(), sbn.cuda())
    torch.testing.assert_close(gr.cpu(), cpu._route(bins, perm, node, sf, sbn))


@pytest.mark.gpu
def test_gpu_gbdt_trains():
    X, y = _data(20000, 12)
    m = HistGBDT(GBDTParams(objective="binary:logistic", n_estimators=10, max_depth=6), "cuda")
    assert m.use_hip
    pred = m.fit(X, y)
    assert m.metric(pred, y.cuda())["accuracy"] > 0.9
    assert m.stats["hist_subtracted"] > 0
    # the host trees converted from the device heap arrays predict what training accumulated
    torch.testing.assert_close(m.predict_margin(X), pred, atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
def test_gpu_quantise_matches_bucketize():
    from kubedl_amd.ops import _ext
    X, _ = _data(5000, 9)
    m = HistGBDT(GBDTParams(max_bin=64), "cpu")
    m.fit_cuts(X)
    X[:7, 3] = float("nan")  # missing values after the cuts: excluded from the comparison
    ref = m.quantise(X)
    got = _ext.load().gbdt_quantise(X.cuda(), m.cuts.cuda(), 64).cpu()
    assert torch.equal(got[7:], ref[7:])


@pytest.mark.gpu
@pytest.mark.parametrize("objective,depth", [("binary:logistic", 6), ("reg:squarederror", 4),
                                             ("multi:softprob", 5)])
def test_gpu_device_trees_match_cpu_reference(objective, depth):
    """The device-resident grower and the torch reference grow the same trees
    from the same quantised data (split features/bins compared node by node,
    up to float-summation near-ties)."""
    X, y = _data(6000, 10, seed=5)
    if objective.startswith("multi"):
        y = (X[:, 0] > 0.5).long() + (X[:, 1] > 0).long()
    kw = dict(objective=objective, n_estimators=3, max_depth=depth, max_bin=64, num_class=3)
    cpu = HistGBDT(GBDTParams(**kw), "cpu")
    cpu.fit_cuts(X, sample=len(X))
    pc = cpu.fit(X, y)
    gpu = HistGBDT(GBDTParams(**kw), "cuda")
    gpu.cuts = cpu.cuts.cuda()
    pg = gpu.fit(X, y)
    same = tot = 0
    for rc, rg in zip(cpu.trees, gpu.trees):
        for tc, tg in zip(rc, rg):
            # walk the cpu tree (list ids) and the gpu tree (heap ids) together
            stack = [(0, 0)]
            while stack:
                a, b = stack.pop()
                tot += 1
                if tc.feature[a] == tg.feature[b] and tc.split_bin[a] == tg.split_bin[b]:
                    same += 1
                    if tc.feature[a] >= 0:
                        stack += [(tc.left[a], tg.left[b]), (tc.right[a], tg.right[b])]
    assert same / tot > 0.9, (same, tot)
    # a near-tie split resolved differently moves the rows below it: compare the
    # bulk of the margins, not every element
    close = torch.isclose(pg.cpu(), pc, atol=5e-2, rtol=5e-2).float().mean()
    assert close > 0.98, float(close)


def _gpu_dist_worker(rank, world, port, X, y, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)  # two ranks share the box's one GPU
    m = HistGBDT(GBDTParams(objective="binary:logistic", n_estimators=3, max_depth=4, max_bin=32), "cuda")
    m.fit_cuts(X.cuda(), sample=len(X))
    m.fit(X[rank::world], y[rank::world])
    out[rank] = [[(t.feature, t.split_bin) for t in r] for r in m.trees]
    dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_device_grower_two_ranks_agree():
    """The multi-rank level sequence (all-reduced counts and histograms between
    level_a/b/c) grows identical trees on every rank."""
    X, y = _data(4000, 6, seed=9)
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_gpu_dist_worker, args=(r, 2, port, X, y, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert out[0] == out[1]


@pytest.mark.gpu
@pytest.mark.parametrize("objective,K", [("binary:logistic", 1), ("reg:squarederror", 1), ("multi:softprob", 4)])
def test_gpu_grad_hess_kernel_matches_torch(objective, K):
    """csrc/gbdt.hip grad_hess_kernel (one launch per round) against the torch
    composition it replaces (fp32; expf vs torch's exp may differ by an ulp)."""
    kw = dict(objective=objective)
    if K > 1:
        kw["num_class"] = K
    m = HistGBDT(GBDTParams(**kw), "cuda")
    torch.manual_seed(0)
    n = 100003
    pred = torch.randn(n, K, device="cuda") * 4
    y = torch.randint(0, K, (n,), device="cuda") if K > 1 else (torch.rand(n, device="cuda") > 0.5).float()
    g, h = m._grad_hess(pred, y)
    m.use_hip = False
    g_ref, h_ref = m._grad_hess(pred, y)
    torch.testing.assert_close(g, g_ref, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(h, h_ref, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("n,F,B", [(200000, 28, 256), (1000, 5, 16), (70000, 3, 64)])
def test_host_cuts_bitwise_equal_fit_cuts(n, F, B):
    """HistGBDT.host_cuts (numpy partition on the host copy, run beside the
    host->device copy) gives bitwise the cuts of fit_cuts (sort + lerp)."""
    from kubedl_amd.models.gbdt import GBDTParams, HistGBDT
    g = torch.Generator().manual_seed(n)
    X = torch.randn(n, F, generator=g)
    X[::97, 0] = 0.0  # ties
    m = HistGBDT(GBDTParams(max_bin=B), device="cpu")
    m.fit_cuts(X)
    assert torch.equal(m.cuts, m.host_cuts(X))


@pytest.mark.gpu
@pytest.mark.parametrize("n,L", [(2_000_000, 32), (2048 * 37 + 5, 8), (300_000, 1), (1000, 4), (2048 * 130, 64)])
def test_gpu_fused_route_scan_matches_two_pass(n, L):
    """The fused route + look-back scan (one launch, csrc/gbdt.hip route_scan_kernel)
    == route_flags + a device scan, bit for bit: many tiles (look-back windows
    of 64 predecessors and more), a ragged last tile, positions of non-split
    nodes and of other levels, and repeated launches on one status array (the
    epoch advancing over the previous launch's words, the ticket re-armed)."""
    from kubedl_amd.ops import _ext
    ext = _ext.load()
    g = torch.Generator().manual_seed(n % 1000 + L)
    F, h0 = 28, L - 1
    bins = torch.randint(0, 256, (n, F), generator=g, dtype=torch.uint8)
    rows = torch.randperm(n, generator=g).int()
    node_pos = (h0 + torch.randint(0, L, (n,), generator=g)).int()
    node_pos[::97] = h0 + L  # a deeper level's position: never routed here
    split = (torch.rand(L, generator=g) < 0.8).int()
    heap = 2 * (h0 + L) + 3
    t_feat = torch.randint(0, F, (heap,), generator=g).int()
    t_bin = torch.randint(0, 255, (heap,), generator=g).int()
    args = [t.cuda() for t in (bins, rows, node_pos, split, t_feat, t_bin)]
    ref_f, ref_s = ext.gbdt_route_scan_test(*args, h0, L, False)
    fm_f, fm_s = ext.gbdt_route_scan_test(*args, h0, L, False, 1, True)  # the grower's feature-major bins
    assert torch.equal(fm_f, ref_f) and torch.equal(fm_s, ref_s)
    for calls in (1, 3):
        f, sc = ext.gbdt_route_scan_test(*args, h0, L, True, calls)
        assert torch.equal(f, ref_f) and torch.equal(sc, ref_s), calls
    assert int(ref_s[-1]) == int(ref_f.sum())


@pytest.mark.gpu
@pytest.mark.parametrize("n,L", [(2_000_000, 32), (1024 * 37 + 5, 8), (300_000, 1), (1000, 4), (1024 * 130, 64)])
def test_gpu_three_launch_level_matches_scan_path(n, L):
    """The three-launch level (route + tile / node counts, one-block plan, per-tile
    rescan + partition) moves every row to the scan path's position and writes the
    same child segments / counts / built-child choice, bit for bit -- segments in
    heap order with positions of non-split nodes and of a shallower leaf between
    them, nodes owning no rows, a ragged last tile."""
    from kubedl_amd.ops import _ext
    ext = _ext.load()
    g = torch.Generator().manual_seed(n % 997 + L)
    F, h0 = 28, L - 1
    bins = torch.randint(0, 256, (n, F), generator=g, dtype=torch.uint8)
    rows = torch.randperm(n, generator=g).int()
    # level segments in heap order, a shallower leaf's rows in front of them
    lead = n // 7
    cuts = torch.sort(torch.randint(lead, n + 1, (L - 1,), generator=g)).values
    bounds = torch.cat([torch.tensor([lead]), cuts, torch.tensor([n])])
    if L > 2:
        bounds[2] = bounds[1]  # node 1 owns no rows
    lo, hi = bounds[:-1].int(), bounds[1:].int()
    node_pos = torch.full((n,), max(h0 - 1, 0) if h0 > 0 else -5, dtype=torch.int32)
    for i in range(L):
        node_pos[lo[i]:hi[i]] = h0 + i
    split = (torch.rand(L, generator=g) < 0.8).int()
    heap = 2 * (h0 + L) + 3
    t_feat = torch.randint(0, F, (heap,), generator=g).int()
    t_bin = torch.randint(0, 255, (heap,), generator=g).int()
    args = [t.cuda() for t in (bins, rows, node_pos, split, t_feat, t_bin, lo, hi)]
    ref = ext.gbdt_level_test(*args, h0, L, False)
    got = ext.gbdt_level_test(*args, h0, L, True)
    for a, b, name in zip(got, ref, ("rows", "node_pos", "lo", "hi", "cnt", "build_child", "blo", "bhi")):
        assert torch.equal(a, b), name


@pytest.mark.gpu
def test_gpu_fused_route_scan_fit_agrees():
    """A whole fit with the fused route + scan grows the two-pass fit's trees (up to
    near-ties of the fp32 flush order) and raises no look-back fault."""
    from kubedl_amd.ops import _ext
    ext = _ext.load()
    X, y = _data(300_000, 12, seed=9)
    res = {}
    try:
        for mode in (0, 1):
            ext.GbdtGrower.set_route_scan(mode)
            m = HistGBDT(GBDTParams(objective="binary:logistic", n_estimators=4, max_depth=6, max_bin=64), "cuda")
            m.fit_cuts(X, sample=len(X))
            pred = m.fit(X, y)
            res[mode] = (m.metric(pred, y.cuda()), m.trees[0][0])
    finally:
        ext.GbdtGrower.set_route_scan(-1)
    assert res[1][1].feature[:7] == res[0][1].feature[:7]  # the first levels of the first tree
    assert abs(res[1][0]["accuracy"] - res[0][0]["accuracy"]) < 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("F", [28, 12, 64, 100, 7])
def test_gpu_row_per_lane_hist_equals_slot_kernel(F):
    """The row-per-lane build (dword bin loads, g / h quantised once per row)
    sums the same fixed-point integers per block as the slot kernel: equal up to
    the order of the fp32 flush atomics, with g and h in one packed 64-bit LDS
    add or two 32-bit ones.  F = 7 (not a multiple of 4) runs the
    slot kernel in both; F = 100 has a 36-feature second tile; F = 64 a 128 KiB
    LDS tile."""
    from kubedl_amd.ops import _ext
    ext = _ext.load()
    g0 = torch.Generator().manual_seed(F)
    N, B, rpb = 50_000, 256, 2048
    bins = torch.randint(0, B, (N, F), generator=g0, dtype=torch.uint8)
    bins[:, 0] = 3  # one hot bin: every lane of a wave adds to the same address
    grad = torch.randn(N, generator=g0)
    hess = torch.rand(N, generator=g0) * 0.25
    rows = torch.randperm(N, generator=g0).int()
    seg = torch.tensor([0, 777, 20_000, N], dtype=torch.int32)
    args = (bins.cuda(), grad.cuda(), hess.cuda(), rows.cuda(), seg.cuda(), B, rpb)
    try:
        ext.set_gbdt_hist_rows(0)
        slot = ext.gbdt_hist_quant(*args).cpu()
        outs = []
        for u in (4, 8):
            for pack in (1, 0):  # g and h in one 64-bit LDS add (default) / two 32-bit adds
                ext.set_gbdt_hist_rows(u)
                ext.set_gbdt_pack64(pack)
                outs.append(ext.gbdt_hist_quant(*args).cpu())
    finally:
        ext.set_gbdt_hist_rows(-2)
        ext.set_gbdt_pack64(-1)
    for got in outs:
        torch.testing.assert_close(got, slot, rtol=1e-5, atol=1e-5)
    # and both are the histogram: counts of the hot bin
    torch.testing.assert_close(outs[0][:, 0, 3, 1].double().sum(), hess.double().sum(), rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("rpb", [2048, 4096])
def test_gpu_quantised_hist_tiny_and_skewed_hessians(rpb):
    """the device grower sums fixed-point integers per block (step =
    rpb * max / 2^30 per row).  With skewed gradients and hessians spanning
    1e-9 .. 0.25 (confidently classified logistic rows next to uncertain ones)
    every bin's G and H stay within half a step per row of the fp64 sums, and
    the best split per (node, feature) at lambda = 1 is the fp64 one."""
    from kubedl_amd.ops import _ext
    ext = _ext.load()
    g0 = torch.Generator().manual_seed(7)
    N, F, B = 100_000, 8, 64
    bins = torch.randint(0, B, (N, F), generator=g0, dtype=torch.uint8)
    grad = torch.randn(N, generator=g0) * 1e-3
    hot = torch.rand(N, generator=g0) < 0.01
    grad[hot] = torch.sign(torch.randn(int(hot.sum()), generator=g0))
    hess = torch.exp(torch.empty(N).uniform_(-20.7, -13.8, generator=g0))  # 1e-9 .. 1e-6
    big = torch.rand(N, generator=g0) < 0.1
    hess[big] = 0.25
    rows = torch.randperm(N, generator=g0).int()
    seg = torch.tensor([0, 30_000, N], dtype=torch.int32)
    got = ext.gbdt_hist_quant(bins.cuda(), grad.cuda(), hess.cuda(), rows.cuda(), seg.cuda(), B, rpb).cpu().double()
    ref = torch.zeros(2, F, B, 2, dtype=torch.float64)
    cnt = torch.zeros(2, F, B, dtype=torch.float64)
    for j in range(2):
        r = rows[seg[j]:seg[j + 1]].long()
        for f in range(F):
            b = bins[r, f].long()
            ref[j, f, :, 0].index_add_(0, b, grad[r].double())
            ref[j, f, :, 1].index_add_(0, b, hess[r].double())
            cnt[j, f].index_add_(0, b, torch.ones(len(r), dtype=torch.float64))
    step_g = rpb * float(grad.abs().max()) / 2 ** 30
    step_h = rpb * float(hess.max()) / 2 ** 30
    for k, step in ((0, step_g), (1, step_h)):
        bound = 0.5 * step * cnt + 1e-6 * ref[..., k].abs() + 1e-9
        err = (got[..., k] - ref[..., k]).abs()
        assert bool((err <= bound).all()), (k, float((err - bound).max()))
    # the split the grower would take: G^2 / (H + lambda) over every bin boundary
    lam = 1.0

    def best(h):
        G, H = h[..., 0].cumsum(-1), h[..., 1].cumsum(-1)
        Gt, Ht = G[..., -1:], H[..., -1:]
        gain = G ** 2 / (H + lam) + (Gt - G) ** 2 / (Ht - H + lam) - Gt ** 2 / (Ht + lam)
        return gain[..., :-1].argmax(-1)
    assert torch.equal(best(got), best(ref))


@pytest.mark.gpu
def test_gpu_long_logistic_fit_matches_cpu_grower():
    """a 40-round depth-6 logistic fit on the device grower (integer
    histograms) reaches the CPU torch grower's (fp32 histograms) log-loss and
    accuracy: late, deep trees whose rows carry tiny hessians are not biased."""
    X, y = _data(30_000, 10, seed=3)
    kw = dict(objective="binary:logistic", n_estimators=40, max_depth=6, max_bin=64)
    cpu = HistGBDT(GBDTParams(**kw), "cpu")
    cpu.fit_cuts(X, sample=len(X))
    mc = cpu.metric(cpu.fit(X, y), y)
    gpu = HistGBDT(GBDTParams(**kw), "cuda")
    gpu.cuts = cpu.cuts.cuda()
    mg = gpu.metric(gpu.fit(X, y), y.cuda())
    assert abs(mg["logloss"] - mc["logloss"]) <= 0.02 * mc["logloss"], (mg, mc)
    assert abs(mg["accuracy"] - mc["accuracy"]) <= 0.005, (mg, mc)
