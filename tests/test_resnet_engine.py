"""The explicit ResNet engine (models/resnet_engine.py) vs the autograd model.

CPU: the engine's TorchKernels backend (same data flow as the HIP path,
plain fp32 PyTorch ops) against autograd on small ResNets, bf16 storage.
GPU: the HipKernels backend (fused 1x1-conv GEMMs + staged BN kernels)
against the autograd model with the eager-PyTorch BN, at ResNet-50 widths.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

from kubedl_amd.models.resnet import ResNet
from kubedl_amd.models.resnet_engine import ResNetEngine


def _setup(layers, width, dev, image, batch, classes=10, seed=0):
    torch.manual_seed(seed)
    model = ResNet(layers, num_classes=classes, width=width)
    # non-trivial BN affine params so masks and scales matter
    with torch.no_grad():
        for m in model.modules():
            if hasattr(m, "running_mean"):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    model = model.to(dev)
    if dev == "cuda":
        model = model.to(memory_format=torch.channels_last)
    for p in model.parameters():
        p.data = p.data.to(torch.bfloat16)
    ref = copy.deepcopy(model)
    ref.set_bn_backend("torch")
    x = torch.randn(batch, 3, image, image, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, classes, (batch,), device=dev)
    return model, ref, x, y


def _ref_step(ref, x, y):
    out = ref(x)
    loss = F.cross_entropy(out.float(), y)
    loss.backward()
    return loss.detach()


def _compare(model, ref, loss, rloss, gtol, stat_tol=2e-2, cos_min=0.99):
    torch.testing.assert_close(loss.float(), rloss.float(), atol=2e-2, rtol=2e-2)
    worst = []
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        g, r = p.grad.float(), q.grad.float()
        scale = r.abs().max().item() + 1e-6
        err = (g - r).abs().max().item() / scale
        cos = F.cosine_similarity(g.flatten(), r.flatten(), dim=0).item()
        worst.append((err, cos, n))
        assert cos > cos_min, f"{n}: cosine {cos:.4f} (rel max err {err:.3f})"
        assert err < gtol, f"{n}: rel max err {err:.3f} (cos {cos:.4f})"
    for (n, b), (_, c) in zip(model.named_buffers(), ref.named_buffers()):
        torch.testing.assert_close(b.float(), c.float(), atol=stat_tol, rtol=stat_tol, msg=n)
    return worst


@pytest.mark.parametrize("layers,width", [((1, 1, 1, 1), 8), ((2, 1, 1, 2), 8), ((1, 1, 1, 1), 64)])
def test_engine_torch_backend_matches_autograd_fp32(layers, width, monkeypatch):
    """Exact data-flow check: fp32 storage, no bf16 rounding points.  Width 64
    puts every 3x3 on the native branches (stride-2 data gradient with the
    mask + sums fused, as the HIP sub-pixel class GEMMs)."""
    import kubedl_amd.models.resnet_engine as RE
    monkeypatch.setattr(RE, "_bfr", lambda t: t.float())
    torch.manual_seed(0)
    model = ResNet(layers, num_classes=10, width=width)
    with torch.no_grad():
        for m in model.modules():
            if hasattr(m, "running_mean"):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    ref = copy.deepcopy(model)
    ref.set_bn_backend("torch")
    x = torch.randn(4, 3, 64, 64)
    y = torch.randint(0, 10, (4,))
    loss = RE.ResNetEngine(model, backend="torch").forward_backward(x, y)
    rloss = _ref_step(ref, x, y)
    torch.testing.assert_close(loss, rloss, atol=1e-5, rtol=1e-5)
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad, atol=1e-4 * (q.grad.abs().max().item() + 1e-6), rtol=1e-3,
                                   msg=n)
    for (n, b), (_, c) in zip(model.named_buffers(), ref.named_buffers()):
        torch.testing.assert_close(b, c, atol=1e-5, rtol=1e-5, msg=n)


def test_engine_width8_stack_matches_autograd_fp32(monkeypatch):
    """A (3, 2, 2, 2) width-8 stack (stage-1 blocks without downsample, stride-2
    blocks at every later stage) is exact in fp32: the same gradients and BN
    buffers as autograd."""
    import kubedl_amd.models.resnet_engine as RE
    monkeypatch.setattr(RE, "_bfr", lambda t: t.float())
    monkeypatch.delenv("KDL_ENGINE", raising=False)
    torch.manual_seed(0)
    model = ResNet((3, 2, 2, 2), num_classes=10, width=8)
    with torch.no_grad():
        for m in model.modules():
            if hasattr(m, "running_mean"):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    ref = copy.deepcopy(model)
    ref.set_bn_backend("torch")
    x = torch.randn(4, 3, 64, 64)
    y = torch.randint(0, 10, (4,))
    eng = RE.ResNetEngine(model, backend="torch")
    loss = eng.forward_backward(x, y)
    rloss = _ref_step(ref, x, y)
    torch.testing.assert_close(loss, rloss, atol=1e-5, rtol=1e-5)
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad, atol=1e-4 * (q.grad.abs().max().item() + 1e-6), rtol=1e-3,
                                   msg=n)
    for (n, b), (_, c) in zip(model.named_buffers(), ref.named_buffers()):
        torch.testing.assert_close(b, c, atol=1e-5, rtol=1e-5, msg=n)


def _vs_truth(model, ref, truth, slack=1.5, add=0.05):
    """bf16 engine error vs an fp32 autograd 'truth' must be comparable to the
    bf16 autograd model's own error (small-batch BN backward amplifies bf16
    rounding a lot, for both)."""
    for (n, p), (_, q), (_, t) in zip(model.named_parameters(), ref.named_parameters(),
                                      truth.named_parameters()):
        tt = t.grad.float()
        ee = ((p.grad.float() - tt).norm() / (tt.norm() + 1e-12)).item()
        er = ((q.grad.float() - tt).norm() / (tt.norm() + 1e-12)).item()
        assert ee <= slack * er + add, f"{n}: engine rel-L2 {ee:.3f} vs autograd {er:.3f}"
    for (n, b), (_, c), (_, t) in zip(model.named_buffers(), ref.named_buffers(), truth.named_buffers()):
        tt = t.float()
        ee = ((b.float() - tt).norm() / (tt.norm() + 1e-12)).item()
        er = ((c.float() - tt).norm() / (tt.norm() + 1e-12)).item()
        assert ee <= slack * er + 0.01, f"{n}: engine rel-L2 {ee:.4f} vs autograd {er:.4f}"


def _vs_truth_strict(model, ref, truth, slack=1.5, add=0.01, cos_min=0.999):
    """the full-network check leaves a localized bug nowhere
    to hide -- per parameter, cosine to the fp32 truth >= ``cos_min`` (or no
    worse than bf16 autograd's own cosine minus 1e-3 where bf16 itself cannot
    reach it), and rel-L2 within ``slack`` x autograd's + ``add`` (1 %)."""
    worst = []
    for (n, p), (_, q), (_, t) in zip(model.named_parameters(), ref.named_parameters(),
                                      truth.named_parameters()):
        tt = t.grad.float().flatten()
        pe, pr = p.grad.float().flatten(), q.grad.float().flatten()
        ce = torch.nn.functional.cosine_similarity(pe, tt, dim=0).item()
        cr = torch.nn.functional.cosine_similarity(pr, tt, dim=0).item()
        ee = ((pe - tt).norm() / (tt.norm() + 1e-12)).item()
        er = ((pr - tt).norm() / (tt.norm() + 1e-12)).item()
        worst.append((ce, n, cr, ee, er))
        # the engine's angular error within 1.5x bf16 autograd's + 1e-3 (the same
        # slack as the rel-L2 bound): a fixed "cr - 1e-3" fails on run-to-run
        # rounding noise wherever bf16 itself is far from the truth (BN weights of
        # the 7x7 stage at cosine ~0.73: engine 0.731 vs autograd 0.734 on one
        # run; the stem BN weight at 0.04-0.26 for both, same seed, different
        # boxes); where bf16 autograd reaches >= 0.999 this is ce >= ~0.998
        # Where bf16 autograd itself is below cosine 0.9 the gradient is rounding noise
        # (a BN weight of a stage-1 block at 0.43 for autograd), and the engine's
        # cosine is a different draw of that noise (0.02 once in five runs, bit-identical
        # forward): there only the rel-L2 bound below applies -- it still fails a
        # localized bug, whose error is not noise-sized
        if cr >= 0.9:
            assert ce >= min(cos_min, 1.0 - 1.5 * (1.0 - cr) - 1e-3), f"{n}: engine cosine {ce:.5f} vs autograd {cr:.5f}"
        assert ee <= slack * er + add, f"{n}: engine rel-L2 {ee:.4f} vs autograd {er:.4f}"
    worst.sort()
    print("lowest engine cosines:", [(n, round(ce, 5), round(cr, 5)) for ce, n, cr, _, _ in worst[:5]])
    for (n, b), (_, c), (_, t) in zip(model.named_buffers(), ref.named_buffers(), truth.named_buffers()):
        tt = t.float()
        ee = ((b.float() - tt).norm() / (tt.norm() + 1e-12)).item()
        er = ((c.float() - tt).norm() / (tt.norm() + 1e-12)).item()
        assert ee <= slack * er + 0.01, f"{n}: engine rel-L2 {ee:.4f} vs autograd {er:.4f}"


def _truth_of(ref, x, y):
    truth = copy.deepcopy(ref).float()
    for p in truth.parameters():
        p.data = p.data.float()
        p.grad = None
    return truth, _ref_step(truth, x.float(), y)


def test_engine_torch_backend_bf16_close_to_autograd():
    model, ref, x, y = _setup((2, 1, 1, 2), 16, "cpu", 64, 8)
    truth, tloss = _truth_of(ref, x, y)
    loss = ResNetEngine(model, backend="torch").forward_backward(x, y)
    _ref_step(ref, x, y)
    torch.testing.assert_close(loss, tloss, atol=2e-2, rtol=2e-2)
    _vs_truth(model, ref, truth)


@pytest.mark.gpu
@pytest.mark.parametrize("wgrad_stream", ["0", "1"])
@pytest.mark.parametrize("layers,image,batch", [((1, 1, 1, 1), 64, 8), ((2, 2, 2, 2), 96, 4)])
def test_engine_hip_matches_autograd(layers, image, batch, wgrad_stream, monkeypatch):
    """``wgrad_stream=1``: weight gradients on the engine's second stream,
    concurrent with the main stream's BN-backward / data-gradient kernels (a
    race there -- a wgrad reading a coefficient block or operand the main
    stream rewrites -- shows up as a gradient far off the fp32 truth).  The two
    schedules are not compared with each other: the first MIOpen call of a
    process may pick a different solver, so runs differ at bf16-noise level."""
    monkeypatch.setenv("KDL_ENGINE", f"side={wgrad_stream}")
    model, ref, x, y = _setup(layers, 64, "cuda", image, batch)
    truth, tloss = _truth_of(ref, x, y)
    eng = ResNetEngine(model, backend="hip")
    assert (eng.side is not None) == (wgrad_stream == "1")
    loss = eng.forward_backward(x, y)
    _ref_step(ref, x, y)
    torch.cuda.synchronize()
    torch.testing.assert_close(loss, tloss, atol=2e-2, rtol=2e-2)
    _vs_truth(model, ref, truth)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [32, 256])
def test_engine_hip_full_resnet50_224_matches_fp32_truth(batch):
    """The shape the bench times: the full (3, 4, 6, 3) ResNet-50 at 224 px
    (56 -> 28 -> 14 -> 7 geometry, stride-2 3x3 convs and strided downsample
    GEMMs), every GEMM on the kdl kernels (LDS-DMA implicit GEMMs for the 3x3
    forward / weight gradients and the long-K 1x1s), weight gradients on the
    side stream -- against fp32 autograd truth, with the same error budget as
    the bf16 autograd model.  Batch 256 is the benchmarked shape itself
    (tile selection and grid sizes change with the batch,
    the round-3 stride-2 MASKX bug existed only there)."""
    model, ref, x, y = _setup((3, 4, 6, 3), 64, "cuda", 224, batch, classes=1000)
    truth, tloss = _truth_of(ref, x, y)
    eng = ResNetEngine(model, backend="hip")
    assert eng.side is not None
    loss = eng.forward_backward(x, y)
    _ref_step(ref, x, y)
    torch.cuda.synchronize()
    torch.testing.assert_close(loss, tloss, atol=2e-2, rtol=2e-2)
    _vs_truth_strict(model, ref, truth)


def _ddp_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    from kubedl_amd.parallel.dist import DistInfo
    from kubedl_amd.workers.resnet50 import ResNetTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    info = DistInfo(rank, world, rank, torch.device("cpu"), "gloo")
    tr = ResNetTrainer(info, batch=2, image=32, num_classes=10, tiny=True, engine="fused",
                       bucket_cap_mb=0.05, seed=0)
    losses = [float(tr.step()) for _ in range(2)]
    # numpy, not tensors: a tensor in a Queue is shared through an fd that dies with this process
    q.put((rank, losses, tr.space.master.numpy().copy(), tr.space.grad.float().numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_engine_ddp_gloo_two_ranks():
    """Direct-mode DDP: the engine announces finished gradients, buckets all-reduce
    during the backward, and both ranks end with identical weights."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (_, l0, m0, g0), (_, l1, m1, g1) = res
    m0, m1, g0, g1 = (torch.as_tensor(a) for a in (m0, m1, g0, g1))
    assert l0 != l1  # different data per rank
    torch.testing.assert_close(m0, m1, atol=0, rtol=0)
    torch.testing.assert_close(g0, g1, atol=0, rtol=0)  # all-reduced
    assert g0.abs().sum() > 0


def _ddp_worker_gpu(rank, world, port, q):
    import os
    import torch.distributed as dist
    from kubedl_amd.parallel.dist import DistInfo
    from kubedl_amd.workers.resnet50 import ResNetTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)  # two ranks share the one GPU of the box
    info = DistInfo(rank, world, 0, torch.device("cuda", 0), "gloo")
    tr = ResNetTrainer(info, batch=4, image=64, num_classes=10, bn_backend="hip", engine="fused",
                       bucket_cap_mb=4.0, seed=0)
    assert tr.engine is not None and tr.engine.K.name == "hip"
    losses = [float(tr.step()) for _ in range(2)]
    torch.cuda.synchronize()
    # numpy copies: pickled by value (a torch CPU tensor would be shared by fd from a process that exits)
    q.put((rank, losses, tr.space.master.cpu().numpy(), tr.space.grad.float().cpu().numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_engine_ddp_two_ranks_hip_gpu():
    """The HIP engine's direct-mode DDP on the GPU: buckets launched from inside
    the fused backward, all-reduced across two ranks (gloo on one MI355X: the
    8-GPU RCCL run is the driver's), identical weights afterwards."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker_gpu, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(2)), key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (_, l0, m0, g0), (_, l1, m1, g1) = res
    m0, m1, g0, g1 = (torch.from_numpy(a) for a in (m0, m1, g0, g1))
    assert all(x == x for x in l0 + l1)
    assert l0 != l1
    torch.testing.assert_close(m0, m1, atol=0, rtol=0)
    torch.testing.assert_close(g0, g1, atol=0, rtol=0)
    assert g0.abs().sum() > 0


@pytest.mark.gpu
def test_engine_bn_finalize_in_gemm_matches_kernel_finalize(monkeypatch):
    """BN finalize folded into the producing GEMMs' last arriving blocks
    (csrc/bn_fin.h, KDL_ENGINE=bn_fin=gemm) vs the separate finalize launches
    (KDL_ENGINE=bn_fin=kernel): the difference must be at the level of two runs of the
    same mode (replica atomics make BN sums order-nondeterministic)."""
    results = []
    for mode in ("kernel", "kernel", "gemm"):
        monkeypatch.setenv("KDL_ENGINE", f"bn_fin={mode}")
        model, ref, x, y = _setup((2, 2, 2, 2), 64, "cuda", 112, 16, classes=10, seed=3)
        eng = ResNetEngine(model, backend="hip")
        assert eng.K.fuse_fin == (mode == "gemm")
        loss = eng.forward_backward(x, y)
        torch.cuda.synchronize()
        results.append((float(loss), {n: p.grad.float().clone() for n, p in model.named_parameters()},
                        {n: b.float().clone() for n, b in model.named_buffers()}))

    def rel(a, b):
        return {n: ((a[n] - b[n]).norm() / (b[n].norm() + 1e-12)).item() for n in b}
    noise = rel(results[1][1], results[0][1])
    fused = rel(results[2][1], results[0][1])
    worst = sorted(fused, key=lambda n: -fused[n])[:8]
    report = "; ".join(f"{n}: fused {fused[n]:.2e} noise {noise[n]:.2e}" for n in worst)
    # forward BN statistics are replica-atomic sums in both modes: the loss moves by
    # ~1e-3 relative between two runs of one mode at this tiny batch (16 x 112 px)
    loss_noise = abs(results[1][0] - results[0][0])
    assert abs(results[2][0] - results[0][0]) < max(3e-3 * max(1.0, abs(results[0][0])), 3 * loss_noise), report
    for n in fused:
        assert fused[n] <= 3 * noise[n] + 2e-3, report
    bnoise = rel(results[1][2], results[0][2])
    bfused = rel(results[2][2], results[0][2])
    for n in bfused:
        assert bfused[n] <= 3 * bnoise[n] + 1e-4, (n, bfused[n], bnoise[n])


def test_engine_options_from_one_variable(monkeypatch):
    """the engine's schedule variants are one dataclass whose
    defaults are the measured winners; A/B overrides come from KDL_ENGINE only."""
    from kubedl_amd.models.resnet_engine import EngineOptions
    monkeypatch.delenv("KDL_ENGINE", raising=False)
    assert EngineOptions.from_env() == EngineOptions()
    monkeypatch.setenv("KDL_ENGINE", "side=0, res_pro_kmax=256,bn_fin=kernel,halo_pro=0")
    o = EngineOptions.from_env()
    assert (o.side, o.res_pro_kmax, o.bn_fin, o.halo_pro) == (False, 256, "kernel", 0)
    monkeypatch.setenv("KDL_ENGINE", "no_such_knob=1")
    with pytest.raises(ValueError, match="unknown option"):
        EngineOptions.from_env()


def test_knob_surface_stays_small():
    """A/B switches live in KDL_TUNE / KDL_ENGINE; every other
    KDL_* name in the package and the native sources is part of the runtime
    contract (pod env, rendezvous, paths) -- fewer than 40 distinct names."""
    import pathlib
    import re
    root = pathlib.Path(__file__).resolve().parents[1]
    names = set()
    for sub, pats in (("kubedl_amd", ("*.py",)), ("csrc", ("*.hip", "*.cpp", "*.h"))):
        for pat in pats:
            for f in (root / sub).rglob(pat):
                names |= set(re.findall(r"KDL_[A-Z0-9_]+", f.read_text(errors="ignore")))
    # the retired names are listed once, only to warn about them (utils/tune.py RETIRED_ENV)
    from kubedl_amd.utils.tune import RETIRED_ENV, warn_retired_env
    names -= set(RETIRED_ENV)
    assert len(names) < 40, sorted(names)
    for gone in ("KDL_HIP_GRAPH", "KDL_GBDT_GRAPH", "KDL_STREAMS", "KDL_MAIN_PRIO", "KDL_DDP_WORLD1"):
        assert gone not in names
    # a retired variable is reported (once), naming its KDL_TUNE key
    import io
    import kubedl_amd.utils.tune as tmod
    tmod._WARNED[0] = False
    buf = io.StringIO()
    import os as _os
    old = _os.environ.get("KDL_STREAMS")
    _os.environ["KDL_STREAMS"] = "dedicated"
    try:
        assert warn_retired_env(buf) == ["KDL_STREAMS"]
        assert 'KDL_TUNE="streams=dedicated"' in buf.getvalue()
        assert warn_retired_env(buf) == ["KDL_STREAMS"] and buf.getvalue().count("retired") == 1
    finally:
        if old is None:
            _os.environ.pop("KDL_STREAMS")
        else:
            _os.environ["KDL_STREAMS"] = old


@pytest.mark.parametrize("mode", [1, 3])
@pytest.mark.parametrize("layers,width", [((1, 1, 1, 1), 8), ((2, 1, 1, 2), 16)])
def test_engine_gram_fold_matches_autograd_fp32(layers, width, mode, monkeypatch):
    """bn_bwd_fuse=3 (default): conv3's weight gradient as diag(k) g^T a2 +
    diag(c1) W3 (a2^T a2) + c0 (1^T a2) -- dc3 never materialised -- is the same
    gradient, exactly in fp32 (the algebra of HipKernels.wgrad_gram); 1: the
    written-through dc3."""
    import kubedl_amd.models.resnet_engine as RE
    monkeypatch.setattr(RE, "_bfr", lambda t: t.float())
    monkeypatch.setenv("KDL_ENGINE", f"bn_bwd_fuse={mode}")
    torch.manual_seed(1)
    model = ResNet(layers, num_classes=10, width=width)
    with torch.no_grad():
        for m in model.modules():
            if hasattr(m, "running_mean"):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    ref = copy.deepcopy(model)
    ref.set_bn_backend("torch")
    x = torch.randn(4, 3, 64, 64)
    y = torch.randint(0, 10, (4,))
    eng = RE.ResNetEngine(model, backend="torch")
    assert eng.fuse_bwd == mode
    loss = eng.forward_backward(x, y)
    rloss = _ref_step(ref, x, y)
    torch.testing.assert_close(loss, rloss, atol=1e-5, rtol=1e-5)
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad, atol=1e-4 * (q.grad.abs().max().item() + 1e-6), rtol=1e-3,
                                   msg=n)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [32, 256])
def test_engine_hip_write_through_full_resnet50_matches_fp32_truth(batch, monkeypatch):
    """bn_bwd_fuse=1 -- conv3's weight gradient from the written-through dc3
    instead of the default Gram fold (csrc/conv1x1.hip conv1x1_gram + gram_fold)
    -- on the benchmarked shape, against fp32 truth with the default's budget."""
    monkeypatch.setenv("KDL_ENGINE", "bn_bwd_fuse=1")
    model, ref, x, y = _setup((3, 4, 6, 3), 64, "cuda", 224, batch, classes=1000)
    truth, tloss = _truth_of(ref, x, y)
    eng = ResNetEngine(model, backend="hip")
    assert eng.fuse_bwd == 1
    loss = eng.forward_backward(x, y)
    _ref_step(ref, x, y)
    torch.cuda.synchronize()
    torch.testing.assert_close(loss, tloss, atol=2e-2, rtol=2e-2)
    _vs_truth_strict(model, ref, truth)


@pytest.mark.gpu
@pytest.mark.parametrize("M,K", [(802816, 64), (200704, 128), (1000, 64), (4160, 128)])
def test_conv1x1_gram_matches_fp32(M, K):
    """Q = a^T a and s = 1^T a of a = bf16(relu(x * scale + shift)) (the conv3
    prologue's operand) against fp32 torch, including M tails."""
    from kubedl_amd.ops import _ext
    ext = _ext.load()
    g = torch.Generator(device="cuda").manual_seed(M)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    pro = torch.cat([torch.rand(K, device="cuda", generator=g) + 0.5, torch.randn(K, device="cuda", generator=g) * 0.3])
    ws = torch.empty(ext.conv1x1_gram_floats(M, K), device="cuda")
    ext.conv1x1_gram(x, pro, ws, M, K)
    a = (x.float() * pro[:K] + pro[K:]).relu().bfloat16().float()
    Q, s = a.t() @ a, a.sum(0)
    torch.testing.assert_close(ws[: K * K].view(K, K), Q, atol=1e-3 * Q.abs().max().item(), rtol=1e-4)
    torch.testing.assert_close(ws[K * K: K * K + K], s, atol=1e-3 * s.abs().max().item(), rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("N,K", [(256, 64), (512, 128), (2048, 512)])
def test_gram_fold_matches_fp32(N, K):
    """gram_fold: k G + c1 (W Q) + c0 s per output row, against fp32 torch."""
    from kubedl_amd.ops import _ext
    ext = _ext.load()
    g = torch.Generator(device="cuda").manual_seed(N + K)
    G = torch.randn(N, K, device="cuda", generator=g)
    QS = torch.randn(K * K + K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g).bfloat16()
    bc = torch.randn(3 * N, device="cuda", generator=g)
    out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    ext.gram_fold(G, QS, W, bc, out, N, K)
    Q, s = QS[: K * K].view(K, K), QS[K * K:]
    ref = bc[:N, None] * G + bc[N: 2 * N, None] * (W.float() @ Q) + bc[2 * N:, None] * s[None]
    torch.testing.assert_close(out.float(), ref, atol=2e-2 * ref.abs().max().item(), rtol=1e-2)
