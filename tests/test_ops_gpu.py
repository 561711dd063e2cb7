"""Numerics of the HIP kernels vs plain PyTorch fp32 references (MI355X only)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ext():
    from kubedl_amd.ops import _ext
    return _ext.load()


def _ref_bn_act(x, w, b, rm, rv, res, relu, training, momentum=0.1, eps=1e-5):
    y = F.batch_norm(x.double(), rm, rv, w.double(), b.double(), training=training,
                     momentum=momentum, eps=eps)
    if res is not None:
        y = y + res.double()
    if relu:
        y = F.relu(y)
    return y


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(4, 64, 14, 14), (2, 256, 7, 7), (3, 24, 5, 5), (8, 2048, 7, 7),
                                   (2, 3000, 2, 2)])
@pytest.mark.parametrize("relu,residual", [(True, False), (True, True), (False, False)])
@pytest.mark.parametrize("training", [True, False])
def test_bn_act_matches_reference(dtype, shape, relu, residual, training):
    from kubedl_amd.ops.bn import batch_norm_act
    torch.manual_seed(0)
    dev = "cuda"
    N, C, H, W = shape
    x = (torch.randn(shape, device=dev) * 2 + 3).to(dtype).contiguous(memory_format=torch.channels_last)
    r = torch.randn(shape, device=dev).to(dtype).contiguous(memory_format=torch.channels_last) if residual else None
    w = (torch.rand(C, device=dev) + 0.5).to(dtype)
    b = torch.randn(C, device=dev).to(dtype)
    rm = torch.randn(C, device=dev)
    rv = torch.rand(C, device=dev) + 0.5
    rm_ref, rv_ref = rm.double().clone(), rv.double().clone()
    x.requires_grad_(True)
    w.requires_grad_(True)
    b.requires_grad_(True)
    if r is not None:
        r.requires_grad_(True)
    y = batch_norm_act(x, w, b, rm, rv, residual=r, relu=relu, training=training, backend="hip")
    xr = x.detach().double().requires_grad_(True)
    wr = w.detach().double().requires_grad_(True)
    br = b.detach().double().requires_grad_(True)
    rr = r.detach().double().requires_grad_(True) if r is not None else None
    yr = _ref_bn_act(xr, wr, br, rm_ref, rv_ref, rr, relu, training)
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.double(), yr, atol=tol, rtol=tol)
    torch.testing.assert_close(rm.double(), rm_ref, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(rv.double(), rv_ref, atol=1e-3, rtol=1e-3)
    g = torch.randn_like(y, dtype=torch.float32).to(dtype)
    y.backward(g)
    yr.backward(g.double())
    gtol = 5e-2 if dtype == torch.bfloat16 else 2e-3
    torch.testing.assert_close(x.grad.double(), xr.grad, atol=gtol, rtol=gtol)
    scale = max(1.0, float(wr.grad.abs().max()))
    torch.testing.assert_close(w.grad.double() / scale, wr.grad / scale, atol=gtol, rtol=gtol)
    scale = max(1.0, float(br.grad.abs().max()))
    torch.testing.assert_close(b.grad.double() / scale, br.grad / scale, atol=gtol, rtol=gtol)
    if r is not None:
        torch.testing.assert_close(r.grad.double(), rr.grad, atol=gtol, rtol=gtol)


def test_bn_large_mean_stability():
    """Shifted-sum stats must survive |mean| >> std (no catastrophic cancellation)."""
    from kubedl_amd.ops.bn import batch_norm_act
    torch.manual_seed(1)
    x = (torch.randn(64, 64, 28, 28, device="cuda") * 0.01 + 100.0).contiguous(
        memory_format=torch.channels_last)
    w = torch.ones(64, device="cuda")
    b = torch.zeros(64, device="cuda")
    y = batch_norm_act(x, w, b, torch.zeros(64, device="cuda"), torch.ones(64, device="cuda"),
                       relu=False, backend="hip")
    yr = _ref_bn_act(x, w, b, None, None, None, False, True)
    torch.testing.assert_close(y.double(), yr, atol=2e-3, rtol=2e-3)


def _flat_case(dev, dtype):
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(37, 64), torch.nn.ReLU(), torch.nn.Linear(64, 10),
                            torch.nn.BatchNorm1d(10)).to(dev)
    with torch.no_grad():
        for p in m.parameters():
            p.data = p.data.to(dtype)
    return m


@pytest.mark.parametrize("nesterov", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fused_sgd_matches_cpu_path(nesterov, dtype):
    from kubedl_amd.ops.optim import FlatParamSpace, FusedSGD
    res = {}
    for dev in ["cpu", "cuda"]:
        m = _flat_case(dev, dtype)
        sp = FlatParamSpace(m)
        opt = FusedSGD(sp, lr=0.05, momentum=0.9, weight_decay=1e-3, nesterov=nesterov)
        opt.grad_scale = 0.5
        g = torch.Generator().manual_seed(3)
        for _ in range(3):
            sp.grad.copy_(torch.randn(sp.numel, generator=g).to(dtype))
            opt.step()
        res[dev] = torch.cat([sp._view(sp.master, sl).reshape(-1) for sl in sp.slots]).cpu()
        assert sp.param.dtype == dtype
    torch.testing.assert_close(res["cuda"], res["cpu"], atol=1e-5, rtol=1e-5)


def test_fused_sgd_matches_torch_optim():
    from kubedl_amd.ops.optim import FlatParamSpace, FusedSGD
    torch.manual_seed(0)
    m1 = torch.nn.Linear(64, 32).cuda()
    m2 = torch.nn.Linear(64, 32).cuda()
    m2.load_state_dict(m1.state_dict())
    sp = FlatParamSpace(m1, no_decay=lambda n, p: False)
    opt = FusedSGD(sp, lr=0.1, momentum=0.9, weight_decay=1e-4)
    ref = torch.optim.SGD(m2.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(16, 64, device="cuda")
    for _ in range(4):
        opt.zero_grad()
        m1(x).square().sum().backward()
        opt.step()
        ref.zero_grad()
        m2(x).square().sum().backward()
        ref.step()
    torch.testing.assert_close(m1.weight, m2.weight, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(m1.bias, m2.bias, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("adam_w", [True, False])
def test_fused_adam_matches_torch_optim(adam_w):
    from kubedl_amd.ops.optim import FlatParamSpace, FusedAdam
    torch.manual_seed(0)
    m1 = torch.nn.Linear(64, 32).cuda()
    m2 = torch.nn.Linear(64, 32).cuda()
    m2.load_state_dict(m1.state_dict())
    sp = FlatParamSpace(m1, no_decay=lambda n, p: False)
    opt = FusedAdam(sp, lr=1e-2, weight_decay=1e-2, adam_w=adam_w)
    cls = torch.optim.AdamW if adam_w else torch.optim.Adam
    ref = cls(m2.parameters(), lr=1e-2, weight_decay=1e-2)
    x = torch.randn(16, 64, device="cuda")
    for _ in range(5):
        opt.zero_grad()
        m1(x).square().sum().backward()
        opt.step()
        ref.zero_grad()
        m2(x).square().sum().backward()
        ref.step()
    torch.testing.assert_close(m1.weight, m2.weight, atol=1e-5, rtol=1e-4)


def test_extension_is_native():
    ext = _ext()
    assert ext.arch == "gfx950"
    import kubedl_amd
    assert ext.__file__.startswith(kubedl_amd.__path__[0])


def test_pack_grads_matches_views():
    """Multi-tensor gather (csrc/multi_tensor.hip) == the per-parameter copy."""
    from kubedl_amd.ops.optim import FlatParamSpace
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3), torch.nn.Conv2d(16, 5, 1),
                            torch.nn.Flatten(), torch.nn.LazyLinear(7)).cuda()
    m(torch.randn(2, 3, 9, 9, device="cuda"))
    m = m.to(memory_format=torch.channels_last)
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    sp = FlatParamSpace(m, grad_mode="pack")
    m[0].bias.requires_grad_(True)
    sp.zero_grad()
    x = torch.randn(2, 3, 9, 9, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    m(x).float().square().sum().backward()
    grads = {s.name: (s.param.grad.clone() if s.param.grad is not None else None) for s in sp.slots}
    sp.pack_grads()
    for s in sp.slots:
        view = sp._view(sp.grad, s)
        if grads[s.name] is None:
            assert torch.count_nonzero(view) == 0
        else:
            torch.testing.assert_close(view, grads[s.name], atol=0, rtol=0)


@pytest.mark.parametrize("nparams", [5, 300])
def test_pack_grads_pointer_args_and_table(nparams):
    """<= pack_arg_ptrs tensors: source pointers as kernel arguments; more: the
    uploaded device table.  Both gather exactly the per-parameter gradients,
    zeros for a parameter without one."""
    from kubedl_amd.ops.optim import FlatParamSpace
    torch.manual_seed(1)
    ext = _ext()
    assert (nparams <= ext.pack_arg_ptrs) == (nparams == 5)
    m = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(3 + i % 7, device="cuda")) for i in range(nparams)])
    sp = FlatParamSpace(m, grad_mode="pack")
    for _ in range(2):  # twice: the second call reuses the packer
        sp.zero_grad()
        loss = sum((p * (i + 1)).sum() for i, p in enumerate(m) if i % 11 != 3)
        loss.backward()
        sp.pack_grads()
        for i, s in enumerate(sp.slots):
            view = sp._view(sp.grad, s)
            if s.param.grad is None:
                assert torch.count_nonzero(view) == 0
            else:
                torch.testing.assert_close(view, s.param.grad, atol=0, rtol=0)


def test_bn_workspace_is_self_cleaning():
    """A persistent per-layer workspace (replicated accumulators re-zeroed by the
    finalize kernels) gives the same results on every reuse as a fresh one."""
    from kubedl_amd.ops.bn import batch_norm_act, workspace_for
    torch.manual_seed(0)
    C = 96
    ws = workspace_for(C, "cuda")
    w = torch.rand(C, device="cuda") + 0.5
    b = torch.randn(C, device="cuda")
    for it in range(3):
        x = torch.randn(8, C, 6, 6, device="cuda").contiguous(memory_format=torch.channels_last)
        outs = []
        for use_ws in (None, ws):
            xi = x.clone().requires_grad_(True)
            wi = w.clone().requires_grad_(True)
            bi = b.clone().requires_grad_(True)
            y = batch_norm_act(xi, wi, bi, torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"),
                               relu=True, backend="hip", workspace=use_ws)
            y.backward(torch.ones_like(y) * (it + 1))
            outs.append((y.detach(), xi.grad, wi.grad, bi.grad))
        for p_, q_ in zip(*outs):
            torch.testing.assert_close(p_, q_, atol=0, rtol=0)
    # layout (csrc/bn_fin.h): [32][2C] fwd replicas | [32][2C] bwd | [5C] coefficients |
    # [32] folded-finalize descriptor | [64] tile counters -- accumulators and counters return to 0
    assert torch.count_nonzero(ws[: 32 * 4 * C]) == 0
    assert torch.count_nonzero(ws[-64:]) == 0


def test_resnet_hip_vs_torch_backend_step():
    """One ResNet-tiny training step: HIP BN path vs the eager composition."""
    from kubedl_amd.models.resnet import resnet_tiny
    res = []
    for backend in ("torch", "hip"):
        torch.manual_seed(0)
        m = resnet_tiny(10).cuda().to(memory_format=torch.channels_last)
        m.set_bn_backend(backend)
        x = torch.randn(8, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
        y = m(x)
        torch.nn.functional.cross_entropy(y, torch.arange(8, device="cuda") % 10).backward()
        res.append((y.detach(), m.conv1.weight.grad.clone(), m.layers[0].bn1.weight.grad.clone()))
    for a, b in zip(*res):
        torch.testing.assert_close(b, a, atol=2e-3, rtol=2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(4, 64, 112, 112), (2, 16, 9, 7), (3, 8, 2, 3)])
@pytest.mark.parametrize("training", [True, False])
def test_bn_relu_maxpool_matches_reference(shape, training):
    """Fused stem op vs fp32 torch: maxpool(relu(bn(x))) forward, and the
    gradients of x, gamma, beta (argmax routing computed on the bf16 ReLU
    output like torch's max-pool over a bf16 tensor)."""
    from kubedl_amd.ops.bn import batch_norm_relu_maxpool, workspace_for
    torch.manual_seed(0)
    dev = "cuda"
    C = shape[1]
    x = torch.randn(shape, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (1 + 0.1 * torch.randn(C, device=dev)).requires_grad_(True)
    b = (0.1 * torch.randn(C, device=dev)).requires_grad_(True)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    rm2, rv2 = rm.clone(), rv.clone()
    xh = x.clone().requires_grad_(True)
    y = batch_norm_relu_maxpool(xh, w, b, rm, rv, training=training, backend="hip",
                                workspace=workspace_for(C, dev))
    # reference: bn in fp32, relu, round to bf16 (what the unfused bf16 model pools over), pool
    xr = x.float().requires_grad_(True)
    wr, br = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    z = torch.nn.functional.batch_norm(xr, rm2, rv2, wr, br, training=training, momentum=0.1, eps=1e-5)
    zb = torch.relu(z)
    zq = zb + (zb.bfloat16().float() - zb).detach()  # straight-through bf16 rounding
    yr = torch.nn.functional.max_pool2d(zq, 3, 2, 1)
    # a 1-ulp bf16 rounding difference between the fused fp32 expression and
    # torch's can flip a near-tie argmax: allow a tiny fraction of mismatches
    def frac_off(a, b, tol):
        return (~torch.isclose(a, b, atol=tol, rtol=tol)).float().mean().item()
    assert frac_off(y.float(), yr, 2e-2) < 1e-3
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g.bfloat16().float())
    assert frac_off(xh.grad.float(), xr.grad, 5e-2) < 1e-3
    torch.testing.assert_close(w.grad, wr.grad, atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(b.grad, br.grad, atol=5e-2, rtol=2e-2)
    if training:
        torch.testing.assert_close(rm, rm2, atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(rv, rv2, atol=1e-4, rtol=1e-3)


@pytest.mark.gpu
def test_transpose_tiles_matches_torch():
    """Batched 64x64-tile transpose (csrc/multi_tensor.hip) incl. ragged edges."""
    from kubedl_amd.ops import _ext
    ext = _ext.load()
    shapes = [(256, 64), (64, 1024), (100, 72), (2048, 512)]
    srcs = [torch.randn(r, c, device="cuda").bfloat16() for r, c in shapes]
    dsts = [torch.empty(c, r, device="cuda", dtype=torch.bfloat16) for r, c in shapes]
    rows = []
    for s, d in zip(srcs, dsts):
        r, c = s.shape
        for r0 in range(0, r, 64):
            for c0 in range(0, c, 64):
                rows.append((s.data_ptr(), d.data_ptr(), r | (c << 32), r0 | (c0 << 32), c | (r << 32)))
    # 3x3 weight [Cout][3][3][Cin] -> per-tap transposed, taps reversed: [Cin][3][3][Cout]
    co, ci = 128, 64
    w = torch.randn(co, ci, 3, 3, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    wd = torch.empty(ci, co, 3, 3, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    esz = 2
    for tap in range(9):
        for r0 in range(0, co, 64):
            for c0 in range(0, ci, 64):
                rows.append((w.data_ptr() + tap * ci * esz, wd.data_ptr() + (8 - tap) * co * esz, co | (ci << 32),
                             r0 | (c0 << 32), (9 * ci) | ((9 * co) << 32)))
    ext.transpose_tiles(torch.tensor(rows, dtype=torch.int64).cuda())
    for s, d in zip(srcs, dsts):
        assert torch.equal(d, s.t().contiguous())
    assert torch.equal(wd, w.flip(2, 3).transpose(0, 1))
