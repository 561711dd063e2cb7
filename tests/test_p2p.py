"""P2P all-reduce over IPC-mapped peer buffers (csrc/p2p.hip, kubedl_amd/parallel/p2p.py).

On the one-GPU box two rank processes share the card: the IPC mapping, the
cross-process signal protocol and the in-place two-phase reduction are the
same code paths as on an 8-GPU node (where the peers sit behind xGMI links);
the handle exchange runs over gloo.  The numerics reference is a plain fp32
sum of the ranks' inputs.
"""
import os
import socket

import pytest
import torch


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(target, world, *args, timeout=240):
    import torch.multiprocessing as mp
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=timeout) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


def test_transport_selection_cpu(monkeypatch):
    from kubedl_amd.parallel import p2p
    monkeypatch.delenv("KDL_ALLREDUCE", raising=False)
    assert not p2p.wanted()
    monkeypatch.setenv("KDL_ALLREDUCE", "P2P")
    assert p2p.wanted()
    monkeypatch.setenv("KDL_ALLREDUCE", "rccl")
    assert not p2p.wanted()
    with pytest.raises(ValueError):
        p2p.P2PAllReduce(torch.zeros(64))


def _ddp_cpu_worker(rank, world, port, q):
    import torch.distributed as dist
    from kubedl_amd.ops.optim import FlatParamSpace
    from kubedl_amd.parallel.ddp import FlatDDP
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KDL_ALLREDUCE="p2p")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = torch.nn.Linear(8, 4)
    sp = FlatParamSpace(m, dtype=torch.float32, device=torch.device("cpu"))
    ddp = FlatDDP(sp, world)
    q.put((rank, ddp.transport is None))
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_keeps_collectives_for_cpu_buffers():
    """KDL_ALLREDUCE=p2p only applies to GPU buffers: CPU ranks keep the process group."""
    res = _spawn(_ddp_cpu_worker, 2, timeout=120)
    assert all(r[1] for r in res)


def _p2p_worker(rank, world, port, q, dtype_name, n, bounds, reps, oneshot=None):
    import torch.distributed as dist
    from kubedl_amd.parallel.p2p import P2PAllReduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dtype = getattr(torch, dtype_name)
    dev = torch.device("cuda", 0)
    buf = torch.empty(n, dtype=dtype, device=dev)
    ar = P2PAllReduce(buf, timeout_s=20.0)
    outs = []
    for it in range(reps):
        g = torch.Generator().manual_seed(1000 * it + rank)
        src = torch.randn(n, generator=g).to(dtype)
        buf.copy_(src.to(dev))
        for lo, hi in bounds:
            ar.all_reduce_(lo, hi, oneshot=oneshot)
        torch.cuda.synchronize()
        outs.append((src.float().numpy(), buf.float().cpu().numpy()))
    err = ar.errors()
    ar.close()
    q.put((rank, outs, err))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype_name,oneshot", [("bfloat16", None), ("float32", None), ("bfloat16", True),
                                                ("float32", False)])
def test_p2p_allreduce_two_ranks_gpu(dtype_name, oneshot):
    """Buckets of several sizes (one unit per rank up to many blocks), reused over
    repeated calls (epochs), against an fp32 sum of the ranks' inputs; size-picked
    (one-shot below 256 KiB, two-shot above), forced one-shot, forced two-shot."""
    n = 1 << 20
    bounds = [(0, 64), (64, 4160), (4160, 100000), (100000, 300000), (300000, n)]
    if oneshot:  # one-shot holds at most 128 blocks x 256 threads x 4 units
        n = 1 << 19
        bounds = [(0, 64), (64, 4160), (4160, 100000), (100000, n)]
    world = 2
    res = _spawn(_p2p_worker, world, dtype_name, n, bounds, 3, oneshot)
    assert all(r[2] == 0 for r in res), "a p2p wait timed out"
    for it in range(3):
        ref = sum(torch.from_numpy(r[1][it][0]) for r in res)
        if dtype_name == "bfloat16":
            ref = ref.to(torch.bfloat16).float()
        for r in res:
            got = torch.from_numpy(r[1][it][1])
            torch.testing.assert_close(got, ref, atol=0, rtol=0)


def _timeout_worker(rank, world, port, q):
    import time
    import torch.distributed as dist
    from kubedl_amd.parallel.p2p import P2PAllReduce, P2PError
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf = torch.ones(4096, dtype=torch.float32, device=torch.device("cuda", 0))
    ar = P2PAllReduce(buf, timeout_s=0.5)
    raised = False
    t = 0.0
    if rank == 0:  # rank 1 never joins: every wait of rank 0 must give up
        t0 = time.time()
        ar.all_reduce_()
        torch.cuda.synchronize()
        t = time.time() - t0
        try:
            ar.check()
        except P2PError:
            raised = True
    dist.barrier()
    err = ar.errors()
    ar.close()
    q.put((rank, err, raised, t))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_p2p_missing_peer_times_out_gpu():
    """A rank whose peer never arrives drains in bounded time and reports it."""
    (r0, e0, raised0, t0), (r1, e1, raised1, _) = _spawn(_timeout_worker, 2, timeout=120)
    assert e0 != 0 and raised0
    assert t0 < 10.0
    assert e1 == 0 and not raised1


def _engine_worker(rank, world, port, q, transport):
    import torch.distributed as dist
    from kubedl_amd.parallel.dist import DistInfo
    from kubedl_amd.workers.resnet50 import ResNetTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KDL_ALLREDUCE=transport)
    # the two transports' runs are compared with each other: MIOpen must pick the
    # same solvers in both (find mode times candidates, and a different split-K
    # wgrad solver for the stem moves its bf16 gradient by several ulps)
    torch.backends.miopen.immediate = True
    torch.backends.cudnn.deterministic = True
    dist.init_process_group("gloo", rank=rank, world_size=world)
    info = DistInfo(rank, world, 0, torch.device("cuda", 0), "gloo")
    tr = ResNetTrainer(info, batch=4, image=64, num_classes=10, bn_backend="hip", engine="fused",
                       bucket_cap_mb=4.0, seed=0)
    assert (tr.ddp.transport is not None) == (transport == "p2p")
    losses = [float(tr.step()) for _ in range(2)]
    torch.cuda.synchronize()
    q.put((rank, losses, tr.space.master.cpu().numpy(), tr.space.grad.float().cpu().numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_engine_ddp_p2p_transport_gpu():
    """The engine's bucketed DDP over the P2P transport: identical weights on both
    ranks and the same gradients as the process-group transport."""
    p = _spawn(_engine_worker, 2, "p2p")
    g = _spawn(_engine_worker, 2, "rccl")
    (_, lp0, mp0, gp0), (_, lp1, mp1, gp1) = p
    (_, lg0, mg0, gg0), _ = g
    mp0, mp1, gp0, gp1, mg0, gg0 = (torch.from_numpy(a) for a in (mp0, mp1, gp0, gp1, mg0, gg0))
    torch.testing.assert_close(mp0, mp1, atol=0, rtol=0)
    torch.testing.assert_close(gp0, gp1, atol=0, rtol=0)
    assert lp0 == pytest.approx(lg0, rel=1e-2)
    # bf16 gradient sums: the p2p kernel rounds once from fp32, gloo per hop
    torch.testing.assert_close(gp0, gg0, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(mp0, mg0, atol=2e-3, rtol=2e-3)


def _selfcheck_worker(rank, world, port, q, corrupt):
    import torch.distributed as dist
    from kubedl_amd.parallel.p2p import P2PError, P2PTransport
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1 << 16
    g = torch.Generator().manual_seed(rank)
    buf = (torch.randn(n, generator=g) * 1e-2).to(torch.bfloat16).to("cuda:0")
    P2PTransport.inject_corrupt_rank = 1 if corrupt else None
    tr = P2PTransport(buf)
    raised, msg = False, ""
    try:
        tr.launch(0, n).wait()
        torch.cuda.synchronize()
        tr.launch(0, 4096).wait()  # verified: the plain path
        torch.cuda.synchronize()
    except P2PError as e:
        raised, msg = True, str(e)
    q.put((rank, raised, tr.verified, tr.self_check_max_err, msg))
    tr.ar.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("corrupt", [False, True])
def test_p2p_transport_self_check_gpu(corrupt):
    """the transport's first bucket goes through both the
    process group and the P2P kernel and is compared.  A clean pair passes
    (one-ulp bf16 agreement) and the transport switches to the plain path; a
    peer buffer corrupted between the two (rank 1 perturbs its bucket after the
    reference copy) makes EVERY rank raise P2PError instead of training on it."""
    res = _spawn(_selfcheck_worker, 2, corrupt, timeout=120)
    for rank, raised, verified, err, msg in res:
        if corrupt:
            assert raised and not verified and "self-check" in msg, (rank, msg)
        else:
            assert not raised and verified, (rank, msg)
            assert err is not None and err <= 2 ** -7 * 0.1, err
