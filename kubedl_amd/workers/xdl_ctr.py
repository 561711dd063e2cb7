"""XDLJob worker: sparse-embedding CTR training with PS / Worker / Scheduler roles.

Role mapping (env from the XDL controller: ``TASK_NAME``, ``TASK_INDEX``,
``ZK_ADDR`` + the runtime's ``KDL_RANK`` / ``KDL_WORLD_SIZE`` /
``KDL_NUM_PS`` / ``KDL_RDZV_ENDPOINT``):

* ``ps``        -- owns a row shard of every embedding table on its GPU and
                   serves pull/push rounds (``ShardedEmbedding.participate``);
* ``worker`` / ``extendrole`` -- generate a batch, pull embeddings, run the
                   MFMA dense tower, push de-duplicated sparse gradients, and
                   all-reduce dense gradients among workers (fused Adam);
* ``scheduler`` -- coordination only: signals Ready and idles until the job
                   completes (its pod is removed by cleanPodPolicy=Running).

Without PS replicas the workers own the shards themselves.  Synthetic data:
``--fields`` categorical fields with Zipf-distributed ids over
``--vocab`` rows each, ``--dense`` dense features, labels from a hidden
logistic model (so the loss visibly falls).  Prints one JSON line from the
first worker: samples/s, steps/s, loss.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import signal
import sys
import time

import torch
import torch.distributed as dist

from kubedl_amd.models.ctr import CTRModel, ShardedEmbedding
from kubedl_amd.ops.optim import FlatParamSpace, FusedAdam
from kubedl_amd.parallel import dist as kdist
from kubedl_amd.parallel.ddp import FlatDDP
from kubedl_amd.workers import common


def synth_batch(B, F, V, nd, gen, w_true):
    """One synthetic batch, generated where ``gen`` lives (the GPU in runs)."""
    dev = w_true.device
    # Zipf-like ids: heavy head, long tail (what makes de-duplication pay)
    u = torch.rand(B, F, generator=gen, device=dev)
    ids = (V * u.pow(3.0)).long().clamp_(max=V - 1)
    dense = torch.randn(B, nd, generator=gen, device=dev)
    logit = (w_true[ids % w_true.numel()].sum(1) * 0.5 + dense[:, 0]).clamp(-8, 8)
    y = (torch.rand(B, generator=gen, device=dev) < torch.sigmoid(logit)).float()
    return ids, dense, y


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=None, help="default 50 (GPU) / 6 (CPU)")
    ap.add_argument("--warmup", type=int, default=None, help="default 5 (GPU) / 1 (CPU)")
    ap.add_argument("--batch", type=int, default=None, help="default 4096 (GPU) / 256 (CPU)")
    ap.add_argument("--fields", type=int, default=26)
    ap.add_argument("--vocab", type=int, default=None, help="rows per field; default 100000 (GPU) / 2000 (CPU)")
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--dense", type=int, default=16)
    ap.add_argument("--hidden", default=None, help="default 1024,512,256 (GPU) / 256,128 (CPU)")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--emb-lr", type=float, default=0.05)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--exchange", choices=("auto", "fixed"), default="auto",
                    help="fixed: the PS + worker fixed-capacity exchange even at world 1 (one-GPU rehearsal: "
                         "RCCL all-to-alls on a 1-rank group, one owner)")
    args, _unknown = ap.parse_known_args(argv)
    # the BASELINE.json config on the GPU; a plumbing-sized job on CPU (the
    # reference's example specs carry no sizes, so they run with these)
    gpu_defaults = (not args.cpu) and torch.cuda.is_available()
    for name, g, c in (("steps", 50, 6), ("warmup", 5, 1), ("batch", 4096, 256), ("vocab", 100000, 2000),
                       ("hidden", "1024,512,256", "256,128")):
        if getattr(args, name) is None:
            setattr(args, name, g if gpu_defaults else c)

    task = os.environ.get("TASK_NAME", "worker").lower()
    if task == "scheduler":
        common.signal_ready({"task": task})
        stop = []
        signal.signal(signal.SIGTERM, lambda *_: stop.append(1))
        while not stop:
            time.sleep(0.2)
        return 0

    rank = int(os.environ.get("KDL_RANK", os.environ.get("RANK", "0")))
    world = int(os.environ.get("KDL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    n_ps = int(os.environ.get("KDL_NUM_PS", "0"))
    ep = os.environ.get("KDL_RDZV_ENDPOINT")
    if ep:
        host, port = ep.rsplit(":", 1)
        os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = host, port
    use_gpu = (not args.cpu) and torch.cuda.is_available()
    # LOCAL_RANK picks this rank's GPU out of the gang's visible set
    device = kdist.local_device(use_gpu)
    if use_gpu:
        torch.cuda.set_device(device)
        kdist.apply_hbm_limit(device)
    # KDL_DIST_BACKEND=gloo: rehearse a multi-rank job on fewer GPUs than ranks
    # (RCCL refuses two ranks on one device; parallel/dist.py init_from_env)
    backend = os.environ.get("KDL_DIST_BACKEND", "nccl") if use_gpu else "gloo"
    rehearse = args.exchange == "fixed" and world == 1
    if world > 1 or rehearse:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(common.free_port()) if rehearse else "29511")
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))
        if use_gpu and backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    common.signal_ready({"rank": rank, "task": task})
    owners = list(range(n_ps)) if n_ps > 0 else list(range(world))
    workers = [r for r in range(world) if r >= n_ps]
    wgroup = dist.new_group(workers) if world > 1 else None
    is_worker = rank in workers
    # every rank knows the per-pull id bound (batch x fields) from the job's
    # command line: the multi-rank exchange runs at that fixed capacity, with
    # equal all-to-all splits and no per-step size round trip to the host
    emb = ShardedEmbedding(args.fields * args.vocab, args.dim, owners, rank, world, device,
                           group=None, lr=args.emb_lr, max_ids=args.batch * args.fields,
                           force_fixed=args.exchange == "fixed", rows_bf16=True)
    total = args.warmup + args.steps
    if not is_worker:  # PS: serve pull/push rounds
        for _ in range(total):
            emb.participate(scale=1.0 / len(workers))  # the workers' push scale
        emb.finalize()
        dist.barrier()
        dist.destroy_process_group()
        return 0

    hidden = tuple(int(h) for h in args.hidden.split(","))
    torch.manual_seed(0)
    model = CTRModel(args.fields, args.vocab, args.dim, args.dense, hidden, emb, device)
    space = FlatParamSpace(model.tower, dtype=torch.bfloat16, device=device)
    ddp = FlatDDP(space, len(workers), process_group=wgroup, broadcast_from=workers[0])
    opt = FusedAdam(space, lr=args.lr)
    opt.grad_scale = ddp.grad_scale
    gen = torch.Generator(device=device).manual_seed(100 + rank)
    w_true = (torch.randn(4096, generator=torch.Generator().manual_seed(7)) * 0.5).to(device)
    # every step's synthetic batch is generated on the device before the timed
    # loop (distinct batches, no host work or H2D copy inside the timed steps)
    batches = [synth_batch(args.batch, args.fields, args.vocab, args.dense, gen, w_true) for _ in range(total)]
    losses = []
    t0 = None
    for it in range(total):
        if it == args.warmup:
            if use_gpu:
                torch.cuda.synchronize()
            if world > 1:
                dist.barrier(group=wgroup)
            t0 = time.perf_counter()
        ids, dense, y = batches[it % len(batches)]
        space.zero_grad()
        x, inv, U = model.build_input(ids, dense)
        if model.tower.fused_ok(x):  # explicit forward + backward (no autograd graph)
            loss, xgrad = model.tower.train_step(x, y, on_ready=ddp.ready if ddp.active else None)
        else:
            x.requires_grad_(True)
            loss, _logit = model.tower.loss(x, y)
            loss.backward()
            xgrad = x.grad
        model.push_grads(xgrad, inv, U, scale=1.0 / len(workers))
        ddp.finish()
        opt.step()
        losses.append(loss.detach())
        common.report_progress(it + 1, final=it + 1 == total)
    # host time to issue the timed steps (no sync inside the loop): ~dt when host-bound
    issue = time.perf_counter() - t0 if t0 is not None else 0.0
    if use_gpu:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0 if t0 is not None else 0.0
    xstats = emb.finalize()  # (after the timed region: reads the last exchanges' agreed fills)
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=wgroup)
        dt = float(t.item())
    first = float(torch.stack(losses[:5]).float().mean())
    last = float(torch.stack(losses[-5:]).float().mean())
    if rank == workers[0]:
        print(json.dumps({"rank": rank, "world_size": world, "ps": n_ps, "workers": len(workers),
                          "steps": args.steps, "batch_per_worker": args.batch, "seconds": dt,
                          "steps_per_sec": args.steps / dt if dt > 0 else 0.0,
                          "host_issue_ms_per_step": round(issue / max(args.steps, 1) * 1e3, 4),
                          "samples_per_sec": args.steps * args.batch * len(workers) / dt if dt > 0 else 0.0,
                          "loss_first": first, "loss_last": last, "device": str(device),
                          "hip_kernels": emb.use_hip, "exchange": "fixed" if emb._fixed() else "sync-free",
                          **xstats}), flush=True)
    if world > 1 or rehearse:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    from kubedl_amd.parallel.dist import run_rank
    sys.exit(run_rank(main))
