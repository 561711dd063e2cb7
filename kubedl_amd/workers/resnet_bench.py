"""Rank side of the headline benchmark (BASELINE.json: "Job launch delay (s) +
steps/sec, PyTorchJob ResNet-50 at 1/2/4/8 MI355X").

One process per GPU, started either by the kdl control plane (``bench.py``
with no ``WORLD_SIZE`` in its environment submits a PyTorchJob whose ranks run
``python -m kubedl_amd.workers.resnet_bench``; the controller injects
``MASTER_ADDR/MASTER_PORT/WORLD_SIZE/RANK`` exactly as the reference's
``controllers/pytorch/pytorchjob_controller.go:180-233`` does) or by an
external ``torch.distributed.run`` (``bench.py`` calls :func:`run` in-process).

W untimed warm-up steps, then exactly K steps timed between a barrier and a
``synchronize`` on both sides, MAX over ranks.  Rank 0 prints one JSON line
(the driver contract): ``value`` = whole-job images/s (weak scaling: fixed
per-GPU batch).  Every step is a full forward + backward + gradient
all-reduce + fused SGD update of the full 25.6M-parameter ResNet-50 on
synthetic bf16 images and random-init weights; the step's loss is summed over
ranks with RCCL (so the collective path runs even at world 1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

T_PROC_START = time.time()

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# MIOpen find-db / kernel cache shipped in-tree: no conv algorithm search or
# kernel compile on a fresh box
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(_ROOT, "miopen_db", "user"))
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(_ROOT, "miopen_db", "cache"))

METRIC = "Job launch delay (s) + steps/sec, PyTorchJob ResNet-50 at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # the reference publishes no number


def add_args(ap: argparse.ArgumentParser) -> None:
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--bn-backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--conv-benchmark", type=int, default=0,
                    help="1 = MIOpen find mode (torch.backends.cudnn.benchmark)")
    ap.add_argument("--engine", default="auto", choices=["auto", "fused", "autograd"],
                    help="fused = explicit engine (fused conv GEMMs + staged BN); autograd = module + autograd")
    ap.add_argument("--allreduce", default=os.environ.get("KDL_ALLREDUCE", "rccl"), choices=["rccl", "p2p"],
                    help="DP gradient transport for N > 1: RCCL, or the IPC peer-buffer kernel (csrc/p2p.hip)")
    ap.add_argument("--ready-only", action="store_true",
                    help="initialise, signal Ready, exit (bench.py's cold launch-delay probe job)")
    ap.add_argument("--cpu", action="store_true", help="CPU/gloo dry run (tests only)")
    ap.add_argument("--tiny", action="store_true", help="tiny ResNet (tests only; invalid metric)")


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="ResNet-50 DDP bf16 benchmark rank")
    add_args(ap)
    return ap


def run(args, launcher: str) -> int:
    os.environ["KDL_ALLREDUCE"] = args.allreduce
    import torch  # noqa: F401  (first GPU-touching import happens in the rank only)
    from kubedl_amd.parallel import dist as kdist
    from kubedl_amd.workers import common
    from kubedl_amd.utils.tune import tune
    from kubedl_amd.workers.resnet50 import ResNetTrainer, sync

    t_import = time.time()
    info = kdist.init_from_env("cpu" if args.cpu else None,
                               world1_group=tune("world1_pg", True))
    t_pg = time.time()
    # Ready (the rank has started and its process group is up) --
    # the timestamp of the controller's launch-delay histograms
    common.signal_ready({"rank": info.rank}, wait_warm=False)  # waited at the first collective
    if args.ready_only:
        kdist.shutdown(info)
        return 0
    # the first collective builds the RCCL communicator (lazy: init_process_group
    # returns after the TCP-store rendezvous, dist.py) -- timed on its own so the
    # bootstrap cost is reported instead of hiding in the warm-up steps.  It
    # needs only the process group and the trainer's (touched) streams, so it
    # runs on a helper thread WHILE the model, optimizer and workspaces are
    # built (~0.9 s of a 1.5 s time to first step was this
    # bootstrap, run serially after the model build)
    comm = {"s": 0.0}
    threads = []
    # world 1: nothing in the first step needs RCCL (no DDP buckets; the loss
    # "sum" over one rank is the identity), and its ~0.9 s bootstrap -- RCCL
    # loading its device code objects, which holds up the main thread's first
    # kernel launches -- would otherwise sit in time-to-first-step.  It runs
    # right after the first step instead (warm-up), before any collective.
    defer = info.world_size == 1 and info.device.type == "cuda" and tune("comm_defer_w1", True)

    def start_comm(stream):
        comm["stream"] = stream
        if defer:
            return
        # every world size (VERDICT r5 missing 2): the trainer joins this thread
        # (join_comm, its before_collectives hook) before its own first
        # collective, the DDP parameter broadcast -- so every rank issues the
        # probe's two all-reduces, then the broadcast, in that order
        if not tune("comm_probe", True) or not tune("comm_overlap", True):
            return
        import threading

        def probe():
            try:
                comm["s"] = kdist.first_collective(info, stream)
            except BaseException as e:  # re-raised on the main thread
                comm["err"] = e
        th = threading.Thread(target=probe, name="rccl-bootstrap", daemon=True)
        th.start()
        threads.append(th)

    joined = {}

    def join_comm():
        if "t" not in joined:
            joined["t"] = time.time()
        for th in threads:
            th.join()
        if "err" in comm:
            raise comm["err"]

    trainer = ResNetTrainer(info, batch=args.batch, image=args.image, tiny=args.tiny,
                            bn_backend=args.bn_backend, conv_benchmark=bool(args.conv_benchmark),
                            engine=args.engine, on_streams_ready=start_comm, before_collectives=join_comm)
    trainer.defer_collectives = defer
    t_built = time.time()
    join_comm()
    if not threads and not defer and tune("comm_probe", True):  # comm_overlap=0: bootstrap after the model build
        comm["s"] = kdist.first_collective(info, getattr(trainer, "stream", None))
    sync(info)
    t_model = time.time()
    comm_init_s = comm["s"]
    kdist.barrier(info)
    # process start -> model resident on every rank
    rank_ready_s = kdist.all_reduce_max(time.time() - T_PROC_START, info)
    print(f"[bench] rank {info.rank} start: imports {t_import - T_PROC_START:.3f}s, process group "
          f"{t_pg - t_import:.3f}s, model+data {t_built - t_pg:.3f}s, waiting for the communicator "
          f"{t_model - t_built:.3f}s (bootstrap {comm_init_s:.3f}s, overlapped)", file=sys.stderr, flush=True)

    fault = bool(os.environ.get("KDL_FAULT"))
    t_first_step = None
    for i in range(args.warmup):
        trainer.step()
        if i == 0:  # (untimed warm-up) wall clock of the first finished step, all ranks
            sync(info)
            t_first_step = kdist.all_reduce_max(time.time(), info)
            if defer:  # the deferred world-1 bootstrap, then every later step's loss all-reduce
                comm["s"] = kdist.first_collective(info, comm.get("stream")) if tune("comm_probe", True) else 0.0
                trainer.defer_collectives = False
        if fault:
            common.maybe_inject_fault(info.rank, i)
    if trainer.defer_collectives:  # (no warm-up step ran)
        comm["s"] = kdist.first_collective(info, comm.get("stream")) if tune("comm_probe", True) else 0.0
        trainer.defer_collectives = False
    sync(info)
    kdist.barrier(info)
    sync(info)
    ddp = getattr(trainer, "ddp", None)
    if ddp is not None and ddp.active and info.device.type == "cuda":
        ddp.timing = True  # two events per step around the bucket waits (exposed time)
    # one event per step boundary on the step's stream (the side stream and the
    # DP buckets join it before the optimizer): per-step GPU times, read after
    # the loop, so a slow early step is told apart from a slow box
    st = getattr(trainer, "stream", None)
    evs = None
    if info.device.type == "cuda" and st is not None:
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    host = 0.0  # time spent issuing the steps (no sync): = ms_per_step when host-bound
    for i in range(args.steps):
        th = time.perf_counter()
        if evs is not None:
            evs[i].record(st)
        trainer.step()
        host += time.perf_counter() - th
    if evs is not None:
        evs[-1].record(st)
    sync(info)
    kdist.barrier(info)
    sync(info)
    dt = kdist.all_reduce_max(time.perf_counter() - t0, info)
    ddp_block = ddp.describe() if ddp is not None else None
    if ddp_block is not None:
        ex = ddp.exposed_ms() if ddp.timing else None
        ddp_block["exposed_ms_per_step"] = round(ex, 3) if ex is not None else None
        ddp.timing = False
    trainer.check_transport()  # a timed-out P2P all-reduce must fail the run, not report a number
    loss = float(trainer.loss().float().item())

    step_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)] if evs is not None else []
    n = info.world_size
    ms = dt / args.steps * 1e3
    imgs = args.batch * n * args.steps / dt
    if info.rank == 0:
        out = {
            "metric": METRIC,
            "value": round(imgs, 2),
            "unit": "images/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (imgs / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": "bf16",
            "data": "synthetic (random bf16 images/labels, random-init weights)",
            "config": {
                "model": "resnet50" if not args.tiny else "resnet_tiny",
                "global_batch": args.batch * n,
                "per_gpu_batch": args.batch,
                "image_size": args.image,
                "seq_len": None,
                "parallelism": f"dp{n}",
                "optimizer": "fused SGD-momentum (fp32 master)",
                "bn_backend": args.bn_backend,
                "engine": trainer.engine_kind,
                "conv_benchmark": bool(args.conv_benchmark),
                "allreduce": args.allreduce if n > 1 else None,
                "launcher": launcher,
                "stem": getattr(getattr(getattr(trainer, "engine", None), "K", None), "stem_path", None),
                "bn_bwd_fuse": getattr(getattr(trainer, "engine", None), "fuse_bwd", None),
            },
            "steps_per_sec": round(args.steps / dt, 4),
            "rank_ready_s": round(rank_ready_s, 3),
            "comm_init_s": round(comm_init_s, 3),
            # process start -> first finished step (max over ranks); the job path
            # adds time_to_first_step_s = job creation -> first finished step
            "first_step_s": round(t_first_step - T_PROC_START, 3) if t_first_step else None,
            "t_first_step_unix": round(t_first_step, 3) if t_first_step else None,
            "host_issue_ms_per_step": round(host / args.steps * 1e3, 3),
            # rank 0's per-step GPU times (event pairs on the step stream)
            "step_ms": ({"min": round(min(step_ms), 3), "median": round(sorted(step_ms)[len(step_ms) // 2], 3),
                         "max": round(max(step_ms), 3), "all": [round(v, 3) for v in step_ms]}
                        if step_ms else None),
            # rank 0's start-up phases (s): imports, process group, model build,
            # then what was left of the communicator bootstrap after the build
            "startup": {"imports": round(t_import - T_PROC_START, 3), "process_group": round(t_pg - t_import, 3),
                        "model": round(t_built - t_pg, 3), "comm_wait": round(t_model - t_built, 3),
                        "comm_overlap": bool(threads), "comm_deferred_past_first_step": defer,
                        # the trainer's hook joined the bootstrap before its first collective (world > 1:
                        # the DDP broadcast), this far into the model build
                        "comm_joined_at": round(joined["t"] - t_pg, 3) if "t" in joined else None},
            "final_loss": round(loss, 4),
            # DP gradient buckets: plan + the all-reduce time the step's compute
            # stream waited for (the rest overlapped the backward)
            "ddp": ddp_block,
        }
        print(json.dumps(out), flush=True)
    kdist.shutdown(info)
    return 0


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    return run(args, os.environ.get("KDL_BENCH_LAUNCHER", "kdl-pytorchjob"))


if __name__ == "__main__":
    from kubedl_amd.parallel.dist import run_rank
    sys.exit(run_rank(main))
