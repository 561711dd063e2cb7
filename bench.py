#!/usr/bin/env python3
"""Headline benchmark: PyTorchJob ResNet-50 DDP bf16 training throughput on MI355X.

Metric/config from BASELINE.json ("Job launch delay (s) + steps/sec, PyTorchJob
ResNet-50 at 1/2/4/8 MI355X"; config "PyTorchJob ResNet-50 DDP bf16, 8 workers").
The reference publishes no number, so ``vs_baseline`` is null.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
it is started by ``torch.distributed.run`` with one rank per GPU.  W untimed
warmup steps, then exactly K steps timed between barrier+synchronize on both
sides, MAX over ranks; rank 0 prints one JSON line.  ``value`` is whole-job
images/s (weak scaling: fixed per-GPU batch), ``steps_per_sec`` is reported
alongside.  Data is synthetic (random bf16 images / labels, fixed per rank),
weights random-init; every step is a full forward + backward + all-reduce +
fused SGD update of the full 25.6M-parameter ResNet-50.

``launch_delay_s`` (process start -> rank ready, i.e. process group up and
model resident) is the rank-side half of the reference's
first/all-pods-launch-delay metric; ``python -m kubedl_amd.cli bench-launch``
measures the full controller path (job submitted -> all ranks Ready).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

T_PROC_START = time.time()

# MIOpen find-db / kernel cache shipped in-tree (populated on an MI355X by
# scripts/gpu_check.sh): conv algorithm search and kernel compiles are not
# repeated on every fresh box.
_ROOT = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(_ROOT, "miopen_db", "user"))
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(_ROOT, "miopen_db", "cache"))

import torch  # noqa: E402

from kubedl_amd.parallel import dist as kdist  # noqa: E402
from kubedl_amd.workers.resnet50 import ResNetTrainer, sync  # noqa: E402
from kubedl_amd.workers import common  # noqa: E402

METRIC = "Job launch delay (s) + steps/sec, PyTorchJob ResNet-50 at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # reference publishes no number


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--bn-backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--conv-benchmark", type=int, default=0,
                    help="1 = MIOpen find mode (torch.backends.cudnn.benchmark)")
    ap.add_argument("--engine", default="auto", choices=["auto", "fused", "autograd"],
                    help="fused = explicit engine (fused 1x1-conv GEMMs + staged BN); autograd = module + autograd")
    ap.add_argument("--allreduce", default=os.environ.get("KDL_ALLREDUCE", "rccl"), choices=["rccl", "p2p"],
                    help="DP gradient transport for N > 1: RCCL, or the IPC peer-buffer kernel (csrc/p2p.hip)")
    ap.add_argument("--cpu", action="store_true", help="CPU/gloo dry run (tests only)")
    ap.add_argument("--tiny", action="store_true", help="tiny ResNet (tests only; invalid metric)")
    args = ap.parse_args(argv)
    os.environ["KDL_ALLREDUCE"] = args.allreduce

    if "WORLD_SIZE" not in os.environ:
        os.environ["WORLD_SIZE"] = "1"
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("LOCAL_RANK", "0")
    info = kdist.init_from_env("cpu" if args.cpu else None)
    if info.world_size != args.gpus and info.rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={info.world_size}",
              file=sys.stderr)

    trainer = ResNetTrainer(info, batch=args.batch, image=args.image, tiny=args.tiny,
                            bn_backend=args.bn_backend, conv_benchmark=bool(args.conv_benchmark),
                            engine=args.engine)
    sync(info)
    kdist.barrier(info)
    launch_delay = kdist.all_reduce_max(time.time() - T_PROC_START, info)
    common.signal_ready({"rank": info.rank})

    for _ in range(args.warmup):
        trainer.step()
    sync(info)
    kdist.barrier(info)
    sync(info)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.step()
    sync(info)
    kdist.barrier(info)
    sync(info)
    dt = kdist.all_reduce_max(time.perf_counter() - t0, info)
    loss = float(trainer.last_loss.float().item())

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
            },
            "steps_per_sec": round(args.steps / dt, 4),
            "launch_delay_s": round(launch_delay, 3),
            "final_loss": round(loss, 4),
        }
        print(json.dumps(out), flush=True)
    kdist.shutdown(info)
    return 0


if __name__ == "__main__":
    sys.exit(main())
