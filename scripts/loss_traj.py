"""Loss trajectory of the ResNet-50 training step under one configuration
(env switches such as KDL_ENGINE=side=0,bn_bwd_fuse=0 / AMD_SERIALIZE_KERNEL
apply as usual): prints one JSON line with the per-step losses and a weight
checksum, so configurations that must compute the same thing can be compared.

Usage: python scripts/loss_traj.py [--steps 8] [--batch 256] [--pg] [--engine fused|autograd] [--sync]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kubedl_amd.parallel import dist as kdist  # noqa: E402
from kubedl_amd.workers.resnet50 import ResNetTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--pg", action="store_true", help="world-1 RCCL group, communicator built before the steps")
    ap.add_argument("--engine", default="fused")
    ap.add_argument("--sync", action="store_true", help="synchronise after every step")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    info = kdist.init_from_env(None, world1_group=a.pg)
    tr = ResNetTrainer(info, batch=a.batch, image=224, engine=a.engine, bn_backend="auto")
    if a.pg:
        kdist.first_collective(info, tr.stream)
    losses = []
    for _ in range(a.steps):
        losses.append(tr.step().detach().float().reshape(1))
        if a.sync:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    ls = [round(float(x), 4) for x in losses]
    m = tr.space.master
    print(json.dumps({"tag": a.tag, "losses": ls, "w_norm": round(float(m.double().norm()), 6),
                      "w_sum": round(float(m.double().sum()), 6)}), flush=True)
    kdist.shutdown(info)


if __name__ == "__main__":
    main()
