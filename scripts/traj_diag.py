"""Multi-step engine run reporting, per step, the parameters whose gradient or
master weight is non-finite / huge (first offenders by flat order).
usage: traj_diag.py [steps] [batch] [autograd_first]   (env: KDL_ENGINE=recomp=256,side=0 ...)
autograd_first = 1: run the autograd trainer for ``steps`` first in the same
process (as tests/test_trajectory_gpu.py's truth fixture does)"""
import json
import sys

import torch

from kubedl_amd.parallel.dist import DistInfo
from kubedl_amd.workers.resnet50 import ResNetTrainer


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    info = DistInfo(0, 1, 0, torch.device("cuda", 0), "nccl")
    if len(sys.argv) > 3 and sys.argv[3] == "1":
        ag = ResNetTrainer(info, batch=batch, image=224, engine="autograd", bn_backend="auto", seed=5)
        print(json.dumps({"autograd": [float(ag.step()) for _ in range(steps)]}), flush=True)
        del ag
    tr = ResNetTrainer(info, batch=batch, image=224, engine="fused", bn_backend="auto", seed=5)
    sp = tr.space
    for s in range(steps):
        loss = float(tr.step())
        torch.cuda.synchronize()
        bad = []
        for slot in sp.slots:
            g = sp.grad[slot.offset:slot.offset + slot.numel].float()
            w = sp.master[slot.offset:slot.offset + slot.numel]
            gm = g.abs().max().item() if torch.isfinite(g).all() else float("inf")
            wm = w.abs().max().item() if torch.isfinite(w).all() else float("inf")
            if gm > 1e4 or wm > 1e4:
                bad.append((slot.name, gm, wm))
        print(json.dumps({"step": s, "loss": loss, "bad": bad[:8], "nbad": len(bad)}), flush=True)


if __name__ == "__main__":
    main()
