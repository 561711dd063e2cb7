"""One ResNet-50 engine forward+backward (batch 256, same weights and batch)
under several stream setups; prints, per setup, the parameters whose gradient
differs most from the two-stream reference run (relative L2), so a setup that
computes something different points at its layer.

Usage: python scripts/grad_diff.py [--batch 256]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kubedl_amd.parallel import dist as kdist  # noqa: E402
from kubedl_amd.workers.resnet50 import ResNetTrainer  # noqa: E402


def grads(tr):
    tr.space.zero_grad()
    with torch.cuda.stream(tr.stream):
        tr.engine.forward_backward(tr.x, tr.y)
    torch.cuda.synchronize()
    return {n: tr.space.grad_view(p).float().clone() for n, p in tr.model.named_parameters()}


def diff(ref, g, top=6):
    rows = []
    for n in ref:
        d = float((g[n] - ref[n]).norm() / (ref[n].norm() + 1e-30))
        rows.append((d, n))
    rows.sort(reverse=True)
    return [(n, round(d, 5)) for d, n in rows[:top]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    info = kdist.init_from_env(None)
    tr = ResNetTrainer(info, batch=a.batch, image=224, engine="fused")
    side = tr.engine.side
    ref = grads(tr)
    out = {"rerun": diff(ref, grads(tr))}
    tr.engine.side = None
    out["one_stream"] = diff(ref, grads(tr))
    torch.cuda.synchronize()
    tr.engine.side = side
    out["rerun2"] = diff(ref, grads(tr))
    for k, v in out.items():
        print(json.dumps({k: v}), flush=True)


if __name__ == "__main__":
    main()
