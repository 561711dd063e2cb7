"""Diagnostic: per-tensor differences of the engine's gradients between
KDL_ENGINE=side=0 runs (baseline noise) and side=1 runs (side-stream wgrads)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from test_resnet_engine import _setup  # noqa: E402
from kubedl_amd.models.resnet_engine import ResNetEngine  # noqa: E402


def run(flag, steps=int(os.environ.get("DIAG_STEPS", "2"))):
    os.environ["KDL_ENGINE"] = f"side={flag}"
    model, _, x, y = _setup((2, 2, 2, 2), 64, "cuda", int(os.environ.get("DIAG_IMAGE", "96")), int(os.environ.get("DIAG_BATCH", "8")))
    eng = ResNetEngine(model, backend="hip")
    for _ in range(steps):
        for p in model.parameters():
            p.grad = None
        loss = eng.forward_backward(x, y)
    torch.cuda.synchronize()
    names = ["loss"] + [n for n, _ in model.named_parameters()] + [n for n, _ in model.named_buffers()]
    vals = [loss] + [p.grad.clone() for p in model.parameters()] + [b.clone() for b in model.buffers()]
    return names, vals


names, base = run("0")
for flag in sys.argv[1:] or ["0", "1", "1"]:
    _, v = run(flag)
    errs = []
    for n, a, b in zip(names, v, base):
        a, b = a.float(), b.float()
        errs.append(((a - b).abs().max().item() / (b.abs().max().item() + 1e-6), n))
    errs.sort(reverse=True)
    print(f"flag={flag} loss={v[0].item():.6f}/{base[0].item():.6f} worst:", [(f"{e:.3g}", n) for e, n in errs[:6]], flush=True)
