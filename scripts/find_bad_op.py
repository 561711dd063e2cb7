"""Find the first engine op whose output goes non-finite or explodes: every
HipKernels call is wrapped to record the fp32 norm of what it produced (its
return value, or the weight gradient it wrote), as a device tensor on the
stream that ran it (no host syncs, so the stream timing stays close to the
real step).  After the steps, prints the first bad record with the ones
before it, and the per-step losses.

Usage: python scripts/find_bad_op.py [--steps 10] [--batch 256]
"""
import argparse
import functools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kubedl_amd.models import resnet_engine as re_  # noqa: E402
from kubedl_amd.parallel import dist as kdist  # noqa: E402
from kubedl_amd.workers.resnet50 import ResNetTrainer  # noqa: E402

REC = []
STEP = [0]


def _norm(x):
    if isinstance(x, torch.Tensor) and x.is_floating_point():
        return torch.linalg.vector_norm(x.float()).reshape(1)
    return None


def wrap(name, fn, out_arg=None, args=False):
    @functools.wraps(fn)
    def w(*a, **k):
        if args:  # the inputs as the kernel sees them
            for i, x in enumerate(a[1:]):
                n = _norm(x)
                if n is not None:
                    REC.append((STEP[0], len(REC), f"{name}.in{i}", tuple(x.shape), n))
        r = fn(*a, **k)
        outs = r if isinstance(r, tuple) else (r,)
        if out_arg is not None and len(a) > out_arg:
            outs = outs + (a[out_arg],)
        for i, o in enumerate(outs):
            n = _norm(o)
            if n is not None:
                REC.append((STEP[0], len(REC), f"{name}[{i}]", tuple(o.shape), n))
        return r
    return w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    H = re_.HipKernels
    # ops returning tensors; (name, index of an in-place output argument)
    for name, oa in [("conv1x1_fwd", None), ("conv3x3_fwd", None), ("bn_apply", None), ("stem_fwd", None),
                     ("head_mask_reduce", None), ("bn_bwd_apply", None), ("bn_bwd_full", None),
                     ("dgrad_maskx", None), ("dgrad3x3_maskx", None), ("dgrad3x3s2_maskx", None),
                     ("dgrad_plain", None), ("dgrad_res", None), ("wgrad", 4), ("wgrad3x3", 4)]:
        setattr(H, name, wrap(name, getattr(H, name), oa, args=name == "dgrad3x3s2_maskx"))
    info = kdist.init_from_env(None)
    tr = ResNetTrainer(info, batch=a.batch, image=224, engine="fused")
    losses = []
    for s in range(a.steps):
        STEP[0] = s
        losses.append(tr.step().detach().float().reshape(1))
    torch.cuda.synchronize()
    ls = [round(float(x), 4) for x in losses]
    norms = torch.cat([r[4] for r in REC]).cpu().tolist()
    bad = None
    for i, v in enumerate(norms):
        if not (v == v) or v > 1e8:
            bad = i
            break
    print(json.dumps({"losses": ls, "records": len(REC), "first_bad": bad}), flush=True)
    if bad is not None:
        for j in range(max(0, bad - 12), min(len(REC), bad + 4)):
            s, idx, name, shape, _ = REC[j]
            print(json.dumps({"step": s, "i": idx, "op": name, "shape": shape, "norm": norms[j]}), flush=True)
    # every stride-2 data gradient of step 0 (inputs and output)
    for j, r in enumerate(REC):
        if r[0] == 0 and r[2].startswith("dgrad3x3s2"):
            print(json.dumps({"s0": r[2], "shape": r[3], "norm": norms[j]}), flush=True)
    from kubedl_amd.ops.conv import s2_dgrad_weights
    eng = tr.engine
    for blk in eng.blocks:
        if blk.conv2.stride[0] == 2:
            b = eng._ball(blk.conv2).float()
            ref = s2_dgrad_weights(blk.conv2.weight).float()
            print(json.dumps({"ball_vs_weights": float((b - ref).abs().max()), "ball_norm": float(b.norm())}),
                  flush=True)
    # the same op in a clean step, for scale
    if bad is not None and REC[bad][0] > 0:
        per = len(REC) // a.steps
        j = bad - per
        print(json.dumps({"prev_step_same_op": REC[j][2], "norm": norms[j]}), flush=True)


if __name__ == "__main__":
    main()
