"""Stride-2 3x3 data gradient (csrc/igemm.hip G_DGRAD2) at a ResNet-50 b256
shape, every tile config and both epilogues: max |dx| for a zero dy (must be
exactly 0) and the max error vs fp32 PyTorch for a random dy.

Usage: python scripts/s2_probe.py [--C 256] [--Hd 14] [--nb 256]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kubedl_amd.ops import _ext  # noqa: E402
from kubedl_amd.ops.conv import s2_dgrad_weights  # noqa: E402


def nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--C", type=int, default=256)
    ap.add_argument("--Hd", type=int, default=14)
    ap.add_argument("--nb", type=int, default=256)
    a = ap.parse_args()
    ext = _ext.load()
    C, Hd, nb = a.C, a.Hd, a.nb
    torch.manual_seed(0)
    w = nhwc((torch.randn(C, C, 3, 3, device="cuda") / (3 * C ** 0.5)).bfloat16())
    ball = s2_dgrad_weights(w)
    xbn = nhwc(torch.randn(nb, C, 2 * Hd, 2 * Hd, device="cuda").bfloat16())
    coef = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.5]).float()
    mean = torch.randn(C, device="cuda") * 0.1
    dyr = nhwc(torch.randn(nb, C, Hd, Hd, device="cuda").bfloat16())
    ref = torch.nn.grad.conv2d_input(xbn.shape, w.float(), dyr.float(), stride=2, padding=1)
    for cfg in (-1, 0, 1, 2, 3):
        if cfg == 0 and C % 256:
            continue
        ext.set_igemm_cfg(cfg)
        for epi in (0, 2):
            row = {"cfg": cfg, "epi": epi}
            for name, dy in (("zero", torch.zeros_like(dyr)), ("rand", dyr)):
                acc = torch.zeros(32 * 2 * C, device="cuda")
                out = nhwc(torch.full((nb, C, 2 * Hd, 2 * Hd), float("nan"), device="cuda", dtype=torch.bfloat16))
                if epi == 0:
                    ext.conv3x3_s2_dgrad(dy, ball, out, nb, Hd, Hd, C, C, 0, None, None, None, None)
                else:
                    ext.conv3x3_s2_dgrad(dy, ball, out, nb, Hd, Hd, C, C, 2, acc, xbn, mean, coef)
                torch.cuda.synchronize()
                o = out.float()
                row[name + "_nan"] = int((~torch.isfinite(o)).sum())
                if name == "zero":
                    row["zero_max"] = float(o.nan_to_num(0).abs().max())
                    bad = (o.nan_to_num(1) != 0)
                    if bad.any():
                        idx = bad.nonzero()
                        row["zero_bad_count"] = int(idx.shape[0])
                        # which images / sub-pixel classes / channels
                        row["bad_imgs"] = sorted(set(idx[:, 0].tolist()))[:8]
                        row["bad_cls"] = sorted(set(((idx[:, 2] % 2) * 2 + idx[:, 3] % 2).tolist()))
                        row["bad_ch"] = [int(idx[:, 1].min()), int(idx[:, 1].max())]
                else:
                    r = ref
                    if epi == 2:
                        mask = (xbn.float() * coef[:C].view(1, C, 1, 1) + coef[C:].view(1, C, 1, 1)) > 0
                        r = torch.where(mask, ref.bfloat16().float(), torch.zeros_like(ref))
                    row["rand_maxerr"] = float((o.nan_to_num(1e9) - r).abs().max())
            print(json.dumps(row), flush=True)
    ext.set_igemm_cfg(-1)


if __name__ == "__main__":
    main()
