"""MASKX epilogue (ReLU mask recomputed from the BN input + BN backward sums)
on every LDS-DMA tile config at the ResNet-50 b256 shapes that run it: the
stride-1 3x3 data gradient (G_CONV3), the stride-2 one (G_DGRAD2) and the 1x1
data gradient (dense).  A zero A operand must give exact zeros; a random one
must match the 128x128 config (checked against fp32 PyTorch in the tests).

Usage: python scripts/maskx_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kubedl_amd.ops import _ext  # noqa: E402
from kubedl_amd.ops.conv import s2_dgrad_weights  # noqa: E402

ext = _ext.load()


def nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def run(kind, A, Bw, xbn, C, nb, H, cfg):
    ext.set_igemm_cfg(cfg)
    coef = torch.cat([torch.ones(C, device="cuda"), torch.full((C,), 0.1, device="cuda")]).float()
    mean = torch.zeros(C, device="cuda")
    acc = torch.zeros(32 * 2 * C, device="cuda")
    out = nhwc(torch.full(xbn.shape, float("nan"), device="cuda", dtype=torch.bfloat16))
    if kind == "s2":
        ext.conv3x3_s2_dgrad(A, Bw, out, nb, H // 2, H // 2, A.shape[1], C, 2, acc, xbn, mean, coef)
    elif kind == "conv3":
        ext.conv3x3_gemm(A, Bw, out, nb, H, H, A.shape[1], C, 1, None, 2, None, acc, xbn, mean, coef)
    else:
        M = nb * H * H
        ext.conv1x1_gemm(A, Bw, out, M, C, A.shape[1], 0, 0, 0, 0, 1, None, 2, None, acc, xbn, mean, coef, None, 1,
                         0, 0, None, None, None, None)
    torch.cuda.synchronize()
    ext.set_igemm_cfg(-1)
    return out.float(), acc.view(32, 2, C).sum(0)


def main():
    torch.manual_seed(0)
    nb = 256
    cases = [("s2", 256, 28, 256), ("conv3", 256, 14, 256), ("dense", 256, 14, 1024), ("s2", 128, 56, 128),
             ("conv3", 512, 7, 512), ("dense", 512, 7, 2048), ("dense", 128, 28, 512)]
    for kind, C, H, Ka in cases:
        xbn = nhwc(torch.randn(nb, C, H, H, device="cuda").bfloat16())
        if kind == "s2":
            A = nhwc(torch.randn(nb, Ka, H // 2, H // 2, device="cuda").bfloat16())
            Bw = s2_dgrad_weights(nhwc((torch.randn(Ka, C, 3, 3, device="cuda") / (3 * Ka ** 0.5)).bfloat16()))
        elif kind == "conv3":
            A = nhwc(torch.randn(nb, Ka, H, H, device="cuda").bfloat16())
            Bw = nhwc((torch.randn(C, Ka, 3, 3, device="cuda") / (3 * Ka ** 0.5)).bfloat16())
        else:
            A = nhwc(torch.randn(nb, Ka, H, H, device="cuda").bfloat16())
            Bw = (torch.randn(C, Ka, device="cuda") / Ka ** 0.5).bfloat16()
        ref, ref_acc = run(kind, A, Bw, xbn, C, nb, H, 2)
        for cfg in (-1, 0, 1, 2, 3):
            if cfg == 0 and C % 256:
                continue
            o0, _ = run(kind, torch.zeros_like(A), Bw, xbn, C, nb, H, cfg)
            o, a = run(kind, A, Bw, xbn, C, nb, H, cfg)
            print(json.dumps({"kind": kind, "C": C, "H": H, "K": Ka, "cfg": cfg,
                              "zero_max": float(o0.nan_to_num(1e30).abs().max()),
                              "nan": int((~torch.isfinite(o)).sum()),
                              "maxdiff_vs_cfg2": float((o.nan_to_num(1e30) - ref).abs().max()),
                              "acc_rel": float((a - ref_acc).norm() / (ref_acc.norm() + 1e-30))}), flush=True)


if __name__ == "__main__":
    main()
