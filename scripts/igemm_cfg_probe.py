#!/usr/bin/env python3
"""Per-config timing of the 3x3 implicit GEMM (csrc/igemm.hip) on the ResNet-50
b256 stage 2-4 shapes: which tile / pipeline depth wins, alone on the GPU.

cfg: 0 = 256x256 (8 waves, 2 LDS stages), 1 = 256x128 (8 waves), 2 = 128x128
(4 waves, 2 blocks/CU), 3 = 256x64, 4 = 256x128 with three LDS stages (two
K-steps of DMA in flight: counted vmcnt + raw barrier), 5 = 256x256 (4 waves of
128x128, accumulators in AGPRs), 6 = 512x128 (4 waves of 128x128), 7 = 256x128
(4 waves of 128x64).  The last line per shape is hipBLASLt (torch.matmul) on the
dense GEMM of the same M x N x K: a yardstick only.  Prints one JSON line per
(shape, epilogue, cfg): mean us over 30 launches, TF/s.
"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kubedl_amd.ops import _ext  # noqa: E402

SHAPES = [  # (name, Nb, C, H)  stride-1 3x3, Cin = Cout = C
    ("stage2", 256, 128, 28),
    ("stage3", 256, 256, 14),
    ("stage4", 256, 512, 7),
]


def nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


CFGS = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1, 2, 3, 4, 5, 6, 7]


def main() -> int:
    ext = _ext.load()
    torch.manual_seed(0)
    for name, nb, c, h in SHAPES:
        x = nhwc(torch.randn(nb, c, h, h, device="cuda").bfloat16())
        w = nhwc((torch.randn(c, c, 3, 3, device="cuda") / (3 * c ** 0.5)).bfloat16())
        y = nhwc(torch.empty(nb, c, h, h, device="cuda", dtype=torch.bfloat16))
        shift = torch.zeros(c, device="cuda")
        acc = torch.zeros(32 * 2 * c, device="cuda")
        flop = 2.0 * nb * h * h * c * 9 * c
        for epi in (0, 1):
            for cfg in CFGS:
                if cfg in (0, 5) and c % 256:
                    continue
                ext.set_igemm_cfg(cfg)
                args = (x, w, y, nb, h, h, c, c, 1, None, epi, shift if epi else None, acc if epi else None,
                        None, None, None)
                for _ in range(3):
                    ext.conv3x3_gemm(*args)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(30):
                    ext.conv3x3_gemm(*args)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / 30
                print(json.dumps({"shape": name, "epi": epi, "cfg": cfg, "us": round(us, 1),
                                  "tflops": round(flop / us / 1e6, 1)}), flush=True)
        ext.set_igemm_cfg(-1)
        # yardstick only (never in the step): hipBLASLt on the dense GEMM of the same M x N x K
        m, k = nb * h * h, 9 * c
        a = torch.randn(m, k, device="cuda").bfloat16()
        b = torch.randn(k, c, device="cuda").bfloat16()
        for _ in range(3):
            torch.matmul(a, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            torch.matmul(a, b)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 30
        print(json.dumps({"shape": name, "hipblaslt_dense": True, "M": m, "N": c, "K": k, "us": round(us, 1),
                          "tflops": round(flop / us / 1e6, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
