#!/usr/bin/env python3
"""Weight-gradient kernels (csrc/wgrad_dma.hip through conv3x3_wgrad / conv1x1_wgrad) on
ResNet-50 b256 shapes, alone on the GPU: mean us over 20 launches (slab reduce included),
TF/s, and the max |error| against an fp32 torch reference on an 8-image slice.

usage: wgrad_probe.py   (KDL_C_PATH selects an A/B build of the extension)
"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kubedl_amd.ops import _ext  # noqa: E402


def nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main() -> int:
    ext = _ext.load()
    torch.manual_seed(0)
    ext.set_wgrad_big(2)  # the ResNet engine's setting with its weight-gradient stream on
    for name, nb, c, h, s in [("3x3_s2_28", 256, 128, 28, 1), ("3x3_s3_14", 256, 256, 14, 1),
                              ("3x3_s4_7", 256, 512, 7, 1), ("3x3_s1_56", 256, 64, 56, 1)]:
        x = nhwc(torch.randn(nb, c, h, h, device="cuda").bfloat16())
        dy = nhwc(torch.randn(nb, c, h, h, device="cuda").bfloat16())
        dW = nhwc(torch.empty(c, c, 3, 3, device="cuda", dtype=torch.bfloat16))
        ws = torch.empty(ext.conv3x3_wgrad_slabs(nb, h, h, c, c, 1) * c * 9 * c, device="cuda")
        us = timed(lambda: ext.conv3x3_wgrad(dy, x, None, ws, dW, 1.0, nb, h, h, c, c, 1))
        ref = torch.nn.grad.conv2d_weight(x[:8].float(), (c, c, 3, 3), dy[:8].float(), stride=1, padding=1)
        ext.conv3x3_wgrad(dy[:8], x[:8], None, ws, dW, 1.0, 8, h, h, c, c, 1)
        torch.cuda.synchronize()
        err = float((dW.float() - ref).abs().max() / ref.abs().max())
        flop = 2.0 * nb * h * h * c * 9 * c
        print(json.dumps({"op": name, "us": round(us, 1), "tflops": round(flop / us / 1e6, 1), "rel_err": err}),
              flush=True)
    for name, M, N, K in [("1x1_s1_256x64", 256 * 56 * 56, 256, 64), ("1x1_s1_64x256", 256 * 56 * 56, 64, 256),
                          ("1x1_s3_1024x256", 256 * 14 * 14, 1024, 256), ("1x1_s4_2048x512", 256 * 7 * 7, 2048, 512)]:
        G = torch.randn(M, N, device="cuda").bfloat16()
        A = torch.randn(M, K, device="cuda").bfloat16()
        dW = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        ws = torch.empty(ext.conv1x1_wgrad_splits(M, N, K) * N * K, device="cuda")
        us = timed(lambda: ext.conv1x1_wgrad(G, A, None, ws, dW, 1.0, M, N, K, 0, 0, 0, 0, 1))
        ref = G[:4096].float().t() @ A[:4096].float()
        ext.conv1x1_wgrad(G[:4096], A[:4096], None, ws, dW, 1.0, 4096, N, K, 0, 0, 0, 0, 1)
        torch.cuda.synchronize()
        err = float((dW.float() - ref).abs().max() / ref.abs().max())
        print(json.dumps({"op": name, "us": round(us, 1), "tflops": round(2.0 * M * N * K / us / 1e6, 1),
                          "rel_err": err}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
