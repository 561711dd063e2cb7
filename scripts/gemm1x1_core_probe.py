#!/usr/bin/env python3
"""Forward 1x1 conv GEMMs with the BN-statistics epilogue (the bottleneck's
conv3, C -> 4C) on the register-staged loop vs the LDS-DMA loop
(csrc/conv1x1.hip vs csrc/igemm.hip), alone on the GPU.

Rows: ``reg+pro`` = the engine's path today (register-staged, BN2 + ReLU
prologue on A); ``reg`` / ``dma`` = the same GEMM without the prologue on each
main loop (set_gemm_core 0 / 1).  If ``dma`` is far below ``reg``, a prologue
applied to the LDS-DMA tile in place is worth building.  One JSON line per row.
"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kubedl_amd.ops import _ext  # noqa: E402

SHAPES = [("stage1", 256 * 56 * 56, 64, 256), ("stage2", 256 * 28 * 28, 128, 512),
          ("stage3", 256 * 14 * 14, 256, 1024), ("stage4", 256 * 7 * 7, 512, 2048)]


def main() -> int:
    ext = _ext.load()
    torch.manual_seed(0)
    for name, M, K, N in SHAPES:
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        coef = torch.cat([torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.1])
        shift = torch.zeros(N, device="cuda")
        acc = torch.zeros(32 * 2 * N, device="cuda")
        flop = 2.0 * M * N * K
        for label, core, pro in (("reg+pro", -1, coef), ("reg", 0, None), ("dma", 1, None)):
            ext.set_gemm_core(core)
            args = (a, b, c, M, N, K, 0, 0, 0, 0, 1, pro, 1, shift, acc, None, None, None, None, 1, 0, 0,
                    None, None, None, None)
            for _ in range(3):
                ext.conv1x1_gemm(*args)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(30):
                ext.conv1x1_gemm(*args)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 30
            byts = (M * K + N * K + M * N) * 2
            print(json.dumps({"shape": name, "M": M, "K": K, "N": N, "path": label, "us": round(us, 1),
                              "tflops": round(flop / us / 1e6, 1), "tbps": round(byts / us / 1e6, 2)}), flush=True)
        ext.set_gemm_core(-1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
