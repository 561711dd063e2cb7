#!/usr/bin/env python3
"""gemm_bias_act (csrc/ctr.hip) at each tile shape on the CTR tower's GEMMs
(batch 4096, tower 1728 -> 1024 -> 512 -> 256: forward C = X W^T and data
gradient dX = dZ W), alone on the GPU.  One JSON line per (shape, tile);
the ``auto`` row is the tile ctr_tile_for picks.  Then the tower's weight
gradients (conv1x1_wgrad: split-batch fp32 slabs + fixed-order reduce) at
several KDL_TUNE wgrad_blocks targets (read per call)."""
import json
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kubedl_amd.ops import _ext  # noqa: E402

B = 4096
SHAPES = [("fwd1", B, 1024, 1728), ("fwd2", B, 512, 1024), ("fwd3", B, 256, 512),
          ("dx1", B, 1728, 1024), ("dx2", B, 1024, 512), ("dx3", B, 512, 256)]


def main() -> int:
    ext = _ext.load()
    torch.manual_seed(0)
    for name, M, N, K in SHAPES:
        a = torch.randn(M, K, device="cuda").bfloat16()
        # the data gradients read the nn.Linear weight [K, N] as stored (trans_w)
        tw = name.startswith("dx")
        w = (torch.randn(K, N, device="cuda") if tw else torch.randn(N, K, device="cuda")).div(K ** 0.5).bfloat16()
        b = None if tw else torch.randn(N, device="cuda").bfloat16()
        for tile in (0, 1, 2, -1):
            ext.set_ctr_tile(tile)
            for _ in range(5):
                ext.gemm_bias_act(a, w, b, not tw, tw)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                ext.gemm_bias_act(a, w, b, not tw, tw)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 50
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "trans_w": tw,
                              "tile": ["128x128", "128x64", "64x64"][ext.ctr_tile_for(M, N)] if tile < 0 else
                              ["128x128", "128x64", "64x64"][tile], "auto": tile < 0, "us": round(us, 2),
                              "tflops": round(2.0 * M * N * K / us / 1e6, 1)}), flush=True)
        ext.set_ctr_tile(-1)
    for name, N, K in (("dw1", 1024, 1728), ("dw2", 512, 1024), ("dw3", 256, 512)):
        dz = torch.randn(B, N, device="cuda").bfloat16()
        x = torch.randn(B, K, device="cuda").bfloat16()
        dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        # "solo" = the CTR model's policy (conv1x1_wgrad(..., solo=True))
        for blocks in (160, 320, 512, 768, 1024, 2048, "solo"):
            solo = blocks == "solo"
            if not solo:
                os.environ["KDL_TUNE"] = f"wgrad_blocks={blocks}"
            else:
                os.environ.pop("KDL_TUNE", None)
            ws = torch.empty(ext.conv1x1_wgrad_splits(B, N, K, solo) * N * K, device="cuda")
            for _ in range(5):
                ext.conv1x1_wgrad(dz, x, None, ws, dw, 1.0, B, N, K, 0, 0, 0, 0, 1, solo)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                ext.conv1x1_wgrad(dz, x, None, ws, dw, 1.0, B, N, K, 0, 0, 0, 0, 1, solo)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 50
            print(json.dumps({"shape": name, "M": B, "N": N, "K": K, "wgrad_blocks": blocks,
                              "splits": ext.conv1x1_wgrad_splits(B, N, K, solo), "us": round(us, 2),
                              "tflops": round(2.0 * B * N * K / us / 1e6, 1)}), flush=True)
        os.environ.pop("KDL_TUNE", None)
    return 0


if __name__ == "__main__":
    sys.exit(main())
