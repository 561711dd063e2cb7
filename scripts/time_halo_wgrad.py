"""Stage-1 3x3 weight gradient (nb 256, 56x56, 64 -> 64): input-halo kernel vs the
LDS-DMA implicit GEMM (a conv1x1_wgrad_splits-sized workspace forces the latter),
same process, events around 20 launches each (slab reduce included)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from kubedl_amd.ops import _ext  # noqa: E402

ext = _ext.load()
nb, H, W, C = 256, 56, 56, 64
x = torch.randn(nb, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
dy = torch.randn(nb, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
dW = torch.empty(C, C, 3, 3, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
flop = 2.0 * nb * H * W * C * 9 * C
arms = {"halo": ext.conv3x3_wgrad_slabs(nb, H, W, C, C, 1), "igemm": ext.conv1x1_wgrad_splits(nb * H * W, C, 9 * C)}
ref = torch.nn.grad.conv2d_weight(x[:8].float(), (C, C, 3, 3), dy[:8].float(), stride=1, padding=1)
for rep in range(2):
    for name, slabs in arms.items():
        ws = torch.empty(slabs * C * 9 * C, device="cuda")
        for _ in range(3):
            ext.conv3x3_wgrad(dy, x, None, ws, dW, 1.0, nb, H, W, C, C, 1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ext.conv3x3_wgrad(dy, x, None, ws, dW, 1.0, nb, H, W, C, C, 1)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 20
        print(json.dumps({"op": "wgrad3x3_s1_56", "variant": name, "slabs": slabs, "rep": rep, "us": round(us, 1),
                          "tflops": round(flop / us / 1e6, 1)}), flush=True)
