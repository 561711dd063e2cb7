"""Run the fused stem backward weight gradient (csrc/stem.hip stem7x7_wgrad_bn)
alone, batch 256 at 224 px, for rocprofv3 timing / PMC passes (the BN
workspace is zero: the work per tile does not depend on the values)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubedl_amd.ops import _ext  # noqa: E402


def main():
    ext = _ext.load()
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    Nb = 256
    cl = torch.channels_last
    x = torch.randn(Nb, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=cl)
    c0 = torch.randn(Nb, 64, 112, 112, device="cuda").bfloat16().contiguous(memory_format=cl)
    dp = torch.randn(Nb, 64, 56, 56, device="cuda").bfloat16().contiguous(memory_format=cl)
    idx = torch.randint(0, 9, (Nb * 56 * 56 * 64,), device="cuda", dtype=torch.uint8)
    ws = torch.zeros(ext.bn_workspace_floats(64), device="cuda")
    dw32 = torch.empty(ext.stem7x7_wgrad_slabs(Nb, 224, 224) * 64 * 224, device="cuda")
    dW = torch.empty(64, 3, 7, 7, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
    for _ in range(reps):
        ext.stem7x7_wgrad_bn(c0, dp, idx, ws, x, dw32, dW)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
