"""Run ONE conv-GEMM configuration a few times (for rocprofv3 --pmc passes).

usage: igemm_one.py 1x1 M N K cfg [iters]
       igemm_one.py 3x3 nb H Cin Cout stride cfg [iters]
cfg: igemm tile config (0..6), or -1 for the register-staged kernel.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kubedl_amd.ops import _ext  # noqa: E402

ext = _ext.load()
dev = torch.device("cuda", 0)


def main(argv):
    op = argv[0]
    if op == "1x1":
        M, N, K, cfg = (int(v) for v in argv[1:5])
        iters = int(argv[5]) if len(argv) > 5 else 5
        A = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        shift = torch.zeros(N, device=dev)
        ws = torch.zeros(ext.bn_workspace_floats(N), device=dev)
        ext.set_gemm_core(0 if cfg < 0 else 1)
        ext.set_igemm_cfg(cfg)
        for _ in range(iters):
            ext.conv1x1_gemm(A, W, C, M, N, K, 0, 0, 0, 0, 1, None, 1, shift, ws, None, None, None, None, 1, 0, 0,
                             None, None, None, None)
    else:
        nb, H, Cin, Cout, stride, cfg = (int(v) for v in argv[1:7])
        iters = int(argv[7]) if len(argv) > 7 else 5
        x = torch.randn(nb, H, H, Cin, device=dev).bfloat16().permute(0, 3, 1, 2)
        w = (torch.randn(Cout, 3, 3, Cin, device=dev) / (3 * Cin ** 0.5)).bfloat16().permute(0, 3, 1, 2)
        Ho = (H - 1) // stride + 1
        y = torch.empty(nb, Ho, Ho, Cout, device=dev, dtype=torch.bfloat16).permute(0, 3, 1, 2)
        shift = torch.zeros(Cout, device=dev)
        acc = torch.zeros(32 * 2 * Cout, device=dev)
        ext.set_gemm_core(0 if cfg < 0 else 1)
        ext.set_igemm_cfg(cfg)
        for _ in range(iters):
            ext.conv3x3_gemm(x, w, y, nb, H, H, Cin, Cout, stride, None, 1, shift, acc, None, None, None)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main(sys.argv[1:])
