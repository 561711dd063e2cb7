"""Time the CTR tower's forward GEMMs (batch 4096: 1728 -> 1024 -> 512 -> 256) on
the register-staged gemm_bias_act kernel vs the LDS-DMA igemm loop with the
BIAS_RELU epilogue (csrc/ctr.hip ctr_igemm_cfg_for), per igemm tile config.

python scripts/ctr_igemm_probe.py [reps]
"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kubedl_amd.ops import _ext  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    ext = _ext.load()
    shapes = [(4096, 1024, 1728), (4096, 512, 1024), (4096, 256, 512)]
    torch.manual_seed(0)
    for M, N, K in shapes:
        a = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16()
        ref = None
        row = []
        for name, mode, cfg in [("reg", 0, -1), ("auto", 1, -1), ("ig-c0", 2, 0), ("ig-c1", 2, 1), ("ig-c2", 2, 2),
                                ("ig-c3", 2, 3), ("ig-c4", 2, 4)]:
            ext.set_ctr_igemm(mode, cfg)
            if mode == 2:
                bn = 256 if cfg == 0 else 64 if cfg == 3 else 128
                if N % bn:
                    continue
            y = ext.gemm_bias_act(a, w, b, True)
            if ref is None:
                ref = y.float()
            err = (y.float() - ref).abs().max().item()
            for _ in range(10):
                ext.gemm_bias_act(a, w, b, True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(reps):
                ext.gemm_bias_act(a, w, b, True)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
            row.append(f"{name} {us:6.1f} us {tf:5.0f} TF/s (max|d| vs reg {err:.3g})")
        ext.set_ctr_igemm(-2, -2)
        print(f"M={M} N={N} K={K}: " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
