"""hipBLASLt (torch.mm) vs the fused 1x1 GEMM kernels on ResNet-50's deep-stage shapes (batch 256)."""
import os
import sys
import torch
sys.path.insert(0, os.environ.get("KDL_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubedl_amd.ops import _ext  # noqa: E402

ext = _ext.load()


def t(fn, reps=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for (K, N, h) in [(64, 256, 56), (256, 64, 56), (128, 512, 28), (512, 128, 28), (256, 1024, 14), (1024, 256, 14),
                  (512, 2048, 7), (2048, 512, 7)]:
    M = 256 * h * h
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    g = torch.randn(M, N, device="cuda").bfloat16()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    dw32 = torch.empty(ext.conv1x1_wgrad_splits(M, N, K) * N * K, device="cuda")
    dW = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    fl = 2 * M * N * K / 1e6
    t_mm = t(lambda: torch.mm(x, w.t(), out=y))
    t_k = t(lambda: ext.conv1x1_gemm(x, w, y, M, N, K, 0, 0, 0, 0, 1, None, 0, None, None, None, None, None, None, 1, 0,
                                     0, None, None, None, None))
    t_wmm = t(lambda: torch.mm(g.t(), x, out=dW))
    t_wk = t(lambda: ext.conv1x1_wgrad(g, x, None, dw32, dW, 1.0, M, N, K, 0, 0, 0, 0, 1))
    print(f"K={K:5d} N={N:5d} hw={h:3d}  fwd: mm {t_mm:7.1f} us ({fl / t_mm:6.1f} TF/s)  kdl {t_k:7.1f} us "
          f"({fl / t_k:6.1f})   wgrad: mm {t_wmm:7.1f} us ({fl / t_wmm:6.1f})  kdl {t_wk:7.1f} us ({fl / t_wk:6.1f})",
          flush=True)
