"""Time the fused 1x1 GEMM (csrc/conv1x1.hip) on ResNet-50 stage shapes, batch 256.

Prints one line per (K, N, H, epilogue, prologue) with the achieved HBM rate of
the bytes the kernel must move (A + C + epilogue operands).
"""
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


CASES = [(64, 256, 56, 1, 0), (64, 256, 56, 0, 0), (64, 256, 56, 3, 0), (256, 64, 56, 1, 1), (256, 64, 56, 2, 0),
         (128, 512, 28, 1, 1), (512, 128, 28, 3, 0), (256, 1024, 14, 1, 1), (1024, 256, 14, 2, 0),
         (512, 2048, 7, 1, 1), (2048, 512, 7, 3, 0)]
total = 0.0
for (K, N, h, epi, pro) in CASES:
    M = 256 * h * h
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ws = torch.zeros(ext.bn_workspace_floats(N), device="cuda")
    acc = ws[:32 * 2 * N]
    sh = torch.zeros(N, device="cuda")
    ex = torch.randn(M, N, device="cuda").bfloat16()
    bits = torch.randint(0, 256, (M * N // 8,), device="cuda", dtype=torch.uint8)
    mean = torch.zeros(N, device="cuda")
    coef = torch.cat([torch.ones(N, device="cuda"), torch.zeros(N, device="cuda")])
    pcoef = torch.cat([torch.ones(K, device="cuda"), torch.zeros(K, device="cuda")]) if pro else None
    gb = M * (K + N) * 2
    if epi == 1:
        args = (1, sh, acc, None, None, None, None, 1, 0, 0, None, None, None, None)
    elif epi == 2:
        args = (2, None, acc, ex, mean, coef, None, 1, 0, 0, None, None, None, None)
        gb += M * N * 2
    elif epi == 3:
        args = (3, None, acc, ex, mean, None, ex, 1, h, h, bits, None, None, None)
        gb += M * N * 4 + M * N // 8
    else:
        args = (0, None, None, None, None, None, None, 1, 0, 0, None, None, None, None)
    f = lambda: ext.conv1x1_gemm(x, w, y, M, N, K, 0, 0, 0, 0, 1, pcoef, *args)
    us = t(f)
    total += us
    print(f"K={K:5d} N={N:5d} hw={h:3d} epi={epi} pro={pro}: {us:8.1f} us  {gb / us / 1e6:5.2f} TB/s", flush=True)
print(f"total {total:.1f} us")

# weight gradients dW[N, K] = G[M, N]^T A[M, K] (+ bf16 cast)
WCASES = [(64, 256, 56, 0), (256, 64, 56, 1), (64, 64, 56, 1), (128, 512, 28, 1), (512, 128, 28, 0),
          (256, 1024, 14, 1), (1024, 256, 14, 0), (512, 2048, 7, 1), (2048, 512, 7, 0)]
wtotal = 0.0
for (K, N, h, pro) in WCASES:
    M = 256 * h * h
    a = torch.randn(M, K, device="cuda").bfloat16()
    g = torch.randn(M, N, device="cuda").bfloat16()
    dw32 = torch.empty(ext.conv1x1_wgrad_splits(M, N, K) * N * K, device="cuda")
    dW = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    pcoef = torch.cat([torch.ones(K, device="cuda"), torch.zeros(K, device="cuda")]) if pro else None
    f = lambda: ext.conv1x1_wgrad(g, a, pcoef, dw32, dW, 1.0, M, N, K, 0, 0, 0, 0, 1)
    try:
        f()
    except RuntimeError:  # older builds: one zeroed [N, K] fp32 atomic accumulator
        dw32 = torch.zeros(N * K, device="cuda")
        f = lambda: ext.conv1x1_wgrad(g, a, pcoef, dw32, dW, 1.0, M, N, K, 0, 0, 0, 0, 1)
    us = t(f)
    wtotal += us
    gb = M * (K + N) * 2
    print(f"wgrad K={K:5d} N={N:5d} hw={h:3d} pro={pro}: {us:8.1f} us  {gb / us / 1e6:5.2f} TB/s "
          f"{2 * M * N * K / us / 1e6:6.1f} TF/s", flush=True)
print(f"wgrad total {wtotal:.1f} us")
