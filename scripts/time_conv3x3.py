"""ResNet-50 3x3 convs (batch 256): MIOpen (F.conv2d / convolution_backward) vs the
implicit-GEMM kernels (fwd with BN+ReLU prologue + stats epilogue; stride-1 dgrad
with the mask+BN-sums epilogue; wgrad with the BN+ReLU prologue)."""
import os
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubedl_amd.ops import _ext  # noqa: E402

ext = _ext.load()
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "miopen_db", "user"))


def t(fn, reps=20):
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


nb = 256
tot = {}
for (C, H, s, cnt) in [(64, 56, 1, 3), (128, 56, 2, 1), (128, 28, 1, 3), (256, 28, 2, 1), (256, 14, 1, 5),
                       (512, 14, 2, 1), (512, 7, 1, 2)]:
    x = torch.randn(nb, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, C, 3, 3, device="cuda") / (3 * C ** 0.5)).bfloat16().contiguous(memory_format=torch.channels_last)
    Ho = (H - 1) // s + 1
    y = torch.empty(nb, C, Ho, Ho, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn_like(y)
    coef = torch.cat([torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")])
    shift = torch.zeros(C, device="cuda")
    acc = torch.zeros(32 * 2 * C, device="cuda")
    M = nb * Ho * Ho
    fl = 2 * M * C * C * 9 / 1e6
    r = {}
    r["miopen_fwd"] = t(lambda: F.conv2d(x, w, stride=s, padding=1))
    r["kdl_fwd"] = t(lambda: ext.conv3x3_gemm(x, w, y, nb, H, H, C, C, s, coef, 1, shift, acc, None, None, None))
    r["miopen_bwd_data"] = t(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [1, 1], [1, 1], False,
                                                                           [0, 0], 1, [True, False, False]))
    if s == 1:
        wd = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x)
        r["kdl_dgrad"] = t(lambda: ext.conv3x3_gemm(dy, wd, dx, nb, H, H, C, C, 1, None, 2, None, acc, x, shift, coef))
    r["miopen_bwd_weight"] = t(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [1, 1], [1, 1],
                                                                             False, [0, 0], 1, [False, True, False]))
    ws = torch.empty(ext.conv1x1_wgrad_splits(M, C, 9 * C) * C * 9 * C, device="cuda")
    dW = torch.empty_like(w)
    r["kdl_wgrad"] = t(lambda: ext.conv3x3_wgrad(dy, x, coef, ws, dW, 1.0, nb, H, H, C, C, s))
    for k, v in r.items():
        tot[k] = tot.get(k, 0.0) + v * cnt
    print(f"C={C:4d} H={H:3d} s={s} x{cnt}: " + "  ".join(f"{k} {v:7.1f}us({fl / v:5.0f}TF)" for k, v in r.items()),
          flush=True)
print("per-step totals (us): " + "  ".join(f"{k} {v:.0f}" for k, v in tot.items()))
