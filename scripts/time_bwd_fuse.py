"""Per-layer A/B of the BN-backward-apply fusion (csrc/conv1x1.hip PRO_BWD,
csrc/wgrad_dma.hip BWDG) on the ResNet-50 b256 shapes, one process, arms
interleaved, events around 10 launches of each arm:

  U   bn_stage_bwd_apply(g, x) -> dc ; data gradient on dc (default routing)
  F1  data gradient on (g, x) with the apply in its A staging, dc written through
  F2  data gradient on (g, x), no write-through
and the weight gradient of the same layer on dc (U / F1) or on (g, x) (W2, BWDG).

Usage: python scripts/time_bwd_fuse.py [--reps 3]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from kubedl_amd.ops import _ext  # noqa: E402

ext = _ext.load()
dev = "cuda"


def nhwc(n, c, h, w):
    return torch.randn(n, c, h, w, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)


def ws_for(C):
    ws = torch.zeros(ext.bn_workspace_floats(C), device=dev)
    off = ext.bn_coef_offset(C)
    ws[off:off + 2 * C] = torch.rand(2 * C, device=dev)          # forward scale | shift (masks)
    ws[off + 2 * C:off + 5 * C] = torch.randn(3 * C, device=dev) * 0.1  # backward k | c1 | c0
    return ws


def gemm(A, B, C, M, N, K, epi=0, ex=None, emean=None, ecoef=None, acc=None, eres=None, ebits=None):
    ext.conv1x1_gemm(A, B, C, M, N, K, 0, 0, 0, 0, 1, None, epi, None, acc, ex, emean, ecoef, eres, 1, 0, 0, ebits,
                     None, None, None)


def timed(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def layer(name, nb, h, w, cg, cout, epi, wg_k, reps):
    """g, x: [nb, cg, h, w] (the BN's gradient and input); the dgrad GEMM is
    A [M, K=cg] . B [N=cout, K]^T with epilogue ``epi``; the weight gradient is
    G [M, cg]^T . X [M, wg_k]."""
    M = nb * h * w
    g, x = nhwc(nb, cg, h, w), nhwc(nb, cg, h, w)
    ws = ws_for(cg)
    wt = (torch.randn(cout, cg, device=dev) / cg ** 0.5).bfloat16()
    out = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
    dc = torch.empty_like(g)
    kw = {}
    wse = torch.zeros(ext.bn_workspace_floats(cout), device=dev)
    if epi == 2:
        kw = dict(ex=torch.randn(M, cout, device=dev).bfloat16(), emean=torch.randn(cout, device=dev),
                  ecoef=torch.randn(2 * cout, device=dev), acc=wse)
    elif epi == 3:
        kw = dict(ex=torch.randn(M, cout, device=dev).bfloat16(), emean=torch.randn(cout, device=dev), acc=wse,
                  eres=torch.randn(M, cout, device=dev).bfloat16(),
                  ebits=torch.randint(0, 256, (M, cout // 8), device=dev, dtype=torch.uint8))
    xa = nhwc(nb, wg_k, h, w)
    dW = torch.empty(cg, wg_k, device=dev, dtype=torch.bfloat16)
    dw32 = torch.empty(ext.conv1x1_wgrad_splits(M, cg, wg_k) * cg * wg_k, device=dev)

    def apply():
        ext.bn_stage_bwd_apply(g, x, ws, dc, None, None, None, M, cg)

    def d_unfused():
        gemm(dc, wt, out, M, cout, cg, epi, **kw)

    def d_f1():
        ext.bn_bwd_pro_arm(x, ws, cg, dc)
        gemm(g, wt, out, M, cout, cg, epi, **kw)

    def d_f2():
        ext.bn_bwd_pro_arm(x, ws, cg, None)
        gemm(g, wt, out, M, cout, cg, epi, **kw)

    def w_plain():
        ext.conv1x1_wgrad(dc, xa, None, dw32, dW, 1.0, M, cg, wg_k, 0, 0, 0, 0, 1)

    def w_bwdg():
        ext.bn_bwd_pro_arm(x, ws, cg, None)
        ext.conv1x1_wgrad(g, xa, None, dw32, dW, 1.0, M, cg, wg_k, 0, 0, 0, 0, 1)

    arms = {"apply": apply, "dgrad_U": d_unfused, "dgrad_F1": d_f1, "dgrad_F2": d_f2, "wgrad_U": w_plain,
            "wgrad_W2": w_bwdg}
    res = {k: [] for k in arms}
    for _ in range(reps):
        for k, f in arms.items():
            res[k].append(timed(f))
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    row = {"layer": name, "M": M, "K": cg, "N": cout, "epi": epi, "wg_k": wg_k}
    row.update({k: round(v, 1) for k, v in med.items()})
    row["main_U"] = round(med["apply"] + med["dgrad_U"], 1)
    row["main_F1"] = med["dgrad_F1"]
    row["main_F2"] = med["dgrad_F2"]
    row["all_U"] = round(med["apply"] + med["dgrad_U"] + med["wgrad_U"], 1)
    row["all_F1"] = round(med["dgrad_F1"] + med["wgrad_U"], 1)
    row["all_F2"] = round(med["dgrad_F2"] + med["wgrad_W2"], 1)
    print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    nb = 256
    # (name, h, cg = BN channels, cout = dgrad N, epi, wgrad K)
    for st, (h, c) in enumerate(((56, 64), (28, 128), (14, 256), (7, 512)), 1):
        layer(f"s{st}_bn3_conv3", nb, h, h, 4 * c, c, 2, c, a.reps)      # dc3 -> conv3 dgrad (MASKX) / wgrad
        layer(f"s{st}_bn1_conv1", nb, h, h, c, 4 * c, 3, 4 * c, a.reps)  # dc1 -> conv1 dgrad (RESBITS) / wgrad
    layer("s1_bnd_down", nb, 56, 56, 256, 64, 0, 64, a.reps)              # dcd -> downsample dgrad / wgrad


if __name__ == "__main__":
    main()
