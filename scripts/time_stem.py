"""ResNet stem forward at batch 256: csrc/stem.hip (conv + BN statistics
epilogue, then BN+ReLU+max-pool from those sums) vs MIOpen conv2d + the
pooling op computing its own statistics.  One JSON line per variant: median us.
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from kubedl_amd.ops import _ext  # noqa: E402
from kubedl_amd.ops.conv import stem_weights  # noqa: E402

ext = _ext.load()
dev = torch.device("cuda", 0)


def timed(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) * 1e3 for a, b in ev)


def main():
    nb = int(os.environ.get("NB", "256"))
    x = torch.randn(nb, 224, 224, 3, device=dev).bfloat16().permute(0, 3, 1, 2)
    w = (torch.randn(64, 3, 7, 7, device=dev) / 12).bfloat16().contiguous(memory_format=torch.channels_last)
    wp = stem_weights(w)
    y = torch.empty(nb, 64, 112, 112, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
    g, b = torch.ones(64, device=dev, dtype=torch.bfloat16), torch.zeros(64, device=dev, dtype=torch.bfloat16)
    ws = torch.zeros(ext.bn_workspace_floats(64), device=dev)
    res = {
        "kdl_stem_plain": timed(lambda: ext.stem7x7_fwd(x, wp, y, None, None)),
        "kdl_stem_stats": timed(lambda: ext.stem7x7_fwd(x, wp, y, rm, ws[:32 * 128])),
        "stem_weights": timed(lambda: stem_weights(w)),
        "miopen_conv": timed(lambda: F.conv2d(x, w, stride=2, padding=3)),
        "bn_pool_own_stats": timed(lambda: ext.bn_pool_fwd(y, g, b, rm, rv, True, 0.1, 1e-5, ws, False, False)),
        "bn_pool_gemm_stats": timed(lambda: ext.bn_pool_fwd(y, g, b, rm, rv, True, 0.1, 1e-5, ws, True, True)),
    }
    dy = torch.randn(nb, 112, 112, 64, device=dev).bfloat16().permute(0, 3, 1, 2)
    wsw = torch.empty(ext.stem7x7_wgrad_slabs(nb) * 64 * 224, device=dev)
    dwk = torch.empty(64, 224, device=dev, dtype=torch.bfloat16)
    res["kdl_stem_wgrad"] = timed(lambda: ext.stem7x7_wgrad(dy, x, wsw, dwk))
    res["miopen_stem_wgrad"] = timed(lambda: torch.ops.aten.convolution_backward(
        dy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1, [False, True, False]))
    c0 = y
    _, _, _, idx, xam = ext.bn_pool_fwd(c0, g, b, rm, rv, True, 0.1, 1e-5, ws, False, True)
    dp = torch.randn(nb, 56, 56, 64, device=dev).bfloat16().permute(0, 3, 1, 2)
    mean, inv = torch.zeros(64, device=dev), torch.ones(64, device=dev)

    def unfused():
        dx = ext.bn_pool_bwd(dp, idx, c0, g, b, mean, inv, True, ws, True)[0]
        ext.stem7x7_wgrad(dx, x, wsw, dwk)

    dg, db = torch.empty_like(g), torch.empty_like(b)

    def fused():
        ext.bn_stage_bwd_reduce(dp, xam, g, b, mean, inv, ws, dp.numel() // 64, 64, True)
        ext.bn_stage_bwd_finalize(ws, c0.numel() // 64, 64, g, mean, inv, dg, db, True)
        ext.stem7x7_wgrad_bn(c0, dp, idx, ws, x, wsw, dwk)
    res["bn_sums_over_cells"] = timed(lambda: ext.bn_stage_bwd_reduce(dp, xam, g, b, mean, inv, ws,
                                                                      dp.numel() // 64, 64, True))
    res["stem_bwd_unfused"] = timed(unfused)
    res["stem_bwd_fused"] = timed(fused)
    res["bn_pool_bwd_sums_only"] = timed(lambda: ext.bn_pool_bwd(dp, idx, c0, g, b, mean, inv, True, ws, False))
    res["kdl_stem_wgrad_bn"] = timed(lambda: ext.stem7x7_wgrad_bn(c0, dp, idx, ws, x, wsw, dwk))
    for bits, name in ((1, "no_mfma"), (2, "no_epilogue"), (4, "no_input"), (3, "no_mfma_no_epi"),
                       (6, "mfma_only"), (5, "epilogue_only")):
        ext.set_stem_drop(bits)
        res[f"kdl_stem_plain_{name}"] = timed(lambda: ext.stem7x7_fwd(x, wp, y, None, None))
        res[f"kdl_stem_stats_{name}"] = timed(lambda: ext.stem7x7_fwd(x, wp, y, rm, ws[:32 * 128]))
    ext.set_stem_drop(0)
    flop = 2 * nb * 112 * 112 * 64 * 147
    for k, v in res.items():
        print(json.dumps({"nb": nb, "variant": k, "us": round(v, 1), "TFps": round(flop / v / 1e6, 1),
                          "out_TBps": round(nb * 112 * 112 * 64 * 2 / v / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
