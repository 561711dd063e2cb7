"""Per-layer A/B of ResNet-50's 1x1 convs: MIOpen (via aten) vs the fused
kdl MFMA GEMMs (csrc/conv1x1.hip), batch 256, bf16 NHWC, on one MI355X.

For every distinct 1x1 layer shape: forward (ours with the BN-stats
epilogue, plus the prologue where the layer consumes a BN+ReLU), data
gradient (ours plain and with the MASKX epilogue), weight gradient, and the
standalone BN stats pass that the STATS epilogue replaces.  Prints one JSON
line per layer and a weighted total (ms per training step).
"""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from kubedl_amd.ops import _ext  # noqa: E402

# (cin, cout, hin, stride, prologue, count) -- ResNet-50 v1.5 bottleneck 1x1 convs
LAYERS = [
    (64, 64, 56, 1, False, 1), (64, 256, 56, 1, True, 3), (64, 256, 56, 1, False, 1), (256, 64, 56, 1, False, 2),
    (256, 128, 56, 1, False, 1), (128, 512, 28, 1, True, 4), (256, 512, 56, 2, False, 1), (512, 128, 28, 1, False, 3),
    (512, 256, 28, 1, False, 1), (256, 1024, 14, 1, True, 6), (512, 1024, 28, 2, False, 1),
    (1024, 256, 14, 1, False, 5),
    (1024, 512, 14, 1, False, 1), (512, 2048, 7, 1, True, 3), (1024, 2048, 14, 2, False, 1),
    (2048, 512, 7, 1, False, 2),
]


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ext = _ext.load()
    torch.backends.cudnn.benchmark = False
    dev = "cuda"
    B = 256
    tot = {}
    for cin, cout, h, s, pro, cnt in LAYERS:
        ho = (h - 1) // s + 1
        M = B * ho * ho
        x = torch.randn(B, cin, h, h, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, 1, 1, device=dev) / cin ** 0.5).bfloat16().contiguous(
            memory_format=torch.channels_last)
        wt = w.view(cout, cin).t().contiguous()
        dy = torch.randn(B, cout, ho, ho, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        y = torch.empty_like(dy)
        dx = torch.empty_like(x) if s == 1 else torch.empty(B, cin, ho, ho, device=dev, dtype=torch.bfloat16
                                                            ).contiguous(memory_format=torch.channels_last)
        ws = torch.zeros(ext.bn_workspace_floats(cout), device=dev)
        wsi = torch.zeros(ext.bn_workspace_floats(cin), device=dev)
        shift = torch.zeros(cout, device=dev)
        coef = torch.cat([torch.ones(cin, device=dev), torch.zeros(cin, device=dev)])
        mean_in = torch.zeros(cin, device=dev)
        r = {"cin": cin, "cout": cout, "hw": h, "stride": s, "count": cnt}
        r["miopen_fwd"] = timeit(lambda: torch.nn.functional.conv2d(x, w, stride=s))
        r["kdl_fwd_stats"] = timeit(lambda: ext.conv1x1_gemm(
            x, w, y, M, cout, cin, ho, ho, h, h, s, coef if pro else None, 1, shift, ws, None, None, None, None, 1,
            0, 0, None, None, None, None))
        r["bn_stats_pass"] = timeit(lambda: ext.bn_stage_fwd_stats(y, ws, M, cout))
        r["miopen_dgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False]))
        if s == 1:
            r["kdl_dgrad"] = timeit(lambda: ext.conv1x1_gemm(
                dy, wt, dx, M, cin, cout, 0, 0, 0, 0, 1, None, 0, None, None, None, None, None, None, 1, 0, 0, None,
                None, None, None))
            r["kdl_dgrad_maskx"] = timeit(lambda: ext.conv1x1_gemm(
                dy, wt, dx, M, cin, cout, 0, 0, 0, 0, 1, None, 2, None, wsi, x, mean_in, coef, None, 1, 0, 0, None,
                None, None, None))
            bits = torch.randint(0, 256, (M * cin // 8,), device=dev, dtype=torch.uint8)
            r["kdl_dgrad_resbits"] = timeit(lambda: ext.conv1x1_gemm(
                dy, wt, dx, M, cin, cout, 0, 0, 0, 0, 1, None, 3, None, wsi, x, mean_in, None, x, 1, h, h, bits,
                None, None, None))
        else:
            dxs = torch.empty(M, cin, device=dev, dtype=torch.bfloat16)
            r["kdl_dgrad"] = timeit(lambda: ext.conv1x1_gemm(
                dy, wt, dxs, M, cin, cout, 0, 0, 0, 0, 1, None, 0, None, None, None, None, None, None, 1, 0, 0, None,
                None, None, None))
        r["miopen_wgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]))
        dw32 = torch.empty(ext.conv1x1_wgrad_splits(M, cout, cin) * cout * cin, device=dev)
        dw = torch.empty(cout, cin, device=dev, dtype=torch.bfloat16)
        r["kdl_wgrad"] = timeit(lambda: ext.conv1x1_wgrad(dy, x, coef if pro else None, dw32, dw, 1.0, M, cout, cin,
                                                          ho, ho, h, h, s))
        gb = (M * cin + M * cout) * 2 / 1e9
        r["kdl_fwd_TBps"] = gb / (r["kdl_fwd_stats"] * 1e-3) / 1e3
        for k, v in r.items():
            if k.startswith(("miopen", "kdl", "bn_")) and not k.endswith("TBps"):
                tot[k] = tot.get(k, 0.0) + v * cnt
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    print(json.dumps({"total_ms_per_step": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
