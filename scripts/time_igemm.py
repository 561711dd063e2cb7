"""Time the conv GEMM main loops on the ResNet-50 (batch 256) shapes.

Register-staged loop (csrc/conv1x1.hip) vs the LDS-DMA loop (csrc/igemm.hip,
every tile config) on 1x1 GEMMs, and the DMA loop's 3x3 implicit GEMM vs
MIOpen (F.conv2d), all on random bf16 data, one process, interleaved rounds.
Prints one JSON line per (shape, variant): median us and TF/s.
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from kubedl_amd.ops import _ext  # noqa: E402

ext = _ext.load()
dev = torch.device("cuda", 0)
REP = 32


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


def gemm1x1(A, W, C, M, N, K, epi, shift, ws):
    ext.conv1x1_gemm(A, W, C, M, N, K, 0, 0, 0, 0, 1, None, epi, shift, ws, None, None, None, None, 1, 0, 0,
                     None, None, None, None)


def variants():
    out = [("reg", 0, -1)]
    for cfg in [int(c) for c in os.environ.get("CFGS", "0,1,2,3,4").split(",")]:
        out.append((f"dma{cfg}", 1, cfg))
    return out


def run_1x1(M, N, K, rounds=3):
    A = torch.randn(M, K, device=dev).bfloat16()
    W = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    shift = torch.zeros(N, device=dev)
    ws = torch.zeros(ext.bn_workspace_floats(N), device=dev)
    res = {}
    for _ in range(rounds):
        for name, core, cfg in variants():
            if cfg in (0,) and N % 256 or cfg in (1, 2, 4, 5, 9) and N % 128:
                continue
            ext.set_gemm_core(core)
            ext.set_igemm_cfg(cfg)
            res.setdefault(name, []).append(timed(lambda: gemm1x1(A, W, C, M, N, K, 1, shift, ws)))
    ext.set_gemm_core(-1)
    ext.set_igemm_cfg(-1)
    fl = 2.0 * M * N * K
    for name, ts in res.items():
        us = min(ts)
        print(json.dumps({"op": "1x1", "M": M, "N": N, "K": K, "variant": name, "us": round(us, 1),
                          "tflops": round(fl / us / 1e6, 1)}), flush=True)


def run_3x3(nb, H, Cin, Cout, stride, rounds=3):
    x = torch.randn(nb, H, H, Cin, device=dev).bfloat16().permute(0, 3, 1, 2)
    w = (torch.randn(Cout, 3, 3, Cin, device=dev) / (3 * Cin ** 0.5)).bfloat16().permute(0, 3, 1, 2)
    Ho = (H - 1) // stride + 1
    y = torch.empty(nb, Ho, Ho, Cout, device=dev, dtype=torch.bfloat16).permute(0, 3, 1, 2)
    shift = torch.zeros(Cout, device=dev)
    acc = torch.zeros(REP * 2 * Cout, device=dev)
    res = {}
    for _ in range(rounds):
        res.setdefault("miopen", []).append(timed(lambda: F.conv2d(x, w, stride=stride, padding=1)))
        for name, core, cfg in variants() + [("halo", 1, -1)]:
            if cfg in (0,) and Cout % 256 or cfg in (1, 2, 4, 5, 9) and Cout % 128:
                continue
            ext.set_halo3x3(1 if name == "halo" else 0)
            ext.set_gemm_core(core)
            ext.set_igemm_cfg(cfg)
            res.setdefault(name, []).append(timed(
                lambda: ext.conv3x3_gemm(x, w, y, nb, H, H, Cin, Cout, stride, None, 1, shift, acc, None, None, None)))
    ext.set_gemm_core(-1)
    ext.set_igemm_cfg(-1)
    ext.set_halo3x3(1)
    fl = 2.0 * nb * Ho * Ho * Cout * 9 * Cin
    for name, ts in res.items():
        us = min(ts)
        print(json.dumps({"op": "3x3", "nb": nb, "H": H, "Cin": Cin, "Cout": Cout, "stride": stride, "variant": name,
                          "us": round(us, 1), "tflops": round(fl / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    torch.manual_seed(0)
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "1x1"):
        for M, N, K in [(50176, 256, 1024), (12544, 512, 2048), (200704, 128, 512), (50176, 1024, 256),
                        (12544, 2048, 512), (802816, 64, 256)]:
            run_1x1(M, N, K)
    if which == "n128":
        run_1x1(200704, 128, 512)
        for nb, H, Cin, Cout, s in [(256, 28, 128, 128, 1), (256, 56, 128, 128, 2)]:
            run_3x3(nb, H, Cin, Cout, s)
    if which in ("all", "3x3"):
        for nb, H, Cin, Cout, s in [(256, 56, 64, 64, 1), (256, 28, 128, 128, 1), (256, 14, 256, 256, 1),
                                    (256, 7, 512, 512, 1), (256, 56, 128, 128, 2), (256, 28, 256, 256, 2),
                                    (256, 14, 512, 512, 2)]:
            run_3x3(nb, H, Cin, Cout, s)


def run_wgrad_1x1(M, N, K, rounds=3):
    A = torch.randn(M, K, device=dev).bfloat16()
    G = torch.randn(M, N, device=dev).bfloat16()
    ws = torch.empty(ext.conv1x1_wgrad_splits(M, N, K) * N * K, device=dev)
    dW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    res = {}
    for _ in range(rounds):
        for name, core in (("reg", 0), ("dma", 1)):
            ext.set_gemm_core(core)
            res.setdefault(name, []).append(timed(
                lambda: ext.conv1x1_wgrad(G, A, None, ws, dW, 1.0, M, N, K, 0, 0, 0, 0, 1)))
    ext.set_gemm_core(-1)
    fl = 2.0 * M * N * K
    for name, ts in res.items():
        us = min(ts)
        print(json.dumps({"op": "wgrad1x1", "M": M, "N": N, "K": K, "variant": name, "us": round(us, 1),
                          "tflops": round(fl / us / 1e6, 1)}), flush=True)


def run_wgrad_3x3(nb, H, Cin, Cout, stride, rounds=3):
    x = torch.randn(nb, H, H, Cin, device=dev).bfloat16().permute(0, 3, 1, 2)
    w = (torch.randn(Cout, 3, 3, Cin, device=dev) / (3 * Cin ** 0.5)).bfloat16().permute(0, 3, 1, 2)
    Ho = (H - 1) // stride + 1
    dy = torch.randn(nb, Ho, Ho, Cout, device=dev).bfloat16().permute(0, 3, 1, 2)
    M = nb * Ho * Ho
    ws = torch.empty(ext.conv3x3_wgrad_slabs(nb, H, H, Cin, Cout, stride) * Cout * 9 * Cin, device=dev)
    dW = torch.empty(Cout, 3, 3, Cin, device=dev, dtype=torch.bfloat16).permute(0, 3, 1, 2)
    res = {}
    for _ in range(rounds):
        res.setdefault("miopen", []).append(timed(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [stride, stride], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])))
        for name, core in (("reg", 0), ("dma", 1)):
            ext.set_gemm_core(core)
            res.setdefault(name, []).append(timed(
                lambda: ext.conv3x3_wgrad(dy, x, None, ws, dW, 1.0, nb, H, H, Cin, Cout, stride)))
    ext.set_gemm_core(-1)
    fl = 2.0 * M * Cout * 9 * Cin
    for name, ts in res.items():
        us = min(ts)
        print(json.dumps({"op": "wgrad3x3", "nb": nb, "H": H, "Cin": Cin, "Cout": Cout, "stride": stride,
                          "variant": name, "us": round(us, 1), "tflops": round(fl / us / 1e6, 1)}), flush=True)


if __name__ == "__main__" and (len(sys.argv) > 1 and sys.argv[1] in ("all", "wgrad")):
    for M, N, K in [(50176, 256, 1024), (12544, 512, 2048), (200704, 128, 512), (802816, 256, 64),
                    (802816, 64, 256), (50176, 1024, 256)]:
        run_wgrad_1x1(M, N, K)
    for nb, H, Cin, Cout, s in [(256, 56, 64, 64, 1), (256, 28, 128, 128, 1), (256, 14, 256, 256, 1),
                                (256, 7, 512, 512, 1), (256, 56, 128, 128, 2), (256, 28, 256, 256, 2),
                                (256, 14, 512, 512, 2)]:
        run_wgrad_3x3(nb, H, Cin, Cout, s)
