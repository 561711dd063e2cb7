"""Time the BN apply / reduce passes on the ResNet-50 (batch 256) tensor shapes
and print achieved HBM bandwidth (bytes the pass must move / time).

usage: bench_bn.py   (one JSON line per (kernel, shape))
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kubedl_amd.ops import _ext  # noqa: E402

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
    for hw, C in [(56 * 56, 256), (56 * 56, 64), (28 * 28, 512), (14 * 14, 1024), (7 * 7, 2048)]:
        M = 256 * hw
        x = torch.randn(M, C, device=dev).bfloat16()
        g = torch.randn(M, C, device=dev).bfloat16()
        r = torch.randn(M, C, device=dev).bfloat16()
        ws = torch.zeros(ext.bn_workspace_floats(C), device=dev)
        y = torch.empty_like(x)
        mb = torch.empty(M * C // 8, dtype=torch.uint8, device=dev)
        nbytes = M * C * 2
        t = timed(lambda: ext.bn_stage_bwd_apply(g, x, ws, y, None, None, None, M, C))
        print(json.dumps({"kernel": "bwd_apply", "M": M, "C": C, "us": round(t, 1),
                          "TBps": round(3 * nbytes / t / 1e6, 2)}), flush=True)
        t = timed(lambda: ext.bn_stage_fwd_apply(x, ws, r, None, None, y, mb, M, C, True))
        print(json.dumps({"kernel": "fwd_apply_res_relu_mask", "M": M, "C": C, "us": round(t, 1),
                          "TBps": round((3 * nbytes + nbytes // 16) / t / 1e6, 2)}), flush=True)
        t = timed(lambda: ext.bn_stage_fwd_apply(x, ws, None, None, None, y, None, M, C, True))
        print(json.dumps({"kernel": "fwd_apply_relu", "M": M, "C": C, "us": round(t, 1),
                          "TBps": round(2 * nbytes / t / 1e6, 2)}), flush=True)
        t = timed(lambda: y.copy_(x))
        print(json.dumps({"kernel": "torch_copy", "M": M, "C": C, "us": round(t, 1),
                          "TBps": round(2 * nbytes / t / 1e6, 2)}), flush=True)
        del x, g, r, y, mb


if __name__ == "__main__":
    main()
