"""Per-layer timing of ResNet-50 convs at batch 256 (bf16, channels_last):
MIOpen conv2d fwd / bwd-data / bwd-weight vs. the same 1x1 stride-1 conv as
plain GEMMs (torch.mm -> hipBLASLt) and our MFMA kernel.  Decides which convs
the model should route through GEMMs.  Prints one line per layer + totals
(ms per training step, each layer weighted by how often it occurs)."""
import argparse
import json
import os

import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(_ROOT, "miopen_db", "user"))
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(_ROOT, "miopen_db", "cache"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

N = 256
# (cin, cout, k, stride, hw_in, count)
LAYERS = [(3, 64, 7, 2, 224, 1)]
for w, n, hw in ((64, 3, 56), (128, 4, 28), (256, 6, 14), (512, 3, 7)):
    cin = 64 if w == 64 else 2 * w
    for b in range(n):
        first = b == 0
        s = 2 if (first and w != 64) else 1
        hin = hw * s
        LAYERS.append(((cin if first else 4 * w), w, 1, 1, hin, 1))   # conv1
        LAYERS.append((w, w, 3, s, hin, 1))                            # conv2
        LAYERS.append((w, 4 * w, 1, 1, hw, 1))                          # conv3
        if first:
            LAYERS.append((cin, 4 * w, 1, s, hin, 1))                   # downsample


def merge(layers):
    d = {}
    for l in layers:
        d[l[:5]] = d.get(l[:5], 0) + l[5]
    return [k + (v,) for k, v in d.items()]


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = False
    dev = "cuda"
    tot = {"conv": 0.0, "gemm": 0.0, "conv_1x1": 0.0}
    rows = []
    for cin, cout, k, s, hin, cnt in merge(LAYERS):
        x = torch.randn(N, cin, hin, hin, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16) * 0.05).to(
            memory_format=torch.channels_last)
        pad = k // 2
        y = F.conv2d(x, w, stride=s, padding=pad)
        dy = torch.randn_like(y)
        t_f = timeit(lambda: F.conv2d(x, w, stride=s, padding=pad), args.iters)
        t_bd = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [pad, pad], [1, 1], False,
                                                                  [0, 0], 1, [True, False, False]), args.iters)
        t_bw = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [pad, pad], [1, 1], False,
                                                                  [0, 0], 1, [False, True, False]), args.iters)
        conv = t_f + t_bd + t_bw
        row = {"cin": cin, "cout": cout, "k": k, "s": s, "hw": hin, "count": cnt,
               "conv_fwd": round(t_f, 4), "conv_bwd_data": round(t_bd, 4), "conv_bwd_wgt": round(t_bw, 4)}
        tot["conv"] += conv * cnt
        if k == 1 and s == 1:
            M = N * hin * hin
            a = x.permute(0, 2, 3, 1).reshape(M, cin)
            wm = w.reshape(cout, cin)
            g = dy.permute(0, 2, 3, 1).reshape(M, cout)
            g_f = timeit(lambda: torch.mm(a, wm.t()), args.iters)
            g_bd = timeit(lambda: torch.mm(g, wm), args.iters)
            g_bw = timeit(lambda: torch.mm(g.t(), a), args.iters)
            row.update(gemm_fwd=round(g_f, 4), gemm_bwd_data=round(g_bd, 4), gemm_bwd_wgt=round(g_bw, 4))
            if cin % 64 == 0:
                try:
                    from kubedl_amd.ops import _ext
                    ext = _ext.load()
                    row["kdl_mfma_fwd"] = round(timeit(lambda: ext.gemm_bias_act(a, wm, None, False), args.iters), 4)
                except Exception as e:  # noqa: BLE001
                    row["kdl_mfma_fwd"] = str(e)[:80]
            tot["gemm"] += min(g_f, t_f) * cnt + min(g_bd, t_bd) * cnt + min(g_bw, t_bw) * cnt
            tot["conv_1x1"] += conv * cnt
        else:
            tot["gemm"] += conv * cnt
        rows.append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps({"total_conv_ms": round(tot["conv"], 3), "total_best_of_ms": round(tot["gemm"], 3),
                      "conv_1x1_s1_ms": round(tot["conv_1x1"], 3)}), flush=True)


if __name__ == "__main__":
    main()
