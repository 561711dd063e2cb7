"""Stride-2 3x3 data gradient on the ResNet-50 (batch 256) shapes: the kdl
sub-pixel class GEMMs (PLAIN and MASKX epilogues, every LDS-DMA tile config)
vs MIOpen's data gradient (+ the BN-backward reduce pass the MASKX epilogue
replaces).  One JSON line per (shape, variant): median us.
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kubedl_amd.ops import _ext  # noqa: E402
from kubedl_amd.ops.conv import s2_dgrad_weights  # noqa: E402

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


def nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def main():
    nb = int(os.environ.get("NB", "256"))
    for C, Hd in [(128, 28), (256, 14), (512, 7)]:
        dy = nhwc(torch.randn(nb, C, Hd, Hd, device=dev).bfloat16())
        w = nhwc((torch.randn(C, C, 3, 3, device=dev) / (3 * C ** 0.5)).bfloat16())
        ball = s2_dgrad_weights(w)
        x1 = nhwc(torch.randn(nb, C, 2 * Hd, 2 * Hd, device=dev).bfloat16())
        dx = torch.empty_like(x1)
        coef = torch.cat([torch.ones(C, device=dev), torch.zeros(C, device=dev)])
        mean = torch.zeros(C, device=dev)
        acc = torch.zeros(REP * 2 * C, device=dev)
        ws = torch.zeros(ext.bn_workspace_floats(C), device=dev)
        gam = torch.ones(C, device=dev, dtype=torch.bfloat16)
        bet = torch.zeros(C, device=dev, dtype=torch.bfloat16)
        inv = torch.ones(C, device=dev)
        flop = 2 * nb * (2 * Hd) ** 2 * C * 9 * C / 4
        res = {}
        for cfg in (-1, 0, 1, 2, 3):
            if cfg == 0 and C % 256:
                continue
            ext.set_igemm_cfg(cfg)
            res[f"kdl_plain_cfg{cfg}"] = timed(lambda: ext.conv3x3_s2_dgrad(dy, ball, dx, nb, Hd, Hd, C, C, 0, None,
                                                                             None, None, None))
            res[f"kdl_maskx_cfg{cfg}"] = timed(lambda: ext.conv3x3_s2_dgrad(dy, ball, dx, nb, Hd, Hd, C, C, 2, acc,
                                                                             x1, mean, coef))
        ext.set_igemm_cfg(-1)

        def miopen():
            return torch.ops.aten.convolution_backward(dy, x1, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1,
                                                       [True, False, False])[0]
        res["miopen_dgrad"] = timed(miopen)
        da = miopen().contiguous(memory_format=torch.channels_last)
        M = nb * 4 * Hd * Hd
        res["bn_bwd_reduce_pass"] = timed(lambda: ext.bn_stage_bwd_reduce(da, x1, gam, bet, mean, inv, ws, M, C, True))
        for k, v in res.items():
            print(json.dumps({"C": C, "Hd": Hd, "nb": nb, "variant": k, "us": round(v, 1),
                              "TFps": round(flop / v / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
