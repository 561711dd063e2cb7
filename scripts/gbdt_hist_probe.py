"""Time the quantised GBDT histogram build standalone (gbdt_hist_quant: absmax +
plan + build + the output zero-fill) on 2M x 28 x 256 bins: the root (one node)
and a depth-6-like level (32 nodes over 1M rows), slot kernel vs row-per-lane
kernel (4 / 8 rows in flight), rows per chunk 1024 / 2048 / 4096.

python scripts/gbdt_hist_probe.py            (KDL_TUNE gbdt_price_noflush=1: the
                                              row-per-lane build without its flush)
"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kubedl_amd.ops import _ext  # noqa: E402


def main():
    ext = _ext.load()
    N, F, B = 2_000_000, 28, 256
    g0 = torch.Generator(device="cuda").manual_seed(0)
    bins = torch.randint(0, B, (N, F), device="cuda", generator=g0, dtype=torch.uint8)
    grad = torch.randn(N, device="cuda", generator=g0)
    hess = torch.rand(N, device="cuda", generator=g0) * 0.25
    rows = torch.randperm(N, device="cuda", generator=g0).int()
    levels = {"root": torch.tensor([0, N], dtype=torch.int32, device="cuda"),
              "32 nodes / 1M rows": torch.linspace(0, N // 2, 33, device="cuda").int()}
    for lname, seg in levels.items():
        for rpb in (1024, 2048, 4096):
            row = []
            for kname, mode in (("slot", 0), ("rows4", 4), ("rows8", 8)):
                ext.set_gbdt_hist_rows(mode)
                for _ in range(3):
                    ext.gbdt_hist_quant(bins, grad, hess, rows, seg, B, rpb)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(20):
                    ext.gbdt_hist_quant(bins, grad, hess, rows, seg, B, rpb)
                e1.record()
                torch.cuda.synchronize()
                row.append(f"{kname} {e0.elapsed_time(e1) * 1e3 / 20:7.1f} us")
            ext.set_gbdt_hist_rows(-2)
            print(f"{lname:20s} rpb {rpb:5d}: " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
