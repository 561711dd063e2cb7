"""Per-launch view of the main stream's LDS-DMA GEMMs (igemm) in a kernel trace of the
ResNet-50 step: duration, grid, and how much of it ran beside side-stream kernels.

usage: igemm_contention.py <run_kernel_trace.csv> [--steps 4]
Prints one line per igemm launch of the last ``steps`` steps (grouped by kernel + grid),
mean duration and the mean fraction of its time that some side-stream kernel overlapped.
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"] if "Stream_Id" in r else r["Queue_Id"],
           int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))) for r in rows]
    ks.sort()
    opt = [k for k in ks if "sgd" in k[2].lower()]
    if len(opt) > a.steps:
        t0 = opt[-a.steps - 1][1]
        ks = [k for k in ks if k[0] >= t0]
    streams = collections.Counter(k[3] for k in ks if "igemm" in k[2])
    main_s = streams.most_common(1)[0][0]
    side = [k for k in ks if k[3] != main_s]
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for s, e, name, st, grid in ks:
        if st != main_s or "igemm" not in name:
            continue
        ov = 0
        for s2, e2, *_ in side:
            lo, hi = max(s, s2), min(e, e2)
            if hi > lo:
                ov += hi - lo
        key = (re.sub(r"\(kdl::gemm::GemmParams.*", "", name).replace("void kdl::(anonymous namespace)::", ""), grid)
        g = agg[key]
        g[0] += 1
        g[1] += (e - s) / 1e3
        g[2] += min(1.0, ov / max(1, e - s))
    tot = 0.0
    for (name, grid), (n, us, ov) in sorted(agg.items(), key=lambda x: -x[1][1]):
        tot += us
        print(f"{name:55s} grid {grid:5d} x{n // a.steps:2d}/step  {us / n:7.1f} us  side-overlap {100 * ov / n:5.1f}%")
    print(f"total {tot / a.steps / 1e3:.3f} ms/step")


if __name__ == "__main__":
    main()
