#!/usr/bin/env python3
"""Idle gaps of the main (critical-path) stream in the last full step of a
rocprofv3 kernel trace, with the kernels on both sides and what the other
streams ran meanwhile -- where the GPU waits for the host (launch issue) or
for a cross-stream event.

usage: main_gaps.py <run_kernel_trace.csv> [min_gap_us]
"""
import csv
import sys


def nm(n):
    n = n.replace("void ", "").replace("kdl::(anonymous namespace)::", "").replace("kdl::gemm::(anonymous namespace)::", "")
    return (n[:n.index("(")] if "(" in n else n)[:60]


def main():
    path = sys.argv[1]
    lim = float(sys.argv[2]) if len(sys.argv) > 2 else 15.0
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows)
    opt = [i for i, k in enumerate(ks) if "sgd_chunk" in k[3]]
    lo, hi = opt[-2], opt[-1]
    step = ks[lo:hi + 1]
    main_s = step[0][2]
    main = [k for k in step if k[2] == main_s]
    other = [k for k in step if k[2] != main_s]
    t0 = step[0][0]
    tot = big = 0.0
    out = []
    for a, b in zip(main, main[1:]):
        g = (b[0] - a[1]) / 1e3
        if g <= 0:
            continue
        tot += g
        if g >= lim:
            big += g
            ov = sorted({nm(s[3]) for s in other if s[0] < b[0] and s[1] > a[1]})
            out.append(f"{g:7.1f} us at {(a[1] - t0) / 1e3:8.1f} us  {nm(a[3])} -> {nm(b[3])}  other streams: {ov[:3]}")
    print(f"step {(step[-1][1] - step[0][1]) / 1e3:.1f} us; main-stream gaps {tot:.1f} us in total, "
          f"{big:.1f} us in {len(out)} gaps >= {lim} us")
    print("\n".join(out))


if __name__ == "__main__":
    main()
