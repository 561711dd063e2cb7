"""Dump one step of a rocprofv3 kernel trace (between the last two optimizer
kernels): per kernel its duration, the idle gap before it on its stream, the
stream, grid size and short name.  usage: step_dump.py <run_kernel_trace.csv>"""
import csv
import sys


def short(n):
    n = n.replace("kdl::(anonymous namespace)::", "").replace("kdl::gemm::(anonymous namespace)::", "")
    n = n.replace("(anonymous namespace)::", "").replace("unsigned short", "u16")
    return n.split("(")[0][:90]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"],
                 r.get("Grid_Size_X", r.get("Grid_Size", "?"))) for r in rows)
    opt = [k[1] for k in ks if "sgd_chunk" in k[3]]
    lo, hi = opt[-2], opt[-1]
    last_end = {}
    print(f"# step window {(hi - lo) / 1e3:.1f} us; columns: start_us dur_us gap_us stream grid kernel")
    for s, e, st, name, grid in ks:
        if s < lo or e > hi:
            continue
        gap = (s - last_end[st]) / 1e3 if st in last_end else 0.0
        last_end[st] = e
        print(f"{(s - lo) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap:7.1f} {st:>3} {grid:>8} {short(name)}")


if __name__ == "__main__":
    main()
