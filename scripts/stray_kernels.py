#!/usr/bin/env python3
"""Non-kdl kernels of one training step, in issue order, with their kdl neighbours.

Splits a rocprofv3 kernel trace into steps at the optimizer kernel and lists,
for the last full step, every kernel that is not a kdl:: kernel together with
the stream it ran on and the nearest kdl kernels before/after it on the same
stream -- enough to say which engine op issued it.

usage: stray_kernels.py <run_kernel_trace.csv>
"""
import collections
import csv
import re
import sys


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    return n[:90]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows)
    opt = [i for i, k in enumerate(ks) if "sgd_chunk" in k[3]]
    lo, hi = opt[-2], opt[-1]
    step = ks[lo + 1: hi + 1]
    by_stream = collections.defaultdict(list)
    for k in step:
        by_stream[k[2]].append(k)
    cnt = collections.Counter()
    tot = collections.Counter()
    print(f"step window: {(ks[hi][1] - ks[lo][1]) / 1e6:.3f} ms, {len(step)} kernels")
    for s, lst in by_stream.items():
        for i, k in enumerate(lst):
            if "kdl::" in k[3]:
                continue
            prev = next((short(x[3]) for x in reversed(lst[:i]) if "kdl::" in x[3]), "-")
            nxt = next((short(x[3]) for x in lst[i + 1:] if "kdl::" in x[3]), "-")
            dur = (k[1] - k[0]) / 1e3
            cnt[short(k[3])] += 1
            tot[short(k[3])] += dur
            print(f"s{s} {dur:7.1f}us {short(k[3])}\n      after {prev}\n      before {nxt}")
    print("\nsummary (count, us):")
    for n, c in cnt.most_common():
        print(f"  {c:3d} {tot[n]:8.1f}  {n}")


if __name__ == "__main__":
    main()
