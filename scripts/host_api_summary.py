#!/usr/bin/env python3
"""Host side of a training step from a rocprofv3 --hip-runtime-trace CSV:
per HIP API function the call count and total time inside the last full
step (bounded by the optimizer kernel's launch calls), and the longest
single calls -- synchronising calls (hipMalloc/hipFree/synchronize/memcpy)
show up here as the reason the GPU idles waiting for the host.

usage: host_api_summary.py <run_hip_api_trace.csv> [steps]
"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    calls = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in rows)
    tot = collections.Counter()
    cnt = collections.Counter()
    span0, span1 = calls[len(calls) // 2][0], calls[-1][1]  # second half of the run (past warm-up)
    longest = []
    for a, b, f in calls:
        if a < span0:
            continue
        tot[f] += b - a
        cnt[f] += 1
        longest.append((b - a, f, a))
    wall = (span1 - span0) / 1e6
    print(f"window {wall:.1f} ms of host time, {sum(cnt.values())} HIP calls")
    for f, t in tot.most_common(15):
        print(f"  {t / 1e6:9.3f} ms  {cnt[f]:6d} x  {f}")
    print("longest calls:")
    for d, f, a in sorted(longest, reverse=True)[:15]:
        print(f"  {d / 1e3:9.1f} us  {f}  at {(a - span0) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
