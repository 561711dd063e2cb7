"""Per-kernel (name, grid) breakdown of the MAIN stream of a rocprofv3 kernel
trace of the ResNet-50 bench, averaged over the last N steps (steps split at
the optimizer kernel).  usage: main_stream_breakdown.py <run_kernel_trace.csv> [N] [top]"""
import collections
import csv
import sys


def short(name):
    for p in ("void ", "kdl::(anonymous namespace)::", "kdl::gemm::(anonymous namespace)::", "kdl::"):
        name = name.replace(p, "")
    return name.split("(")[0]


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"],
                   int(r["Grid_Size_X"])) for r in csv.DictReader(open(path)))
    opt = [r for r in rows if "sgd_chunk" in r[3]]
    lo, hi = opt[-n - 1], opt[-1]
    step = [r for r in rows if lo[1] <= r[0] and r[1] <= hi[1]]
    busy = collections.Counter()
    for r in step:
        busy[r[2]] += r[1] - r[0]
    main_s = busy.most_common(1)[0][0]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in step:
        if r[2] == main_s:
            a = agg[(short(r[3]), r[4])]
            a[0] += 1
            a[1] += (r[1] - r[0]) / 1e3
    print(f"main stream {main_s}: busy {sum(v[1] for v in agg.values()) / n:.1f} us/step over {n} steps")
    for (name, grid), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{t / n:8.1f} us/step {c // n:3d}/step {t / c:7.1f} us/call grid {grid:>7}  {name[:90]}")


if __name__ == "__main__":
    main()
