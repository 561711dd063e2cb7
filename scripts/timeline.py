"""Critical-path view of a rocprofv3 kernel trace of the ResNet-50 bench.

Splits the trace into steps at the optimizer kernel, then for the last steps
reports per stream the busy time, the wall time of the step, the time no
kernel runs at all (launch gaps / host stalls), and the time only the side
stream runs (the tail the main stream waits for).

usage: timeline.py <run_kernel_trace.csv> [--steps 4]
"""
import argparse
import collections
import csv


def fam(name):
    n = name.lower()
    for key, f in (("wgrad_reduce", "wgrad_reduce"), ("wgrad", "wgrad"), ("halo3x3", "halo3x3"), ("igemm", "igemm"),
                   ("gemm1x1", "gemm1x1"), ("finalize", "bn_finalize"), ("bn_", "bn"), ("miopen", "miopen"),
                   ("sgd", "optim"), ("wt_batch", "transpose")):
        if key in n:
            return f
    if "igemm" in n or "naive_conv" in n or "conv" in n:
        return "miopen"
    return "other"


def union(iv):
    iv = sorted(iv)
    tot, cur = 0, None
    for a, b in iv:
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        tot += cur[1] - cur[0]
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows))
    opt = [k[1] for k in ks if "sgd_chunk" in k[3]]
    bounds = opt[-a.steps - 1:]
    per = collections.defaultdict(float)
    famt = collections.defaultdict(lambda: collections.defaultdict(float))
    wall = idle = side_only = 0.0
    for lo, hi in zip(bounds, bounds[1:]):
        win = [k for k in ks if k[0] >= lo and k[1] <= hi]
        wall += hi - lo
        streams = collections.Counter(k[2] for k in win)
        main = streams.most_common(1)[0][0]
        iv_all = [(k[0], k[1]) for k in win]
        iv_main = [(k[0], k[1]) for k in win if k[2] == main]
        idle += (hi - lo) - union(iv_all)
        side_only += union(iv_all) - union(iv_main)
        for k in win:
            per["main" if k[2] == main else "side" + k[2]] += k[1] - k[0]
            famt["main" if k[2] == main else "side"][fam(k[3])] += k[1] - k[0]
    n = len(bounds) - 1
    ms = lambda v: round(v / n / 1e6, 3)
    print(f"steps {n}: wall {ms(wall)} ms/step, no kernel running {ms(idle)}, only side streams running {ms(side_only)}")
    for s, v in sorted(per.items()):
        print(f"  busy {s}: {ms(v)} ms/step")
    for s, d in famt.items():
        print(f"  {s}: " + ", ".join(f"{f} {ms(v)}" for f, v in sorted(d.items(), key=lambda x: -x[1])))


if __name__ == "__main__":
    main()
