"""Per-kernel roofline table from rocprofv3 --pmc passes (scripts/gpu_r04_pmc.sh).

Each pass directory holds ``run_counter_collection.csv`` (one row per dispatch
and counter).  Dispatches are serialised under --pmc, so Start/End timestamps
give an uncontended kernel time.  Per kernel (grouped by name with template
arguments, summed over its dispatches):

  us      mean kernel time per dispatch (pass P1's timestamps)
  GB/s    HBM-side traffic: (2*FETCH_SIZE + WRITE_SIZE) KB / time.  FETCH_SIZE
          reads 1/2 of a wide coalesced read's bytes on gfx950
          (MI355X_MICROARCH.md "HBM"), so it is doubled; writes are exact
  %HBM    GB/s against 6300 GB/s achievable
  TF/s    bf16 MFMA rate: SQ_VALU_MFMA_BUSY_CYCLES counts 32 cycles per
          32x32x16 bf16 MFMA (32768 flop) per SIMD, i.e. 1024 flop per busy
          cycle
  %MFMA   TF/s against 2500 TF/s dense bf16
  bound   the larger of %HBM and %MFMA names the roof the kernel is nearer
  LDSconf SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS (both quad-cycle units)
  L2hit   TCC_HIT / (TCC_HIT + TCC_MISS)

Usage: python scripts/pmc_summary.py gpurun_out/pmc4 [--top 30] [--kdl]
"""
import argparse
import collections
import csv
import os
import re
import sys

csv.field_size_limit(1 << 30)


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            name = name[:i]
            break
    name = name.replace("void ", "").strip()
    return name[:110]


def load(path):
    """dispatch id -> (name, start, end, {counter: value})"""
    out = {}
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            d = int(r["Dispatch_Id"])
            e = out.get(d)
            if e is None:
                e = out[d] = [short(r["Kernel_Name"]), int(r["Start_Timestamp"]),
                              int(r["End_Timestamp"]), {}]
            e[3][r["Counter_Name"]] = e[3].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--kdl", action="store_true", help="only kdl:: kernels")
    ap.add_argument("--steps", type=int, default=0, help="steps in the run: print per-step GB and TFLOP totals")
    a = ap.parse_args()
    passes = {}
    for p in ("P1", "P2", "P3"):
        fp = os.path.join(a.root, p, "run_counter_collection.csv")
        if os.path.exists(fp):
            passes[p] = load(fp)
    if "P1" not in passes:
        print("no P1 pass", file=sys.stderr)
        return 1
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for p, disp in passes.items():
        for name, t0, t1, cs in disp.values():
            g = agg[name]
            if p == "P1":
                g["n"] += 1
                g["ns"] += t1 - t0
            for c, v in cs.items():
                g[c] += v
    rows = []
    for name, g in agg.items():
        if a.kdl and "kdl::" not in name:
            continue
        if g["n"] == 0 or g["ns"] <= 0:
            continue
        s = g["ns"] * 1e-9
        hbm = (2 * g.get("FETCH_SIZE", 0) + g.get("WRITE_SIZE", 0)) * 1024
        gbs = hbm / s / 1e9
        tfs = g.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) * 1024 / s / 1e12
        lds = g.get("SQ_ACTIVE_INST_LDS", 0)
        hit, miss = g.get("TCC_HIT_sum", 0), g.get("TCC_MISS_sum", 0)
        rows.append(dict(
            rd=2 * g.get("FETCH_SIZE", 0) * 1024, wr=g.get("WRITE_SIZE", 0) * 1024,
            flop=g.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) * 1024,
            name=name, n=int(g["n"]), us=g["ns"] / g["n"] / 1e3, tot_ms=g["ns"] / 1e6,
            gbs=gbs, hbm=100 * gbs / 6300, tfs=tfs, mfma=100 * tfs / 2500,
            ldsc=(100 * g.get("SQ_LDS_BANK_CONFLICT", 0) / lds) if lds else 0.0,
            l2=(100 * hit / (hit + miss)) if hit + miss else 0.0))
    rows.sort(key=lambda r: -r["tot_ms"])
    tot = sum(r["tot_ms"] for r in rows)
    print(f"{'kernel':<90} {'n':>5} {'us':>8} {'%time':>6} {'GB/s':>6} {'%HBM':>5} "
          f"{'TF/s':>6} {'%MFMA':>5} {'bound':>5} {'LDSc%':>5} {'L2hit':>5}")
    for r in rows[:a.top]:
        bound = "HBM" if r["hbm"] >= r["mfma"] else "MFMA"
        print(f"{r['name'][:90]:<90} {r['n']:>5} {r['us']:>8.1f} {100*r['tot_ms']/tot:>6.2f} "
              f"{r['gbs']:>6.0f} {r['hbm']:>5.1f} {r['tfs']:>6.0f} {r['mfma']:>5.1f} "
              f"{bound:>5} {r['ldsc']:>5.1f} {r['l2']:>5.1f}")
    print(f"total serialised kernel time {tot:.1f} ms over {sum(r['n'] for r in rows)} dispatches")
    if a.steps:
        rd, wr, fl = (sum(r[k] for r in rows) / a.steps for k in ("rd", "wr", "flop"))
        print(f"per step ({a.steps} steps): read {rd / 1e9:.2f} GB + write {wr / 1e9:.2f} GB = {(rd + wr) / 1e9:.1f} GB; "
              f"MFMA work {fl / 1e12:.3f} TFLOP")
    return 0


if __name__ == "__main__":
    sys.exit(main())
