"""Sum rocprofv3 --pmc counters per kernel over pass directories (one table row per kernel).

usage: pmc_quick.py DIR [DIR ...]   (each DIR holds run_counter_collection.csv)
Counters from several passes of the same program are merged by kernel name; the
derived columns: MFMA busy % of SQ_BUSY_CYCLES x 4 SIMDs, waits as % of wave cycles.
"""
import collections
import csv
import re
import sys

csv.field_size_limit(1 << 30)


def short(name):
    name = re.sub(r"kdl::\(anonymous namespace\)::", "", name)
    return name[:110]


def main(dirs):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in dirs:
        with open(f"{d}/run_counter_collection.csv") as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((d, r["Dispatch_Id"]))
    for k, c in tot.items():
        if "igemm" not in k and "gemm" not in k and len(sys.argv) < 3:
            pass
        n = max(1, len({x[1] for x in disp[k]}))
        out = {kk: v / n for kk, v in sorted(c.items())}
        wc = out.get("SQ_WAVE_CYCLES", 0)
        line = [k, f"dispatches={n}"]
        if wc:
            for w in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if w in out:
                    line.append(f"{w[3:]}={100 * out[w] / wc:.1f}%")
        if "SQ_LDS_BANK_CONFLICT" in out and "SQ_ACTIVE_INST_LDS" in out and out["SQ_ACTIVE_INST_LDS"]:
            line.append(f"LDSconf/LDSactive={out['SQ_LDS_BANK_CONFLICT'] / out['SQ_ACTIVE_INST_LDS']:.2f}")
        print("  ".join(line))
        print("    " + "  ".join(f"{kk}={v:.4g}" for kk, v in out.items()))


if __name__ == "__main__":
    main(sys.argv[1:])
