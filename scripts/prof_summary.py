#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace into per-step ms by kernel family.

usage: prof_summary.py <run_kernel_stats.csv | run_results.db> [steps]
(the .db is rocprofv3's default rocpd output; the csv needs --output-format csv)
"""
import csv
import re
import sqlite3
import sys

FAMILIES = [
    ("conv-gemm(kdl)", r"kdl::.*(gemm1x1|wgrad1x1|igemm)"),
    ("bn(kdl)", r"kdl::.*bn_"),
    ("optim(kdl)", r"kdl::.*(sgd|adam|sumsq|cast)"),
    ("kdl-other", r"kdl::"),
    ("conv-fwd(miopen)", r"igemm_fwd|conv_fwd|ConvFwd|naive_conv_.*fwd|grouped_conv_fwd"),
    ("conv-bwd-data(miopen)", r"igemm_bwd|conv_bwd_data|grouped_conv_bwd_data"),
    ("conv-bwd-wgt(miopen)", r"igemm_wrw|bwd_weight|grouped_conv_bwd_weight"),
    ("miopen-tensorop", r"SubTensorOp|Op2dTensor|Op1dTensor|transpose|MIOpen"),
    ("gemm(blas)", r"Cijk_|gemm|Gemm"),
    ("elementwise(torch)", r"elementwise|CUDAFunctor|reduce_kernel|fill|copy"),
    ("pool(torch)", r"pool"),
    ("softmax/loss(torch)", r"softmax|nll|cross"),
    ("rccl", r"nccl|rccl"),
]


def family(name):
    for fam, pat in FAMILIES:
        if re.search(pat, name):
            return fam
    return "other"


def load(path):
    """(name, calls, total ns) per kernel name."""
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        q = "select name, count(*), sum(end - start) from kernels group by name"
        return [(n, int(k), float(t)) for n, k, t in con.execute(q)]
    with open(path) as f:
        return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(f)]


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    fam_ns, fam_calls, rows = {}, {}, []
    for name, calls, ns in load(path):
        fam = family(name)
        fam_ns[fam] = fam_ns.get(fam, 0.0) + ns
        fam_calls[fam] = fam_calls.get(fam, 0) + calls
        rows.append((ns, calls, name[:110]))
    tot = sum(fam_ns.values())
    print(f"total GPU kernel time per step: {tot / steps / 1e6:.3f} ms  (steps={steps:g})")
    print(f"{'family':28s} {'ms/step':>9s} {'%':>6s} {'launches/step':>14s}")
    for fam, ns in sorted(fam_ns.items(), key=lambda kv: -kv[1]):
        print(f"{fam:28s} {ns / steps / 1e6:9.3f} {100 * ns / tot:6.1f} {fam_calls[fam] / steps:14.1f}")
    print("\ntop kernels:")
    for ns, calls, name in sorted(rows, reverse=True)[:25]:
        print(f"{ns / steps / 1e6:8.3f} ms/step {calls / steps:7.1f}/step  {name}")


if __name__ == "__main__":
    main()
