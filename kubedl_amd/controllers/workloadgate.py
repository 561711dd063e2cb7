"""Workload gate: which workload controllers to start.

Reference ``pkg/util/workloadgate/workload_gate.go``:

* flag ``--workloads`` (default ``auto``) or env ``WORKLOADS_ENABLE``;
* syntax: comma list, ``*`` enables all, ``-Kind`` marks a kind disabled;
* ``auto`` = enable the kind if its CRD is installed (discovery client; the
  local runtime has every CRD built in, so ``auto`` enables all -- the same
  answer the reference gives with ``KUBEDL_CI=true``).

Quirks kept: the gate checks *presence* in the parsed map,
not the value, so ``-Kind`` ENABLES Kind; and ``WORKLOADS_ENABLE`` is only
consulted when the flag is not ``auto`` (the flag's ``auto`` returns first).
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Optional, Tuple

ENV_WORKLOAD_ENABLE = "WORKLOADS_ENABLE"
AUTO = "auto"


def parse_workloads_enabled(workloads: str) -> Tuple[Dict[str, bool], bool]:
    enable_all = False
    enables: Dict[str, bool] = {}
    for w in workloads.split(","):
        w = w.strip()
        enable = True
        if w.startswith("-"):
            enable = False
            w = w[1:]
        if w == "*":
            if enable:
                enable_all = True
            continue
        if w == "":
            continue
        enables[w] = enable
    return enables, enable_all


def is_workload_enable(kind: str, workloads: Optional[str] = AUTO,
                       crd_installed: Optional[Callable[[str], bool]] = None,
                       env: Optional[dict] = None) -> bool:
    env = os.environ if env is None else env
    installed = crd_installed or (lambda k: True)
    enables: Dict[str, bool] = {}
    enable_all = False
    if workloads is not None:
        if workloads == AUTO:
            return installed(kind)
        enables, enable_all = parse_workloads_enabled(workloads)
    env_w = env.get(ENV_WORKLOAD_ENABLE, "")
    if env_w:
        if env_w == AUTO:
            return installed(kind)
        enables, enable_all = parse_workloads_enabled(env_w)
    if enable_all:
        return True
    return kind in enables
