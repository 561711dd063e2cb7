"""Helpers shared by every rank-process worker (readiness, progress, faults).

Readiness: the runtime's launch-delay metrics (``kubedl_jobs_first_pod_launch_
delay_seconds`` / ``..._all_pods_...``, reference ``pkg/metrics/job_metrics.go:
53-60``) need a "pod Ready" time.  For a rank process, Ready means the process
is up and its process group is initialised; the worker reports it by writing
``KDL_READY_FILE`` (the supervisor watches that path).

Fault injection: ``KDL_FAULT=<rank>:<step>:<exitcode>`` makes
rank ``rank`` exit with ``exitcode`` when it reaches ``step`` -- used by the
ExitCode-restart / backoff tests.
"""
from __future__ import annotations

import json
import os
import sys
import time


def signal_ready(extra: dict | None = None) -> None:
    path = os.environ.get("KDL_READY_FILE")
    if not path:
        return
    payload = {"ready_time": time.time(), "pid": os.getpid()}
    if extra:
        payload.update(extra)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(payload, f)
    os.replace(tmp, path)


def report_progress(step: int, steps_per_sec: float | None = None, **kw) -> None:
    path = os.environ.get("KDL_PROGRESS_FILE")
    if not path:
        return
    payload = {"step": step, "time": time.time(), "steps_per_sec": steps_per_sec}
    payload.update(kw)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(payload, f)
    os.replace(tmp, path)


def maybe_inject_fault(rank: int, step: int) -> None:
    spec = os.environ.get("KDL_FAULT")
    if not spec:
        return
    try:
        r, s, code = (int(v) for v in spec.split(":"))
    except ValueError:
        return
    if r == rank and s == step:
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(code)
