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


def signal_ready(extra: dict | None = None, wait_warm: bool = True) -> None:
    """Report Ready; then (``wait_warm``) wait for the node warm-up's lock
    (parallel/dist.py ``wait_node_warm``) before the caller's first
    collective -- AFTER Ready, so the launch delay never includes it.  Callers
    that overlap the wait with other start-up work pass False and wait at
    their first collective instead (dist.first_collective, FlatDDP)."""
    path = os.environ.get("KDL_READY_FILE")
    if path:
        payload = {"ready_time": time.time(), "pid": os.getpid()}
        if extra:
            payload.update(extra)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(payload, f)
        os.replace(tmp, path)
    if wait_warm and os.environ.get("KDL_NODE_WARM_LOCK"):
        from kubedl_amd.parallel.dist import wait_node_warm
        wait_node_warm()


_PROGRESS_LAST = [0.0]  # monotonic time of the last progress write


def report_progress(step: int, steps_per_sec: float | None = None, final: bool = False, **kw) -> None:
    """Write the step counter for the kubelet (``KDL_PROGRESS_FILE``).  Writes are
    throttled to one per ``KDL_TUNE progress_min_s`` seconds (default 0.2): a file
    write + rename costs tens of us of host time, ~10 % of a 0.47 ms CTR step
    when done every step.  The first call and ``final=True`` always write."""
    path = os.environ.get("KDL_PROGRESS_FILE")
    if not path:
        return
    now = time.monotonic()
    from kubedl_amd.utils.tune import tune
    min_s = tune("progress_min_s", 0.2)
    if not final and _PROGRESS_LAST[0] and now - _PROGRESS_LAST[0] < min_s:
        return
    _PROGRESS_LAST[0] = now
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


def free_port() -> int:
    """An unused 127.0.0.1 TCP port (a one-rank process group's rendezvous)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
