"""Python side of the single A/B-knob variable ``KDL_TUNE`` (csrc/tune.h).

``KDL_TUNE="main_prio=-1,ddp_world1=copy,p2p_timeout_s=60"`` -- the same
comma-separated ``key=value`` list the native kernels read, so every
experiment switch lives in one variable (``KDL_ENGINE`` holds the ResNet
engine's schedule options).  Python keys (defaults are the measured winners,
docs/perf_notes.md):

==================  ==========  ================================================
key                 default     meaning
==================  ==========  ================================================
streams             pool        step streams: pool | dedicated | null (ops/streams.py)
main_prio           -1          HIP priority of the step's compute stream
loss_allreduce      1           sum the step loss over ranks (RCCL) every step
comm_probe          1           time the first collective (RCCL bootstrap) apart
comm_overlap        1           run that bootstrap on a helper thread during the model build
comm_defer_w1       1           world 1: build the communicator after the first step instead
world1_pg           1           build a one-rank process group at world 1
pg_eager            0           bind the RCCL communicator at init_process_group
ddp_world1          0           world-1 DDP rehearsal: 0 | 1 | copy (parallel/ddp.py)
ddp_reduce          bf16        bucket all-reduce dtype: bf16 | fp32
p2p_oneshot_bytes   262144      P2P all-reduce one-shot threshold (parallel/p2p.py)
p2p_timeout_s       300         P2P all-reduce bounded-wait timeout
progress_min_s      0.2         seconds between rank progress-file writes
ctr_a2a_slack       0           CTR exchange capacity = slack x recent fill (0: exact)
ctr_a2a_strict      1           raise on a CTR exchange overflow (0: lossy, counted)
ctr_fused_relu_bwd  1           CTR tower: ReLU backward + bias grads inside the producing launches
==================  ==========  ================================================
"""
from __future__ import annotations

import os
from typing import Callable, Optional, TypeVar

T = TypeVar("T")


# stand-alone variables of earlier rounds, now KDL_TUNE keys: setting one does
# nothing, so it is reported once instead of silently ignored
RETIRED_ENV = {
    "KDL_STREAMS": "streams", "KDL_MAIN_PRIO": "main_prio", "KDL_DDP_WORLD1": "ddp_world1",
    "KDL_DDP_REDUCE": "ddp_reduce", "KDL_P2P_TIMEOUT_S": "p2p_timeout_s",
    "KDL_P2P_ONESHOT_BYTES": "p2p_oneshot_bytes", "KDL_PG_EAGER": "pg_eager",
    "KDL_PROGRESS_MIN_S": "progress_min_s", "KDL_CTR_A2A_SLACK": "ctr_a2a_slack",
    "KDL_CTR_A2A_STRICT": "ctr_a2a_strict", "KDL_WORLD1_PG": "world1_pg",
    "KDL_LOSS_ALLREDUCE": "loss_allreduce", "KDL_COMM_PROBE": "comm_probe",
    "KDL_COMM_OVERLAP": "comm_overlap",
}
_WARNED = [False]


def warn_retired_env(stream=None) -> list:
    """Print one line per retired ``KDL_*`` variable set in the environment,
    naming the KDL_TUNE key that replaced it (once per process)."""
    import sys
    found = [k for k in RETIRED_ENV if k in os.environ]
    if found and not _WARNED[0]:
        _WARNED[0] = True
        for k in found:
            print(f"[kdl] warning: {k} is retired and ignored; use KDL_TUNE=\"{RETIRED_ENV[k]}="
                  f"{os.environ[k]}\"", file=stream or sys.stderr, flush=True)
    return found


def tune_find(name: str) -> Optional[str]:
    """The raw value of ``name`` in KDL_TUNE, or None when the key is absent."""
    spec = os.environ.get("KDL_TUNE", "")
    for item in spec.split(","):
        key, sep, val = item.strip().partition("=")
        if sep and key == name:
            return val.strip()
    return None


def tune(name: str, default: T, cast: Optional[Callable[[str], T]] = None) -> T:
    """``name``'s value in KDL_TUNE cast like ``default`` (or by ``cast``)."""
    v = tune_find(name)
    if v is None:
        return default
    if cast is not None:
        return cast(v)
    if isinstance(default, bool):
        return v.lower() in ("1", "true", "on", "yes")
    if isinstance(default, int):
        return int(v)
    if isinstance(default, float):
        return float(v)
    return type(default)(v) if default is not None else v  # type: ignore[return-value]
