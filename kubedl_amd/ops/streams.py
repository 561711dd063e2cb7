"""Stream selection for the training step.

Measured on MI355X (``profiles/r02_world1_pg_streams_ab.txt``): once an RCCL
process group exists, a ResNet-50 step issued on the device's NULL stream
loses its weight-gradient side-stream overlap (11.3k -> 10.4k img/s at batch
256; without a process group the same step runs 11.3k).  Issuing the step on
an ordinary non-blocking pool stream instead (``torch.cuda.Stream``) keeps the
full rate with the process group present: the legacy null stream is
implicitly ordered against the other blocking streams of the process, and
RCCL creates some.  So the trainer runs every step on a stream of its own and
the engine's side stream is a second pool stream.

``KDL_TUNE streams=`` selects the variant (A/B switch):

* ``pool`` (default): pool streams (``torch.cuda.Stream``);
* ``dedicated``: streams with an explicit full CU mask, which HIP always
  places on a hardware queue of their own (csrc/streams.hip).  Measured
  slower for this step (10.2k img/s): kept for experiments only;
* ``null``: the step runs on the caller's (null) stream, as before.
"""
from __future__ import annotations

import os
import time
from typing import Optional

import torch

_KEEP = []  # handles of dedicated streams (ExternalStream does not own them)


def mode() -> str:
    from kubedl_amd.utils.tune import tune
    return tune("streams", "pool")


def compute_stream(device: torch.device) -> Optional[torch.cuda.Stream]:
    """The stream a training step runs on (None = the caller's stream)."""
    m = mode()
    if device.type != "cuda" or m == "null":
        return None
    # the step's stream at high priority (KDL_TUNE main_prio, default -1): the
    # dispatcher hands CUs to its critical-path kernels before the
    # weight-gradient side stream's (torch: lower number = higher priority);
    # measured 12,574-12,661 -> 12,740-12,751 img/s (profiles/r02_stream_priority_ab.txt)
    from kubedl_amd.utils.tune import tune
    return side_stream(device, tune("main_prio", -1))


def side_stream(device: torch.device, priority: int = 0) -> torch.cuda.Stream:
    # (a CU-masked side stream -- any mask, even all 256 CUs -- runs the ResNet-50
    # step at ~9.7k img/s vs 13.6k: profiles/r04_side_stream_cu_mask_ab.txt)
    if mode() == "dedicated":
        return dedicated_stream(device, priority)
    return torch.cuda.Stream(device=device, priority=priority)


def dedicated_stream(device: torch.device, priority: int = 0, cus: int = 0) -> torch.cuda.Stream:
    """A stream on a hardware queue of its own (a full CU mask, or ``cus`` CUs)."""
    if device.type != "cuda":
        raise ValueError("dedicated_stream needs a GPU device")
    from kubedl_amd.ops import _ext
    ext = _ext.load()
    with torch.cuda.device(device):
        h = ext.make_stream(True, priority, cus)
    _KEEP.append(h)
    return torch.cuda.ExternalStream(h, device=device)


def overlap_ratio(a: torch.cuda.Stream, b: torch.cuda.Stream, us: float = 3000.0) -> float:
    """Wall time of one ``us``-long spin kernel on each of ``a`` and ``b``,
    launched back to back, over ``us``: ~1 when the streams run concurrently,
    ~2 when they serialise (diagnostic, scripts/probe_queues.py)."""
    from kubedl_amd.ops import _ext
    ext = _ext.load()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(a):
        ext.spin(us)
    with torch.cuda.stream(b):
        ext.spin(us)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6 / us
