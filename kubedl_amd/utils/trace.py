"""Tracing (SURVEY.md §5 "Tracing / profiling"): roctx ranges + per-step timing log.

``trace_range(name)`` pushes/pops a roctx range (``librocprofiler-sdk-roctx``),
which ``rocprofv3 --marker-trace`` records next to the kernel trace -- the
train-step phases (forward+backward, all-reduce wait, optimizer) and the
controller's reconcile passes are wrapped in ranges.  With no roctx library, or
``KDL_ROCTX=0``, the ranges are no-ops (the library itself only records when a
profiler is attached).

``StepLog`` appends one JSON line per step to ``KDL_STEP_LOG`` (step, wall ms,
loss, phases) -- the per-step timing record of a rank.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import time
from typing import Optional

_LIB = None
_TRIED = False


def _lib():
    global _LIB, _TRIED
    if _TRIED:
        return _LIB
    _TRIED = True
    if os.environ.get("KDL_ROCTX", "1") == "0":
        return None
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so"):
        for cand in (os.path.join(rocm, "lib", name), name):
            try:
                lib = ctypes.CDLL(cand)
            except OSError:
                continue
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _LIB = lib
            return _LIB
    return None


def available() -> bool:
    return _lib() is not None


@contextlib.contextmanager
def trace_range(name: str):
    lib = _lib()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class StepLog:
    """JSONL per-step record (``KDL_STEP_LOG``); a no-op when unset."""

    def __init__(self, path: Optional[str] = None, rank: int = 0):
        self.path = path if path is not None else os.environ.get("KDL_STEP_LOG")
        self.rank = rank
        self._f = open(self.path, "a", buffering=1) if self.path else None

    @property
    def enabled(self) -> bool:
        return self._f is not None

    def write(self, step: int, ms: float, **kw) -> None:
        if self._f is None:
            return
        rec = {"rank": self.rank, "step": step, "ms": round(ms, 3), "time": time.time()}
        rec.update(kw)
        self._f.write(json.dumps(rec) + "\n")

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None
