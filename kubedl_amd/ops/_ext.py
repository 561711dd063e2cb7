"""Loader for the in-tree HIP extension ``kubedl_amd._C``.

Policy: on a machine with a GPU the HIP kernels are the ONLY path for the ops
they implement -- if the extension is missing we fail loudly instead of
silently falling back to eager PyTorch (set ``KDL_ALLOW_TORCH_FALLBACK=1`` to
opt out, e.g. for A/B benchmarking).  On CPU-only hosts the PyTorch
compositions are the implementation (and the numerics reference).
"""
from __future__ import annotations

import importlib
import os

_mod = None
_err: Exception | None = None


def load():
    global _mod, _err
    if _mod is not None:
        return _mod
    try:
        alt = os.environ.get("KDL_C_PATH")
        if alt:  # an A/B build of the same module (ops/build.py ``out`` / ``defines``)
            import sys
            from importlib import machinery, util
            loader = machinery.ExtensionFileLoader("kubedl_amd._C", alt)
            spec = util.spec_from_file_location("kubedl_amd._C", alt, loader=loader)
            mod = util.module_from_spec(spec)
            loader.exec_module(mod)
            sys.modules["kubedl_amd._C"] = mod
            _mod = mod
            return _mod
        _mod = importlib.import_module("kubedl_amd._C")
        return _mod
    except Exception as e:  # pragma: no cover - depends on build state
        _err = e
        raise RuntimeError(
            "kubedl_amd HIP extension is not built: run `python -m kubedl_amd.ops.build` "
            f"(import error: {e})") from e


def available() -> bool:
    try:
        load()
        return True
    except RuntimeError:
        return False


def require_on_gpu(op: str) -> None:
    if os.environ.get("KDL_ALLOW_TORCH_FALLBACK") == "1":
        return
    raise RuntimeError(f"{op}: GPU tensor but the kubedl_amd HIP extension is unavailable ({_err}); "
                       "build it with `python -m kubedl_amd.ops.build`")
