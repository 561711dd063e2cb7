"""Loader of the host runtime's native module (``csrc/runtime/*.cpp`` ->
``kubedl_amd/_native.so``: fork/exec spawner, reaper, process-group kill,
child subreaper, NUMA best-fit GPU placement).

``KDL_NATIVE_SO=<path>`` loads another build of the same module instead --
``make native-asan`` builds ``build/asan/_native.so`` with
``-fsanitize=address,undefined`` and runs the runtime's process-supervision
paths against it (``tests/test_native_asan.py``, ``scripts/native_stress.py``).
"""
from __future__ import annotations

import importlib.machinery
import importlib.util
import os
import sys

_MOD = None


def load():
    """The native module, or None if it is not built."""
    global _MOD
    if _MOD is not None:
        return _MOD
    path = os.environ.get("KDL_NATIVE_SO")
    if path:
        name = "kubedl_amd._native"
        loader = importlib.machinery.ExtensionFileLoader(name, path)
        spec = importlib.util.spec_from_file_location(name, path, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        sys.modules[name] = mod
        _MOD = mod
        return mod
    try:
        from kubedl_amd import _native
    except ImportError:
        return None
    _MOD = _native
    return _native
