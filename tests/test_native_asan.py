"""The native host runtime (csrc/runtime/spawn.cpp, gpu_alloc.cpp) under
AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 race detection /
sanitizers).

Builds build/kdl_ext/asan/_native.so with -fsanitize=address,undefined and
runs scripts/native_stress.py against it in a child interpreter with libasan
preloaded: fork/exec (incl. exec failure), status pipes, reaping, process
group kills, the child subreaper, the NUMA best-fit placement, and the whole
control plane driving plain-python ranks through success, permanent failure,
OnFailure, a gang restart and a deletion.  Any sanitizer report fails it.
Host code only (no GPU sanitizers on this pool)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _libasan():
    if shutil.which(os.environ.get("CXX", "g++")) is None:
        return None
    r = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True)
    path = r.stdout.strip()
    return path if r.returncode == 0 and os.path.isabs(path) and os.path.exists(path) else None


def test_native_runtime_under_asan_ubsan():
    lib = _libasan()
    if lib is None:
        pytest.skip("no g++/libasan on this host")
    from kubedl_amd.ops.build import build_native
    so = build_native(sanitize=True, verbose=False)
    env = dict(os.environ)
    env.update(KDL_NATIVE_SO=str(so), KDL_ZYGOTE="0",
               LD_PRELOAD=lib + ((":" + env["LD_PRELOAD"]) if env.get("LD_PRELOAD") else ""),
               ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "native_stress.py")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert r.returncode == 0 and "native stress ok" in r.stdout, out[-4000:]
    assert "asan" in r.stdout  # the sanitizer build was the one loaded
