"""In-tree build of the kubedl_amd HIP extension for gfx950.

No hipify, no CUDA sources: ``csrc/*.hip`` are compiled by ``hipcc
--offload-arch=gfx950`` and ``csrc/*.cpp`` (pybind11/torch bindings, native
runtime helpers) as host C++; everything is linked into
``kubedl_amd/_C.so`` next to the package so the ``.so`` travels with the repo
snapshot to the GPU box.  Objects are cached by content hash (source + flags
+ included headers), so a rebuild after a one-file edit recompiles one file.

Usage: ``python -m kubedl_amd.ops.build [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "kdl_ext"
OUT = ROOT / "kubedl_amd" / "_C.so"
ARCH = os.environ.get("KDL_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _common_flags(abi: int):
    return [
        "-O3", "-std=c++17", "-fPIC",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DUSE_ROCM=1",
        "-Wno-unused-result", "-Wno-deprecated-declarations",
    ]


def _headers_digest() -> str:
    h = hashlib.sha256()
    for p in sorted(CSRC.glob("*.h")):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def _compile(src: Path, flags, hdr_digest: str, force: bool, bdir: Path = BUILD) -> Path:
    key = hashlib.sha256(src.read_bytes() + " ".join(flags).encode() + hdr_digest.encode()).hexdigest()[:16]
    obj = bdir / f"{src.stem}.{src.suffix[1:]}.{key}.o"
    if obj.exists() and not force:
        return obj
    for old in bdir.glob(f"{src.stem}.{src.suffix[1:]}.*.o"):
        old.unlink()
    cmd = [HIPCC] + flags + ["-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = True, out: Path | None = None,
          defines: tuple = ()) -> Path:
    """``out`` / ``defines``: an A/B variant of the extension (e.g. ``-DIGEMM_VARIANT=1`` into
    ``kubedl_amd/_C_alt.so``), loaded instead of ``_C.so`` with ``KDL_C_PATH`` (ops/_ext.py)."""
    out = Path(out) if out is not None else OUT
    bdir = BUILD if out == OUT else BUILD / out.stem  # a variant keeps its own objects
    bdir.mkdir(parents=True, exist_ok=True)
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    common = _common_flags(abi) + [f"-D{d}" for d in defines]
    hip_flags = common + [f"--offload-arch={ARCH}", "-x", "hip", f"-I{CSRC}",
                          "-munsafe-fp-atomics"]
    cpp_flags = common + [f"-I{CSRC}", f"-I{py_inc}"] + [f"-I{p}" for p in inc] + [
        "-D__HIP_PLATFORM_AMD__=1", "-DHIPBLAS_V2", "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-DTORCH_EXTENSION_NAME=_C", "-Wno-ignored-attributes"]
    hdr = _headers_digest()
    srcs = sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cpp"))
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = {ex.submit(_compile, s, hip_flags if s.suffix == ".hip" else cpp_flags, hdr, force, bdir): s
                for s in srcs}
        objs = []
        for f in cf.as_completed(futs):
            objs.append(f.result())
            if verbose:
                print(f"[kdl-build] {futs[f].name}", flush=True)
    objs.sort()
    link_key = hashlib.sha256(" ".join(str(o) for o in objs).encode()).hexdigest()[:16]
    stamp = BUILD / ("link.stamp" if out == OUT else f"link.{out.stem}.stamp")
    if out.exists() and stamp.exists() and stamp.read_text() == link_key and not force:
        return out
    tmp = out.with_suffix(".so.tmp")
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(tmp)] + [str(o) for o in objs] + [
        f"-L{lib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
        f"-Wl,-rpath,{lib}", "-Wl,--no-as-needed"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    stamp.write_text(link_key)
    if verbose:
        print(f"[kdl-build] linked {out}", flush=True)
    return out


NATIVE_OUT = ROOT / "kubedl_amd" / "_native.so"


NATIVE_ASAN_OUT = BUILD / "asan" / "_native.so"
SANITIZE_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                  "-fno-sanitize-recover=undefined"]


def build_native(force: bool = False, verbose: bool = True, sanitize: bool = False) -> Path:
    """Host-only C++ runtime module (process supervisor + gang placement core).

    Plain CPython C API, no torch/HIP dependency, so the controller process
    never needs to import torch or touch the GPU.  ``sanitize=True`` builds the
    AddressSanitizer + UBSan variant into build/asan/_native.so (host code only;
    loaded with ``KDL_NATIVE_SO`` under an LD_PRELOADed libasan)."""
    srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    py_inc = sysconfig.get_paths()["include"]
    h = hashlib.sha256()
    for p in srcs:
        h.update(p.read_bytes())
    opt = SANITIZE_FLAGS if sanitize else ["-O2"]
    h.update(" ".join(opt).encode())
    key = h.hexdigest()[:16]
    out = NATIVE_ASAN_OUT if sanitize else NATIVE_OUT
    stamp = BUILD / ("native_asan.stamp" if sanitize else "native.stamp")
    out.parent.mkdir(parents=True, exist_ok=True)
    BUILD.mkdir(parents=True, exist_ok=True)
    if out.exists() and stamp.exists() and stamp.read_text() == key and not force:
        return out
    cxx = os.environ.get("CXX", "g++")
    tmp = out.with_suffix(".so.tmp")
    cmd = [cxx] + opt + ["-std=c++17", "-fPIC", "-shared", "-Wall", f"-I{py_inc}", "-o", str(tmp)] + \
        [str(p) for p in srcs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    stamp.write_text(key)
    if verbose:
        print(f"[kdl-build] linked {out}", flush=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--native-only", action="store_true")
    ap.add_argument("--native-asan", action="store_true", help="only the ASan+UBSan host-runtime variant")
    a = ap.parse_args(argv)
    if a.native_asan:
        build_native(force=a.force, sanitize=True)
        return
    build_native(force=a.force)
    if not a.native_only:
        build(force=a.force, jobs=a.jobs)


if __name__ == "__main__":
    sys.exit(main())
