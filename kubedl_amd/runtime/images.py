"""Local "image registry": what a container image means on a single node.

Kubernetes pulls an image and runs its entrypoint; the local runtime has no
images.  A container therefore runs

1. its own ``command`` (+ ``args``) when the command can be executed here; or
2. the entrypoint registered for its image below (``args`` appended), which
   is how the reference's example YAMLs (``kubedl/pytorch-dist-example``,
   ``kubedl/tf-mnist-with-summaries``, ``merlintang/xgboost-dist-iris``,
   ``kubedl/xdl``...) run unchanged: each maps to the bundled MI355X worker
   for that framework.

``readiness`` says how the runtime decides "pod Ready" for the launch-delay
metrics: ``file`` = the worker writes ``$KDL_READY_FILE`` once its process
group is up (bundled workers); ``start`` = ready when the process starts
(arbitrary commands, like a pod without a readiness probe).
"""
from __future__ import annotations

import os
import shutil
import sys
from dataclasses import dataclass
from typing import Dict, List, Optional


@dataclass(frozen=True)
class ImageEntry:
    entrypoint: List[str]
    readiness: str = "file"


def _py(mod: str) -> List[str]:
    return [sys.executable, "-u", "-m", mod]


# image name (without tag/registry) -> bundled worker
REGISTRY: Dict[str, ImageEntry] = {
    # reference examples
    "kubedl/pytorch-dist-example": ImageEntry(_py("kubedl_amd.workers.pytorch_dist")),
    "kubedl/tf-mnist-with-summaries": ImageEntry(_py("kubedl_amd.workers.tf_stub")),
    "merlintang/xgboost-dist-iris": ImageEntry(_py("kubedl_amd.workers.xgboost_dist")),
    "kubedl/xdl": ImageEntry(_py("kubedl_amd.workers.xdl_ctr")),
    "kubedl/xdl-mnist-example": ImageEntry(_py("kubedl_amd.workers.xdl_ctr")),
    "xdl": ImageEntry(_py("kubedl_amd.workers.xdl_ctr")),
    "kubedl/git-sync": ImageEntry(_py("kubedl_amd.code_sync.git_sync"), readiness="start"),
    # bundled MI355X workloads
    "kubedl-amd/resnet50": ImageEntry(_py("kubedl_amd.workers.resnet50")),
    "kubedl-amd/pytorch-dist": ImageEntry(_py("kubedl_amd.workers.pytorch_dist")),
    "kubedl-amd/gbdt": ImageEntry(_py("kubedl_amd.workers.xgboost_dist")),
    "kubedl-amd/xdl-ctr": ImageEntry(_py("kubedl_amd.workers.xdl_ctr")),
    "kubedl-amd/tf-stub": ImageEntry(_py("kubedl_amd.workers.tf_stub")),
    "kubedl-amd/sleep": ImageEntry([sys.executable, "-c", "import sys,time; time.sleep(float(sys.argv[1]) if len(sys.argv)>1 else 3600)"], readiness="start"),
}


def image_name(image: str) -> str:
    """Strip registry host, tag and digest: ``docker.io/merlintang/xgboost-dist-iris:1.1``
    -> ``merlintang/xgboost-dist-iris``."""
    img = (image or "").split("@", 1)[0]
    last = img.rsplit("/", 1)[-1]
    if ":" in last:
        img = img[: len(img) - len(last)] + last.split(":", 1)[0]
    parts = img.split("/")
    if len(parts) > 2 or (len(parts) == 2 and ("." in parts[0] or ":" in parts[0])):
        if "." in parts[0] or ":" in parts[0] or parts[0] == "localhost":
            parts = parts[1:]
    return "/".join(parts)


def lookup(image: str) -> Optional[ImageEntry]:
    return REGISTRY.get(image_name(image))


def _runnable(cmd0: str, cwd: Optional[str], path: str) -> bool:
    if os.path.isabs(cmd0):
        return os.access(cmd0, os.X_OK)
    if "/" in cmd0:
        return os.access(os.path.join(cwd or ".", cmd0), os.X_OK)
    return shutil.which(cmd0, path=path) is not None


def _script_exists(argv: List[str], cwd: Optional[str]) -> bool:
    """``python /var/tf_mnist/x.py``: the interpreter exists but its script may
    not.  Shell wrappers (``bash -c "exec python mnist.py ..."``, the XDL
    example) are looked through: the check applies to the wrapped command."""
    if len(argv) >= 3 and os.path.basename(argv[0]) in ("bash", "sh") and argv[1] == "-c":
        import shlex
        try:
            inner = shlex.split(argv[2])
        except ValueError:
            return True
        while inner and inner[0] == "exec":
            inner = inner[1:]
        return _script_exists(inner, cwd)
    if len(argv) >= 2 and os.path.basename(argv[0]).startswith("python") and not argv[1].startswith("-"):
        p = argv[1] if os.path.isabs(argv[1]) else os.path.join(cwd or ".", argv[1])
        return os.path.exists(p)
    return True


def expand_env_refs(s: str, env: Dict[str, str]) -> str:
    """Kubernetes dependent-variable expansion of a command/arg string:
    ``$(NAME)`` becomes the container's ``NAME`` when it is defined (else it is
    left as written), ``$$(NAME)`` is the escaped literal ``$(NAME)``."""
    out, i, n = [], 0, len(s)
    while i < n:
        if s.startswith("$$", i):
            out.append("$")
            i += 2
        elif s.startswith("$(", i):
            j = s.find(")", i + 2)
            name = s[i + 2:j] if j > 0 else ""
            if j > 0 and name in env:
                out.append(env[name])
                i = j + 1
            else:
                out.append(s[i:j + 1] if j > 0 else s[i:])
                i = j + 1 if j > 0 else n
        else:
            out.append(s[i])
            i += 1
    return "".join(out)


def resolve_argv(container: dict, cwd: Optional[str], path: str) -> (List[str], str):
    """Return (argv, readiness) for a container spec."""
    cmd = list(container.get("command") or [])
    args = [str(a) for a in (container.get("args") or [])]
    entry = lookup(container.get("image", ""))
    if cmd and _runnable(cmd[0], cwd, path) and _script_exists(cmd, cwd):
        if cmd[0] in ("python", "python3"):
            cmd[0] = sys.executable
        return cmd + args, (entry.readiness if entry else "start")
    if entry is not None:
        return list(entry.entrypoint) + args, entry.readiness
    if cmd:
        return cmd + args, "start"  # let exec fail with 127 like a container runtime
    raise ValueError(f"container {container.get('name')!r}: no command and unknown image "
                     f"{container.get('image')!r}")
