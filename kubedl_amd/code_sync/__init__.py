"""Remote code sync (``pkg/code_sync``): git-sync init container injection.

If the job carries the annotation ``kubedl.io/git-sync-config`` (JSON, see
``docs/sync_code.md``), every replica template gets

* an init container ``git-sync-code`` (image ``kubedl/git-sync:v1`` unless
  overridden, ``GIT_SYNC_*`` env, one-time sync) whose resources copy those
  of container 0,
* an ``emptyDir`` volume ``git-sync``,
* a mount of that volume (``subPath: <dest>``) into every container at
  ``<workingDir>/<dest>``.

Reference: ``sync_handler.go:33-73`` and ``git_sync_handler.go:12-152``
(defaults: rootPath ``/code``, destPath = last path element of ``source``
without ``.git``, maxFailures 3).  The option key is ``revision`` as in the
code (the docs' ``revison`` is a typo).

On the local runtime the init container runs ``python -m
kubedl_amd.code_sync.git_sync`` (a ``git clone`` driven by the same
``GIT_SYNC_*`` variables) inside the pod sandbox before the main container.
"""
from __future__ import annotations

import json
import posixpath
from typing import Dict, List, Tuple

from kubedl_amd.api import common as c

DEFAULT_CODE_ROOT_PATH = "/code"
DEFAULT_GIT_SYNC_IMAGE = "kubedl/git-sync:v1"
INIT_CONTAINER_NAME = "git-sync-code"
VOLUME_NAME = "git-sync"


def _set_default_sync_opts(o: dict) -> None:
    if not o.get("rootPath"):
        o["rootPath"] = DEFAULT_CODE_ROOT_PATH
    if not o.get("destPath"):
        parts = (o.get("source") or "").strip("/").split("/")
        dest = parts[-1]
        if dest.endswith(".git"):
            dest = dest[:-4]
        o["destPath"] = dest
    if not o.get("image"):
        o["image"] = DEFAULT_GIT_SYNC_IMAGE
    if not o.get("maxFailures"):
        o["maxFailures"] = 3


def _sync_envs(o: dict) -> List[dict]:
    envs = list(o.get("envs") or [])
    envs.append({"name": "GIT_SYNC_REPO", "value": o.get("source", "")})
    envs.append({"name": "GIT_SYNC_ONE_TIME", "value": "true"})
    if int(o.get("maxFailures", 0)) >= 0:
        envs.append({"name": "GIT_SYNC_MAX_SYNC_FAILURES", "value": str(int(o["maxFailures"]))})
    if o.get("branch"):
        envs.append({"name": "GIT_SYNC_BRANCH", "value": o["branch"]})
    if o.get("revision"):
        envs.append({"name": "GIT_SYNC_REV", "value": o["revision"]})
    if o.get("depth"):
        envs.append({"name": "GIT_SYNC_DEPTH", "value": str(o["depth"])})
    if o.get("rootPath"):
        envs.append({"name": "GIT_SYNC_ROOT", "value": o["rootPath"]})
    if o.get("destPath"):
        envs.append({"name": "GIT_SYNC_DEST", "value": o["destPath"]})
    if o.get("ssh"):
        envs.append({"name": "GIT_SYNC_SSH", "value": "true"})
    if o.get("ssh") and o.get("sshFile"):
        envs.append({"name": "GIT_SSH_KEY_FILE", "value": o["sshFile"]})
    if o.get("user"):
        envs.append({"name": "GIT_SYNC_USERNAME", "value": o["user"]})
    if o.get("password"):
        envs.append({"name": "GIT_SYNC_PASSWORD", "value": o["password"]})
    return envs


def git_sync_init_container(opts_json: str, volume: dict) -> Tuple[dict, str]:
    """gitSyncHandler.InitContainer -> (container, destPath)."""
    opts = json.loads(opts_json)
    if not isinstance(opts, dict):
        raise ValueError("git-sync-config must be a JSON object")
    _set_default_sync_opts(opts)
    ctr = {
        "name": INIT_CONTAINER_NAME,
        "image": opts["image"],
        "env": _sync_envs(opts),
        "imagePullPolicy": "IfNotPresent",
        "volumeMounts": [{"name": volume["name"], "readOnly": False, "mountPath": opts["rootPath"]}],
    }
    return ctr, opts["destPath"]


def inject_code_sync_init_containers(job_meta: dict, specs: Dict[str, dict]) -> None:
    """InjectCodeSyncInitContainers: mutate the (in-memory) replica specs."""
    cfg = ((job_meta or {}).get("annotations") or {}).get(c.ANNOTATION_GIT_SYNC_CONFIG)
    if cfg is None:
        return
    volume = {"name": VOLUME_NAME, "emptyDir": {}}
    init, dest = git_sync_init_container(cfg, volume)
    for spec in specs.values():
        pod_spec = spec.setdefault("template", {}).setdefault("spec", {})
        ctrs = pod_spec.get("containers") or []
        ic = json.loads(json.dumps(init))
        if ctrs:
            ic["resources"] = json.loads(json.dumps(ctrs[0].get("resources") or {}))
        pod_spec.setdefault("initContainers", []).append(ic)
        pod_spec.setdefault("volumes", []).append(dict(volume))
        for ctr in ctrs:
            ctr.setdefault("volumeMounts", []).append({
                "name": VOLUME_NAME, "readOnly": False,
                "mountPath": posixpath.join(ctr.get("workingDir") or "", dest),
                "subPath": dest,
            })
