"""Persistence data model (DMO) and converters.

Row shapes are the reference's gorm models (``pkg/storage/dmo/types.go``):
tables ``job_info`` (Job), ``replica_info`` (Pod), ``event_info`` (Event)
with the same column names (``gmt_created``/``gmt_modified``/
``gmt_started``/``gmt_finished``, ``deleted``, ``is_in_etcd``,
``resources`` JSON, ``deploy_region``, ``tenant``/``owner``, ``remark``).

Converters follow ``pkg/storage/dmo/converters/{job,pod,event}.go``:

* job status = type of the LAST condition (``Created`` when none);
* job resources = per replica type ``{"resources": <pod resources>,
  "replicas": n}``; pod resources = max(max over init containers, sum over
  containers) for requests and limits (``computePodResources``);
* tenancy annotation ``kubedl.io/tenancy`` -> tenant / owner (user) and the
  region fallback;
* pod status = phase; started/finished from the default container's state;
  failed pods carry ``Reason/ExitCode/Message`` in ``remark``;
* [fix] event rows keep ``obj_namespace/obj_name/obj_uid`` (the reference's
  converter drops them, ``converters/event.go:28-38``) and ``count`` gets its
  own column (the reference maps it onto ``reason``, ``types.go:129``).
"""
from __future__ import annotations

import json
import re
from fractions import Fraction
from typing import Dict, Optional

from kubedl_amd.api import common as c
from kubedl_amd.api import kinds as K
from kubedl_amd.utils import k8sutil

# ---------------------------------------------------------------- quantities
from kubedl_amd.api.common import QUANTITY_SUFFIX as _SUFFIX, parse_quantity  # noqa: E402,F401


def format_quantity(v: Fraction, binary: bool = False) -> str:
    if v.denominator != 1:
        milli = v * 1000
        return f"{int(milli)}m" if milli.denominator == 1 else str(float(v))
    n = int(v)
    if binary and n:
        for suf in ("Ei", "Pi", "Ti", "Gi", "Mi", "Ki"):
            if n % _SUFFIX[suf] == 0:
                return f"{n // _SUFFIX[suf]}{suf}"
    return str(n)


def _is_binary(name: str) -> bool:
    return name in ("memory", "ephemeral-storage", "storage") or name.endswith("-memory")


def _res_sum(lists):
    out: Dict[str, Fraction] = {}
    for d in lists:
        for k, v in (d or {}).items():
            out[k] = out.get(k, Fraction(0)) + parse_quantity(v)
    return out


def _res_max(a: Dict[str, Fraction], b: Dict[str, Fraction]):
    out = dict(a)
    for k, v in b.items():
        out[k] = max(out.get(k, v), v)
    return out


def compute_pod_resources(pod_spec: dict) -> dict:
    """max(max over init containers, sum over containers), requests and limits.
    Key order is the serialised ``ResourceRequirements`` (limits, requests;
    resource names sorted) so ``go_json`` reproduces the reference's column."""
    res = {}
    for sect in ("limits", "requests"):
        init_max: Dict[str, Fraction] = {}
        for ic in pod_spec.get("initContainers") or []:
            cur = {k: parse_quantity(v) for k, v in ((ic.get("resources") or {}).get(sect) or {}).items()}
            init_max = _res_max(init_max, cur)
        run = _res_sum(((ct.get("resources") or {}).get(sect) or {}) for ct in pod_spec.get("containers") or [])
        tot = _res_max(init_max, run)
        if tot:
            res[sect] = {k: format_quantity(v, _is_binary(k)) for k, v in sorted(tot.items())}
    return res


def go_json(obj) -> str:
    """``encoding/json`` shape: compact separators, dict order as built."""
    return json.dumps(obj, separators=(",", ":"))


# ---------------------------------------------------------------- tenancy
def get_tenancy(meta: dict) -> Optional[dict]:
    raw = (meta.get("annotations") or {}).get(c.ANNOTATION_TENANCY_INFO)
    if raw is None:
        return None
    t = json.loads(raw)
    return {"tenant": t.get("tenant", ""), "user": t.get("user", ""), "idc": t.get("idc", ""),
            "region": t.get("region", "")}


# ---------------------------------------------------------------- converters
def job_to_dmo(job: dict, region: str = "") -> dict:
    md = job["metadata"]
    st = job.get("status") or {}
    specs = K.replica_specs(job) if job.get("kind") in K.BY_KIND else {}
    row = {"name": md["name"], "namespace": md["namespace"], "job_id": md.get("uid", ""),
           "version": md.get("resourceVersion", ""), "kind": job["kind"], "resources": "",
           "gmt_created": md.get("creationTimestamp"), "deploy_region": region or None,
           "tenant": "", "owner": "", "deleted": 0, "is_in_etcd": 1, "gmt_finished": None}
    try:
        tn = get_tenancy(md)
    except ValueError:
        tn = None
    if tn is not None:
        row["tenant"], row["owner"] = tn["tenant"], tn["user"]
        if not row["deploy_region"] and tn["region"]:
            row["deploy_region"] = tn["region"]
    conds = st.get("conditions") or []
    row["status"] = conds[-1]["type"] if conds else c.JOB_CREATED
    if st.get("completionTime"):
        row["gmt_finished"] = st["completionTime"]
    res = {}
    for rt in sorted(specs):  # Go marshals map keys sorted; struct fields in declaration order
        spec = specs[rt]
        res[rt] = {"resources": compute_pod_resources((spec.get("template") or {}).get("spec") or {}),
                   "replicas": int(spec["replicas"]) if spec.get("replicas") is not None else 0}
    row["resources"] = go_json(res)
    return row


class ConvertError(ValueError):
    pass


def pod_to_dmo(pod: dict, default_container: str, region: str = "") -> dict:
    md = pod["metadata"]
    job_id, _ = k8sutil.resolve_dependent_owner(pod)
    if not job_id:
        raise ConvertError("object has no dependent owner")
    rtype = (md.get("labels") or {}).get(c.REPLICA_TYPE_LABEL)
    if rtype is None:
        raise ConvertError(f"object has no replica type label [{c.REPLICA_TYPE_LABEL}]")
    spec = pod.get("spec") or {}
    st = pod.get("status") or {}
    row = {"name": md["name"], "namespace": md["namespace"], "pod_id": md.get("uid", ""),
           "version": md.get("resourceVersion", ""), "gmt_created": md.get("creationTimestamp"),
           "deploy_region": region or None, "job_id": job_id, "replica_type": rtype,
           "resources": go_json(compute_pod_resources(spec)),
           "deleted": 0, "is_in_etcd": 1, "pod_ip": st.get("podIP") or None,
           "host_ip": st.get("hostIP") or None, "image": "", "status": "",
           "gmt_started": None, "gmt_finished": None, "remark": None}
    ctrs = spec.get("containers") or []
    if not ctrs:
        return row
    image = ctrs[0].get("image", "")
    for ct in ctrs:
        if ct.get("name") == default_container:
            image = ct.get("image", "")
            break
    row["image"] = image
    row["status"] = "Unknown"  # defaulted once the pod has containers (converters/pod.go:97)
    css = st.get("containerStatuses") or []
    if not css:
        return row
    cs = css[0]
    for x in css[1:]:
        if x.get("name") == default_container:
            cs = x
            break
    phase = st.get("phase", "")
    row["status"] = phase
    state = cs.get("state") or {}
    if phase == "Running":
        row["gmt_started"] = (state.get("running") or {}).get("startedAt") or md.get("creationTimestamp")
    elif phase in ("Succeeded", "Failed"):
        term = state.get("terminated")
        if term is not None:
            row["gmt_started"] = term.get("startedAt")
            row["gmt_finished"] = term.get("finishedAt")
            if phase == "Failed":
                row["remark"] = (f"Reason: {term.get('reason', '')}\nExitCode: {term.get('exitCode', 0)}\n"
                                 f"Message: {term.get('message', '')}")
        row["gmt_started"] = row["gmt_started"] or md.get("creationTimestamp")
        row["gmt_finished"] = row["gmt_finished"] or c.now()
    return row


def event_to_dmo(ev: dict, region: str = "") -> dict:
    io = ev.get("involvedObject") or {}
    return {"name": ev["metadata"]["name"], "kind": io.get("kind", ""), "type": ev.get("type", ""),
            "obj_namespace": io.get("namespace", ""), "obj_name": io.get("name", ""),
            "obj_uid": io.get("uid", ""), "reason": ev.get("reason", ""), "message": ev.get("message", ""),
            "count": int(ev.get("count") or 0), "region": region or None,
            "first_timestamp": ev.get("firstTimestamp"), "last_timestamp": ev.get("lastTimestamp")}
