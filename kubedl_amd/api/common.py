"""Common job API shared by every workload kind (the kubeflow ``common/v1`` types).

Wire format is kept bit-for-bit with the reference CRDs: objects are plain
JSON-shaped dicts (``apiVersion/kind/metadata/spec/status``) exactly as a
``kubectl get -o json`` would show them, so specs written for KubeDL load
unchanged and ``status`` round-trips in the ``JobStatus`` persist format.

Reference: ``pkg/job_controller/api/v1/types.go:23-191`` (JobStatus,
ReplicaStatus, ReplicaSpec, JobCondition, CleanPodPolicy, RestartPolicy,
RunPolicy, SchedulingPolicy) and ``constants.go:3-32`` (labels/annotations).
Condition helpers mirror ``pkg/util/status.go:9-137``; the exit-code policy
mirrors ``pkg/util/train/train_util.go:18-52``.
"""
from __future__ import annotations

import copy
import datetime as _dt
import re
from fractions import Fraction
from typing import Any, Dict, List, Optional

# ---- condition types (types.go:101-127)
JOB_CREATED = "Created"
JOB_RUNNING = "Running"
JOB_RESTARTING = "Restarting"
JOB_SUCCEEDED = "Succeeded"
JOB_FAILED = "Failed"
CONDITION_TYPES = (JOB_CREATED, JOB_RUNNING, JOB_RESTARTING, JOB_SUCCEEDED, JOB_FAILED)

# ---- condition reasons (pkg/util/status.go:9-24)
JOB_CREATED_REASON = "JobCreated"
JOB_SUCCEEDED_REASON = "JobSucceeded"
JOB_RUNNING_REASON = "JobRunning"
JOB_FAILED_REASON = "JobFailed"
JOB_RESTARTING_REASON = "JobRestarting"

# ---- clean pod policy (types.go:130-137)
CLEAN_POD_POLICY_UNDEFINED = ""
CLEAN_POD_POLICY_ALL = "All"
CLEAN_POD_POLICY_RUNNING = "Running"
CLEAN_POD_POLICY_NONE = "None"

# ---- restart policy (types.go:143-156)
RESTART_POLICY_ALWAYS = "Always"
RESTART_POLICY_ON_FAILURE = "OnFailure"
RESTART_POLICY_NEVER = "Never"
RESTART_POLICY_EXIT_CODE = "ExitCode"

# ---- labels / annotations (constants.go:3-32)
REPLICA_INDEX_LABEL = "replica-index"
REPLICA_TYPE_LABEL = "replica-type"
GROUP_NAME_LABEL = "group-name"
JOB_NAME_LABEL = "job-name"
JOB_ROLE_LABEL = "job-role"
KUBEDL_PREFIX = "kubedl.io"
ANNOTATION_GIT_SYNC_CONFIG = KUBEDL_PREFIX + "/git-sync-config"
ANNOTATION_TENANCY_INFO = KUBEDL_PREFIX + "/tenancy"
DEFAULT_KUBEDL_NAMESPACE = "kubedl"

# resource names a replica template may use to ask for GPUs (gang allocator)
GPU_RESOURCE_NAMES = ("amd.com/gpu", "nvidia.com/gpu", "gpu")

CONDITION_TRUE = "True"
CONDITION_FALSE = "False"


# --------------------------------------------------------------------------
# time helpers: metav1.Time serialises as RFC3339 with second precision; we
# keep sub-second precision (RFC3339Nano, also valid metav1.Time input) so the
# launch-delay metrics are meaningful on a local runtime that starts ranks in
# milliseconds rather than the seconds a kubelet takes.

def now() -> str:
    return format_time(_dt.datetime.now(_dt.timezone.utc))


def format_time(t: _dt.datetime) -> str:
    if t.tzinfo is None:
        t = t.replace(tzinfo=_dt.timezone.utc)
    t = t.astimezone(_dt.timezone.utc)
    return t.strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def parse_time(s: Optional[str]) -> Optional[_dt.datetime]:
    if not s:
        return None
    if isinstance(s, _dt.datetime):
        return s
    s = s.strip()
    if s.endswith("Z"):
        s = s[:-1] + "+00:00"
    # python <3.11 fromisoformat wants exactly 6 fractional digits
    if "." in s:
        head, rest = s.split(".", 1)
        frac, tz = rest, ""
        for sep in ("+", "-"):
            if sep in rest:
                frac, tz = rest.split(sep, 1)
                tz = sep + tz
                break
        frac = (frac + "000000")[:6]
        s = f"{head}.{frac}{tz}"
    return _dt.datetime.fromisoformat(s)


def to_epoch(s: Optional[str]) -> Optional[float]:
    t = parse_time(s)
    return t.timestamp() if t is not None else None


# --------------------------------------------------------------------------
# JobStatus helpers (operate on the JSON dict form)

def new_job_status() -> Dict[str, Any]:
    return {"conditions": [], "replicaStatuses": {}}


def ensure_status(job: Dict[str, Any]) -> Dict[str, Any]:
    st = job.get("status")
    if not st:
        st = new_job_status()
        job["status"] = st
    st.setdefault("conditions", [])
    if st.get("replicaStatuses") is None:
        st["replicaStatuses"] = {}
    return st


def replica_status(status: Dict[str, Any], rtype: str) -> Dict[str, int]:
    rs = status.setdefault("replicaStatuses", {})
    if rs.get(rtype) is None:
        rs[rtype] = {}
    return rs[rtype]


def rs_get(rs: Optional[Dict[str, int]], field: str) -> int:
    """ReplicaStatus fields are int32 ``omitempty``: a missing key is 0."""
    if not rs:
        return 0
    return int(rs.get(field, 0) or 0)


def rs_inc(rs: Dict[str, int], field: str, by: int = 1) -> None:
    v = rs_get(rs, field) + by
    if v:
        rs[field] = v
    else:
        rs.pop(field, None)


def rs_set(rs: Dict[str, int], field: str, value: int) -> None:
    if value:
        rs[field] = int(value)
    else:
        rs.pop(field, None)


def has_condition(status: Dict[str, Any], ctype: str) -> bool:
    for c in (status or {}).get("conditions") or []:
        if c.get("type") == ctype and c.get("status") == CONDITION_TRUE:
            return True
    return False


def is_succeeded(status) -> bool:
    return has_condition(status, JOB_SUCCEEDED)


def is_failed(status) -> bool:
    return has_condition(status, JOB_FAILED)


def is_running(status) -> bool:
    return has_condition(status, JOB_RUNNING)


def is_created(status) -> bool:
    return has_condition(status, JOB_CREATED)


def is_restarting(status) -> bool:
    return has_condition(status, JOB_RESTARTING)


def get_condition(status: Dict[str, Any], ctype: str) -> Optional[Dict[str, Any]]:
    for c in (status or {}).get("conditions") or []:
        if c.get("type") == ctype:
            return c
    return None


def new_condition(ctype: str, reason: str, message: str, ts: Optional[str] = None) -> Dict[str, Any]:
    t = ts or now()
    return {"type": ctype, "status": CONDITION_TRUE, "reason": reason, "message": message,
            "lastUpdateTime": t, "lastTransitionTime": t}


def _filter_out_condition(conds: List[Dict[str, Any]], ctype: str) -> List[Dict[str, Any]]:
    out = []
    for c in conds:
        # Running and Restarting are mutually exclusive (status.go:111-118)
        if ctype == JOB_RESTARTING and c.get("type") == JOB_RUNNING:
            continue
        if ctype == JOB_RUNNING and c.get("type") == JOB_RESTARTING:
            continue
        if c.get("type") == ctype:
            continue
        if ctype in (JOB_FAILED, JOB_SUCCEEDED) and c.get("type") == JOB_RUNNING:
            c = dict(c)
            c["status"] = CONDITION_FALSE
        out.append(c)
    return out


def update_job_conditions(status: Dict[str, Any], ctype: str, reason: str, message: str,
                          ts: Optional[str] = None) -> None:
    """``UpdateJobConditions``: append/replace a condition with reference semantics.

    * no-op once the job is Failed;
    * same type + status + reason already present => no-op;
    * same type + status => keep the old lastTransitionTime;
    * Running <-> Restarting replace each other; Succeeded/Failed flip Running to False.
    """
    cond = new_condition(ctype, reason, message, ts)
    if is_failed(status):
        return
    cur = get_condition(status, ctype)
    if cur is not None and cur.get("status") == cond["status"] and cur.get("reason") == cond["reason"]:
        return
    if cur is not None and cur.get("status") == cond["status"]:
        cond["lastTransitionTime"] = cur.get("lastTransitionTime")
    status["conditions"] = _filter_out_condition(status.get("conditions") or [], ctype) + [cond]


def last_condition_type(status: Dict[str, Any]) -> str:
    conds = (status or {}).get("conditions") or []
    return conds[-1].get("type", "") if conds else ""


# --------------------------------------------------------------------------
# exit-code policy (train_util.go:18-52).  NOTE: the API comment at
# types.go:150-155 claims 128-255 are retryable; the code (which we follow)
# treats only 130/137/143 (SIGINT/SIGKILL/SIGTERM) and 138 (SIGUSR1, the
# user-requested retry) as retryable, everything else as permanent.

def is_retryable_exit_code(code: int) -> bool:
    if code in (1, 2, 126, 127, 128, 139):
        return False
    if code in (130, 137, 143):
        return True
    if code == 138:
        return True
    return False


# --------------------------------------------------------------------------
# replica-spec helpers

def replicas_of(spec: Dict[str, Any]) -> int:
    r = spec.get("replicas")
    return 1 if r is None else int(r)


def total_replicas(specs: Dict[str, Dict[str, Any]]) -> int:
    """k8sutil.GetTotalReplicas (replicas default to 1 when unset)."""
    return sum(replicas_of(s) for s in (specs or {}).values())


def total_active(replica_statuses: Dict[str, Any]) -> int:
    return sum(rs_get(v, "active") for v in (replica_statuses or {}).values())


def total_failed(replica_statuses: Dict[str, Any]) -> int:
    return sum(rs_get(v, "failed") for v in (replica_statuses or {}).values())


def containers_of(spec: Dict[str, Any]) -> List[Dict[str, Any]]:
    return (((spec.get("template") or {}).get("spec") or {}).get("containers")) or []


def port_from_job(specs: Dict[str, Dict[str, Any]], rtype: str, container_name: str,
                  port_name: str) -> int:
    """job_controller.GetPortFromJob (util.go:59-73)."""
    spec = specs.get(rtype)
    if spec is None:
        raise KeyError(f"replica type {rtype} not in job")
    for c in containers_of(spec):
        if c.get("name") == container_name:
            for p in c.get("ports") or []:
                if p.get("name") == port_name:
                    return int(p.get("containerPort"))
    raise LookupError("failed to found the port")


def gpus_requested(container: Dict[str, Any]) -> int:
    res = container.get("resources") or {}
    for section in ("limits", "requests"):
        d = res.get(section) or {}
        for k in GPU_RESOURCE_NAMES:
            if k in d:
                return int(str(d[k]))
    return 0


def pod_template_gpus(template: Dict[str, Any]) -> int:
    return sum(gpus_requested(c) for c in ((template or {}).get("spec") or {}).get("containers") or [])


HBM_RESOURCE = "kubedl.io/hbm-gb"

# Kubernetes resource quantities (k8s.io/apimachinery resource.Quantity syntax)
QUANTITY_SUFFIX = {"": 1, "m": Fraction(1, 1000), "k": 10 ** 3, "M": 10 ** 6, "G": 10 ** 9, "T": 10 ** 12,
                   "P": 10 ** 15, "E": 10 ** 18, "Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40,
                   "Pi": 2 ** 50, "Ei": 2 ** 60}
_QRE = re.compile(r"^([+-]?[0-9.]+(?:[eE][+-]?[0-9]+)?)(Ki|Mi|Gi|Ti|Pi|Ei|m|k|M|G|T|P|E)?$")


def parse_quantity(q) -> Fraction:
    if isinstance(q, (int, float)):
        return Fraction(q)
    m = _QRE.match(str(q).strip())
    if not m:
        raise ValueError(f"bad quantity {q!r}")
    return Fraction(m.group(1)) * QUANTITY_SUFFIX[m.group(2) or ""]


def parse_hbm_gb(v) -> float:
    """A ``kubedl.io/hbm-gb`` value in GB: a bare number is GB; a quantity with
    a byte suffix (``32G``, ``32Gi``, ``512Mi``) is bytes converted to GB.
    Raises ValueError on garbage or a negative request."""
    s = str(v).strip()
    q = parse_quantity(s)
    m = _QRE.match(s)
    suf = m.group(2) if m else None
    gb = float(q) if not suf or suf == "m" else float(q) / 1e9
    if gb < 0:
        raise ValueError(f"negative {HBM_RESOURCE} request {v!r}")
    return gb


def hbm_requested(container: Dict[str, Any]) -> float:
    """``kubedl.io/hbm-gb`` of a container (limits, else requests), in GB."""
    res = container.get("resources") or {}
    for section in ("limits", "requests"):
        d = res.get(section) or {}
        if HBM_RESOURCE in d:
            return parse_hbm_gb(d[HBM_RESOURCE])
    return 0.0


def pod_template_hbm(template: Dict[str, Any]) -> float:
    return sum(hbm_requested(c) for c in ((template or {}).get("spec") or {}).get("containers") or [])


def gen_general_name(job_name: str, rtype: str, index) -> str:
    """GenGeneralName (util.go:29-32): ``<job>-<rtype>-<index>`` with '/' -> '-'."""
    return f"{job_name}-{rtype}-{index}".replace("/", "-")


def gen_expectation_pods_key(job_key: str, rtype: str) -> str:
    return f"{job_key}/{rtype.lower()}/pods"


def gen_expectation_services_key(job_key: str, rtype: str) -> str:
    return f"{job_key}/{rtype.lower()}/services"


def deepcopy(o):
    return copy.deepcopy(o)
