"""The four workload kinds: schema constants + defaulting (``SetDefaults_*``).

One ``KindInfo`` per CRD carries what the reference spreads over
``api/<fw>/<ver>/{types,constants,register,defaults}.go``:

=============  =====================================  ==================  ===========================
kind           group/version                          replica-spec field  reference
=============  =====================================  ==================  ===========================
TFJob          kubeflow.org/v1                        tfReplicaSpecs      api/tensorflow/v1/*.go
PyTorchJob     kubeflow.org/v1                        pytorchReplicaSpecs api/pytorch/v1/*.go
XGBoostJob     xgboostjob.kubeflow.org/v1alpha1       xgbReplicaSpecs     api/xgboost/v1alpha1/*.go
XDLJob         xdl.kubedl.io/v1alpha1                 xdlReplicaSpecs     api/xdl/v1alpha1/*.go
=============  =====================================  ==================  ===========================

Per-kind defaulting quirks preserved:

* TFJob: cleanPodPolicy ``Running``; replicas 1; restartPolicy ``ExitCode``;
  default port ``tfjob-port``/2222 added to every replica type
  (``api/tensorflow/v1/defaults.go:36-108``).
* PyTorchJob: cleanPodPolicy ``None``; Master restart ``ExitCode``, Worker
  restart ``OnFailure``; the port is added ONLY to Master
  (``api/pytorch/v1/defaults.go:36-117``).
* XGBoostJob: cleanPodPolicy ``None``; ttlSecondsAfterFinished 100; replicas 1;
  NO default restart policy (``api/xgboost/v1alpha1/defaults.go:37-109``).
* XDLJob: cleanPodPolicy ``Running``; ``minFinishWorkRate`` 90 when neither
  min-finish field is set; backoffLimit 20; restart ``Never``
  (``api/xdl/v1alpha1/defaults.go:37-119``).

Replica-type keys are case-normalised (``ps`` -> ``PS``) the way
``setTypeNameToCamelCase`` does: only the first case-insensitive match per
canonical type is renamed.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

from kubedl_amd.api import common as c


@dataclass(frozen=True)
class KindInfo:
    kind: str
    group: str
    version: str
    plural: str
    singular: str
    spec_field: str
    replica_types: Tuple[str, ...]
    default_container: str
    default_port_name: str
    default_port: int
    # order in which ReconcilePods visits replica types (GetReconcileOrders)
    reconcile_order: Tuple[str, ...]
    # value of the group-name label put on pods/services (GetGroupNameLabelValue)
    group_label: str
    defaulter: Callable[[dict], None] = field(compare=False, repr=False, default=None)

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}"

    @property
    def crd_name(self) -> str:
        return f"{self.plural}.{self.group}"


# ---------------------------------------------------------------- helpers

def _set_default_port(pod_spec: dict, container_name: str, port_name: str, port: int) -> None:
    """setDefaultPort: pick the container named ``container_name`` (index 0
    when absent) and append ``{name: port_name, containerPort: port}`` unless a
    port with that name already exists."""
    containers = pod_spec.setdefault("containers", [])
    if not containers:
        return  # the reference would panic on Containers[0]; an empty template gets no port
    idx = 0
    for i, ctr in enumerate(containers):
        if ctr.get("name") == container_name:
            idx = i
            break
    ports = containers[idx].setdefault("ports", [])
    if not any(p.get("name") == port_name for p in ports):
        ports.append({"name": port_name, "containerPort": port})


def _camel_case_types(specs: dict, canonical: Tuple[str, ...]) -> None:
    for typ in canonical:
        for t in list(specs.keys()):
            if t.lower() == typ.lower() and t != typ:
                specs[typ] = specs.pop(t)
                break


def _pod_spec(replica_spec: dict) -> dict:
    tmpl = replica_spec.setdefault("template", {})
    return tmpl.setdefault("spec", {})


# ---------------------------------------------------------------- TFJob

TF_PS, TF_WORKER, TF_CHIEF, TF_MASTER, TF_EVAL = "PS", "Worker", "Chief", "Master", "Evaluator"


def _default_tfjob(job: dict) -> None:
    spec = job.setdefault("spec", {})
    if spec.get("cleanPodPolicy") is None:
        spec["cleanPodPolicy"] = c.CLEAN_POD_POLICY_RUNNING
    specs = spec.setdefault("tfReplicaSpecs", {}) or {}
    spec["tfReplicaSpecs"] = specs
    _camel_case_types(specs, (TF_PS, TF_WORKER, TF_CHIEF, TF_MASTER, TF_EVAL))
    for rs in specs.values():
        if rs.get("replicas") is None:
            rs["replicas"] = 1
        if not rs.get("restartPolicy"):
            rs["restartPolicy"] = c.RESTART_POLICY_EXIT_CODE
        _set_default_port(_pod_spec(rs), "tensorflow", "tfjob-port", 2222)


TFJOB = KindInfo(
    kind="TFJob", group="kubeflow.org", version="v1", plural="tfjobs", singular="tfjob",
    spec_field="tfReplicaSpecs", replica_types=(TF_PS, TF_WORKER, TF_CHIEF, TF_MASTER, TF_EVAL),
    default_container="tensorflow", default_port_name="tfjob-port", default_port=2222,
    # Evaluator is absent on purpose: the reference never creates Evaluator
    # pods (controllers/tensorflow/tfjob_controller.go:263-270).
    reconcile_order=(TF_PS, TF_MASTER, TF_CHIEF, TF_WORKER),
    group_label="kubeflow.org", defaulter=_default_tfjob)


def tf_is_chief_or_master(rtype: str) -> bool:
    return rtype in (TF_CHIEF, TF_MASTER)


# ---------------------------------------------------------------- PyTorchJob

PT_MASTER, PT_WORKER = "Master", "Worker"


def _default_pytorchjob(job: dict) -> None:
    spec = job.setdefault("spec", {})
    if spec.get("cleanPodPolicy") is None:
        spec["cleanPodPolicy"] = c.CLEAN_POD_POLICY_NONE
    specs = spec.setdefault("pytorchReplicaSpecs", {}) or {}
    spec["pytorchReplicaSpecs"] = specs
    _camel_case_types(specs, (PT_MASTER, PT_WORKER))
    for rtype, rs in specs.items():
        if rtype == PT_WORKER:
            if rs.get("replicas") is None:
                rs["replicas"] = 1
            if not rs.get("restartPolicy"):
                rs["restartPolicy"] = c.RESTART_POLICY_ON_FAILURE
        if rtype == PT_MASTER:
            if rs.get("replicas") is None:
                rs["replicas"] = 1
            if not rs.get("restartPolicy"):
                rs["restartPolicy"] = c.RESTART_POLICY_EXIT_CODE
            _set_default_port(_pod_spec(rs), "pytorch", "pytorchjob-port", 23456)


PYTORCHJOB = KindInfo(
    kind="PyTorchJob", group="kubeflow.org", version="v1", plural="pytorchjobs",
    singular="pytorchjob", spec_field="pytorchReplicaSpecs", replica_types=(PT_MASTER, PT_WORKER),
    default_container="pytorch", default_port_name="pytorchjob-port", default_port=23456,
    reconcile_order=(PT_MASTER, PT_WORKER), group_label="kubeflow.org",
    defaulter=_default_pytorchjob)


# ---------------------------------------------------------------- XGBoostJob

XGB_MASTER, XGB_WORKER = "Master", "Worker"


def _default_xgboostjob(job: dict) -> None:
    spec = job.setdefault("spec", {})
    # RunPolicy is inlined into the spec (CRD: spec.cleanPodPolicy ...)
    if spec.get("cleanPodPolicy") is None:
        spec["cleanPodPolicy"] = c.CLEAN_POD_POLICY_NONE
    if spec.get("ttlSecondsAfterFinished") is None:
        spec["ttlSecondsAfterFinished"] = 100
    specs = spec.setdefault("xgbReplicaSpecs", {}) or {}
    spec["xgbReplicaSpecs"] = specs
    _camel_case_types(specs, (XGB_MASTER, XGB_WORKER))
    for rs in specs.values():
        if rs.get("replicas") is None:
            rs["replicas"] = 1
        # no default restart policy for XGBoost (defaults.go:84-88)
        _set_default_port(_pod_spec(rs), "xgboostjob", "xgboostjob-port", 9999)


XGBOOSTJOB = KindInfo(
    kind="XGBoostJob", group="xgboostjob.kubeflow.org", version="v1alpha1", plural="xgboostjobs",
    singular="xgboostjob", spec_field="xgbReplicaSpecs", replica_types=(XGB_MASTER, XGB_WORKER),
    default_container="xgboostjob", default_port_name="xgboostjob-port", default_port=9999,
    reconcile_order=(XGB_MASTER, XGB_WORKER),
    # quirk: the group-name label is "kubeflow.org", not the API group
    # (controllers/xgboost/xgboostjob_controller.go:168-170 -> constants.go:24)
    group_label="kubeflow.org", defaulter=_default_xgboostjob)


# ---------------------------------------------------------------- XDLJob

XDL_PS, XDL_WORKER, XDL_SCHEDULER, XDL_EXTEND = "PS", "Worker", "Scheduler", "ExtendRole"
XDL_DEFAULT_MIN_FINISH_WORK_RATE = 90
XDL_DEFAULT_BACKOFF_LIMIT = 20


def _default_xdljob(job: dict) -> None:
    spec = job.setdefault("spec", {})
    if spec.get("cleanPodPolicy") is None:
        spec["cleanPodPolicy"] = c.CLEAN_POD_POLICY_RUNNING
    if spec.get("minFinishWorkNum") is None and spec.get("minFinishWorkRate") is None:
        spec["minFinishWorkRate"] = XDL_DEFAULT_MIN_FINISH_WORK_RATE
    if spec.get("backoffLimit") is None:
        spec["backoffLimit"] = XDL_DEFAULT_BACKOFF_LIMIT
    specs = spec.setdefault("xdlReplicaSpecs", {}) or {}
    spec["xdlReplicaSpecs"] = specs
    _camel_case_types(specs, (XDL_WORKER, XDL_PS, XDL_SCHEDULER, XDL_EXTEND))
    for rs in specs.values():
        if rs.get("replicas") is None:
            rs["replicas"] = 1
        if not rs.get("restartPolicy"):
            rs["restartPolicy"] = c.RESTART_POLICY_NEVER
        _set_default_port(_pod_spec(rs), "xdl", "xdljob-port", 2222)


XDLJOB = KindInfo(
    kind="XDLJob", group="xdl.kubedl.io", version="v1alpha1", plural="xdljobs", singular="xdljob",
    spec_field="xdlReplicaSpecs", replica_types=(XDL_PS, XDL_WORKER, XDL_SCHEDULER, XDL_EXTEND),
    default_container="xdl", default_port_name="xdljob-port", default_port=2222,
    reconcile_order=(XDL_PS, XDL_SCHEDULER, XDL_WORKER, XDL_EXTEND),
    group_label="xdl.kubedl.io", defaulter=_default_xdljob)


ALL_KINDS: Tuple[KindInfo, ...] = (TFJOB, PYTORCHJOB, XGBOOSTJOB, XDLJOB)
BY_KIND: Dict[str, KindInfo] = {k.kind: k for k in ALL_KINDS}
_ALIASES: Dict[str, KindInfo] = {}
for _k in ALL_KINDS:
    for _a in (_k.kind, _k.kind.lower(), _k.plural, _k.singular):
        _ALIASES[_a.lower()] = _k
# README.md:54 spells it "PytorchJob"; accept it as an alias
_ALIASES["pytorchjob"] = PYTORCHJOB
_ALIASES["tf"] = TFJOB
_ALIASES["pytorch"] = PYTORCHJOB
_ALIASES["xgboost"] = XGBOOSTJOB
_ALIASES["xdl"] = XDLJOB


def lookup(name: str) -> KindInfo:
    k = _ALIASES.get(str(name).lower())
    if k is None:
        raise KeyError(f"unknown workload kind {name!r}; known: {[x.kind for x in ALL_KINDS]}")
    return k


def is_job_kind(kind: str) -> bool:
    return kind in BY_KIND


def set_defaults(job: dict) -> dict:
    """Scheme.Default: apply the kind's SetDefaults_* in place; returns job."""
    info = BY_KIND[job["kind"]]
    info.defaulter(job)
    md = job.setdefault("metadata", {})
    md.setdefault("namespace", "default")
    return job


def replica_specs(job: dict) -> Dict[str, dict]:
    spec = job.get("spec") or {}
    info = BY_KIND.get(job["kind"])
    if info is None:  # a kind outside the four (e.g. the engine's TestJob): its single *ReplicaSpecs map
        for k, v in spec.items():
            if k.endswith("ReplicaSpecs") and isinstance(v, dict):
                return v
        return {}
    return spec.get(info.spec_field) or {}


RUN_POLICY_FIELDS = ("cleanPodPolicy", "ttlSecondsAfterFinished", "activeDeadlineSeconds",
                     "backoffLimit", "schedulingPolicy")


def run_policy(job: dict) -> dict:
    """RunPolicy is inlined into every JobSpec; return a view-copy of its fields."""
    spec = job.get("spec") or {}
    return {k: spec[k] for k in RUN_POLICY_FIELDS if spec.get(k) is not None}


def validate(job: dict) -> List[str]:
    """Structural validation equivalent to the CRD openAPI ``required`` lists."""
    errs: List[str] = []
    if job.get("kind") not in BY_KIND:
        return [f"unknown kind {job.get('kind')!r}"]
    info = BY_KIND[job["kind"]]
    if job.get("apiVersion") != info.api_version:
        errs.append(f"apiVersion must be {info.api_version}, got {job.get('apiVersion')!r}")
    md = job.get("metadata") or {}
    if not md.get("name"):
        errs.append("metadata.name is required")
    spec = job.get("spec")
    if not isinstance(spec, dict):
        errs.append("spec is required")
        return errs
    if not isinstance(spec.get(info.spec_field), dict) or not spec.get(info.spec_field):
        errs.append(f"spec.{info.spec_field} is required")
        return errs
    for rtype, rs in spec[info.spec_field].items():
        if rtype not in info.replica_types and rtype.lower() not in [t.lower() for t in info.replica_types]:
            errs.append(f"unknown replica type {rtype!r} for {info.kind}")
        if not isinstance(rs, dict):
            errs.append(f"replica spec {rtype} must be an object")
            continue
        r = rs.get("replicas")
        if r is not None and (not isinstance(r, int) or r < 0):
            errs.append(f"{rtype}.replicas must be a non-negative integer")
        rp = rs.get("restartPolicy")
        if rp and rp not in (c.RESTART_POLICY_ALWAYS, c.RESTART_POLICY_ON_FAILURE,
                             c.RESTART_POLICY_NEVER, c.RESTART_POLICY_EXIT_CODE):
            errs.append(f"{rtype}.restartPolicy {rp!r} invalid")
        ctrs = ((rs.get("template") or {}).get("spec") or {}).get("containers")
        if not ctrs:
            errs.append(f"{rtype}.template.spec.containers is required")
    cpp = spec.get("cleanPodPolicy")
    if cpp is not None and cpp not in (c.CLEAN_POD_POLICY_ALL, c.CLEAN_POD_POLICY_RUNNING,
                                       c.CLEAN_POD_POLICY_NONE, c.CLEAN_POD_POLICY_UNDEFINED):
        errs.append(f"cleanPodPolicy {cpp!r} invalid")
    return errs


def print_columns(job: dict, now_epoch: Optional[float] = None) -> Dict[str, str]:
    """kubebuilder printcolumns shared by all kinds: State/Age/Finished-TTL/Max-Lifetime
    (``api/tensorflow/v1/types.go:28-31``)."""
    import time
    now_epoch = now_epoch if now_epoch is not None else time.time()
    st = job.get("status") or {}
    conds = st.get("conditions") or []
    state = conds[-1].get("type", "") if conds else ""
    created = c.to_epoch((job.get("metadata") or {}).get("creationTimestamp"))
    age = _human_duration(now_epoch - created) if created else ""
    spec = job.get("spec") or {}
    ttl = spec.get("ttlSecondsAfterFinished")
    dl = spec.get("activeDeadlineSeconds")
    return {"NAME": job["metadata"]["name"], "STATE": state, "AGE": age,
            "FINISHED-TTL": "" if ttl is None else str(ttl),
            "MAX-LIFETIME": "" if dl is None else str(dl)}


def _human_duration(s: float) -> str:
    s = max(0, int(s))
    if s < 120:
        return f"{s}s"
    m = s // 60
    if m < 120:
        return f"{m}m"
    h = m // 60
    if h < 48:
        return f"{h}h"
    return f"{h // 24}d"
