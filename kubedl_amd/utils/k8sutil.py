"""Pod / replica helpers over the object dicts of ``kubedl_amd.store``.

Reference: ``pkg/util/k8sutil/k8sutil.go:95-160``.  ``filter_active_pods`` and
``filter_pod_count`` are the engine's own (``engine/job_controller.py``),
re-exported here so every caller shares one definition.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from kubedl_amd.api import common as c
from kubedl_amd.engine.job_controller import filter_active_pods, filter_pod_count, pod_phase

__all__ = ["filter_active_pods", "filter_pod_count", "is_pod_active", "pod_phase", "get_total_replicas",
           "get_total_failed_replicas", "get_total_active_replicas", "resolve_dependent_owner",
           "get_replica_type"]


def is_pod_active(pod: dict) -> bool:
    """Not Succeeded, not Failed, not being deleted."""
    return pod_phase(pod) not in ("Succeeded", "Failed") and not (pod.get("metadata") or {}).get("deletionTimestamp")


def get_total_replicas(specs: Dict[str, dict]) -> int:
    return c.total_replicas(specs)


def _sum_status(statuses: Dict[str, Dict[str, int]], field: str) -> int:
    return sum(c.rs_get(rs, field) for rs in (statuses or {}).values())


def get_total_failed_replicas(statuses: Dict[str, Dict[str, int]]) -> int:
    return _sum_status(statuses, "failed")


def get_total_active_replicas(statuses: Dict[str, Dict[str, int]]) -> int:
    return _sum_status(statuses, "active")


def resolve_dependent_owner(obj: dict) -> Tuple[str, str]:
    """(uid, name) of the controller owner reference, or ("", "")."""
    for ref in (obj.get("metadata") or {}).get("ownerReferences") or []:
        if ref.get("controller"):
            return ref.get("uid", ""), ref.get("name", "")
    return "", ""


def get_replica_type(pod: dict) -> Optional[str]:
    """The ``replica-type`` label, or None."""
    return ((pod.get("metadata") or {}).get("labels") or {}).get(c.REPLICA_TYPE_LABEL)


def pods_by_replica_type(pods: List[dict], rtype: str) -> List[dict]:
    """Pods whose replica-type label matches (case-insensitively, as the engine keys replica types)."""
    want = rtype.lower()
    return [p for p in pods if (get_replica_type(p) or "").lower() == want]
