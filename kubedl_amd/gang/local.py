"""Local gang scheduler: PodGroup objects + all-or-nothing GPU admission.

``create_gang`` mirrors kube-batch's ``CreateGang``
(``pkg/gang_schedule/batch_scheduler/scheduler.go:38-119``): a ``PodGroup``
named after the job, owned by it, with ``minMember = sum(replicas)`` (the
reference ignores ``schedulingPolicy.minAvailable``; so do we).
``bind_pod_to_gang`` sets ``spec.schedulerName`` and the
``scheduling.k8s.io/group-name`` annotation; the node scheduler
(``kubedl_amd.runtime.scheduler``) then admits the group only when all
``minMember`` pods exist and their GPUs can be reserved together.
"""
from __future__ import annotations

from typing import Dict, Optional

from kubedl_amd.api import common as c
from kubedl_amd.gang import interface
from kubedl_amd.store import AlreadyExists, NotFound

GROUP_ANNOTATION = "scheduling.k8s.io/group-name"
PODGROUP_API = "scheduling.incubator.k8s.io/v1alpha1"


class LocalGangScheduler(interface.GangScheduler):
    NAME = "kdl-gang"

    def __init__(self, store, name: Optional[str] = None, **_):
        self.store = store
        self._name = name or self.NAME

    def name(self) -> str:
        return self._name

    def create_gang(self, job: dict, replicas: Dict[str, dict]) -> dict:
        md = job["metadata"]
        pg = self.get_gang(md["namespace"], md["name"])
        if pg is not None:
            return pg
        min_member = c.total_replicas(replicas)
        gpus = sum(c.replicas_of(s) * c.pod_template_gpus(s.get("template") or {})
                   for s in replicas.values())
        obj = {
            "apiVersion": PODGROUP_API, "kind": "PodGroup",
            "metadata": {"name": md["name"], "namespace": md["namespace"],
                         "ownerReferences": [_owner_ref(job)]},
            "spec": {"minMember": min_member, "minResources": {"amd.com/gpu": gpus}},
            "status": {"phase": "Pending"},
        }
        try:
            return self.store.create(obj)
        except AlreadyExists:
            return self.store.get("PodGroup", md["namespace"], md["name"])

    def bind_pod_to_gang(self, pod_template: dict, entity: dict) -> None:
        spec = pod_template.setdefault("spec", {})
        spec["schedulerName"] = self._name
        md = pod_template.setdefault("metadata", {})
        md.setdefault("annotations", {})[GROUP_ANNOTATION] = entity["metadata"]["name"]

    def get_gang(self, namespace: str, name: str) -> Optional[dict]:
        return self.store.try_get("PodGroup", namespace, name)

    def delete_gang(self, namespace: str, name: str) -> None:
        try:
            self.store.delete("PodGroup", namespace, name)
        except NotFound:
            pass  # tolerated, like the reference


def _owner_ref(job: dict) -> dict:
    md = job["metadata"]
    return {"apiVersion": job["apiVersion"], "kind": job["kind"], "name": md["name"],
            "uid": md["uid"], "controller": True, "blockOwnerDeletion": True}


interface.register(LocalGangScheduler.NAME, lambda store, **kw: LocalGangScheduler(store, **kw))
# accept the reference's scheduler name so `--gang-scheduler-name=kube-batch` works unchanged
interface.register("kube-batch", lambda store, **kw: LocalGangScheduler(store, name="kube-batch", **kw))
