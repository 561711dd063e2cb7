"""Pod / Service control: the only write path of the job engine to the store.

``pkg/job_controller/pod_control.go:50-189`` and ``service_control.go:42-161``
wrap the API client so every create/delete emits the matching event and so
tests can swap in fakes (``service_control.go:163-234``).  Same here: the
``JobController`` never writes pods/services directly; it calls a
``PodControl`` / ``ServiceControl`` (real ones below, fakes in
``kubedl_amd.engine.testing``).

``ControllerRefManager`` is the adopt/release logic of
``service_ref_manager.go:30-158`` (a port of k8s ``PodControllerRefManager``)
applied to both kinds: an orphan whose labels match the job's selector is
adopted (owner reference patched in) unless the job is being deleted; an
object controlled by the job whose labels no longer match is released (its
controller reference removed).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

from kubedl_amd.store import NORMAL, WARNING, AlreadyExists, EventRecorder, NotFound, Store

SUCCESSFUL_CREATE_POD = "SuccessfulCreatePod"
FAILED_CREATE_POD = "FailedCreatePod"
SUCCESSFUL_DELETE_POD = "SuccessfulDeletePod"
FAILED_DELETE_POD = "FailedDeletePod"
SUCCESSFUL_CREATE_SERVICE = "SuccessfulCreateService"
FAILED_CREATE_SERVICE = "FailedCreateService"
SUCCESSFUL_DELETE_SERVICE = "SuccessfulDeleteService"
FAILED_DELETE_SERVICE = "FailedDeleteService"


class _ObjectControl:
    KIND = ""
    OK_CREATE = FAIL_CREATE = OK_DELETE = FAIL_DELETE = ""

    def __init__(self, store: Store, recorder: EventRecorder):
        self.store = store
        self.recorder = recorder

    def create(self, job: dict, obj: dict) -> dict:
        """Create ``obj`` (already carrying its owner reference); AlreadyExists
        propagates silently, any other error is recorded on the job."""
        try:
            out = self.store.create(obj)
        except AlreadyExists:
            raise
        except Exception as e:
            self.recorder.event(job, WARNING, self.FAIL_CREATE, f"Error creating: {e}")
            raise
        self.recorder.event(job, NORMAL, self.OK_CREATE,
                            f"Created {self.KIND.lower()}: {obj['metadata']['name']}")
        return out

    def delete(self, job: dict, namespace: str, name: str) -> None:
        """Delete; NotFound propagates (callers lower their expectations)."""
        try:
            self.store.delete(self.KIND, namespace, name)
        except NotFound:
            raise
        except Exception as e:
            self.recorder.event(job, WARNING, self.FAIL_DELETE, f"Error deleting: {e}")
            raise
        self.recorder.event(job, NORMAL, self.OK_DELETE, f"Deleted {self.KIND.lower()}: {name}")

    def patch(self, namespace: str, name: str, fn: Callable[[dict], None]) -> dict:
        return self.store.patch(self.KIND, namespace, name, fn)


class PodControl(_ObjectControl):
    KIND = "Pod"
    OK_CREATE, FAIL_CREATE = SUCCESSFUL_CREATE_POD, FAILED_CREATE_POD
    OK_DELETE, FAIL_DELETE = SUCCESSFUL_DELETE_POD, FAILED_DELETE_POD


class ServiceControl(_ObjectControl):
    KIND = "Service"
    OK_CREATE, FAIL_CREATE = SUCCESSFUL_CREATE_SERVICE, FAILED_CREATE_SERVICE
    OK_DELETE, FAIL_DELETE = SUCCESSFUL_DELETE_SERVICE, FAILED_DELETE_SERVICE


def controller_of(obj: dict) -> Optional[dict]:
    for ref in obj["metadata"].get("ownerReferences") or []:
        if ref.get("controller"):
            return ref
    return None


def _matches(labels: Dict[str, str], selector: Dict[str, str]) -> bool:
    return all(labels.get(k) == v for k, v in selector.items())


class ControllerRefManager:
    """Claim objects for a job: keep owned+matching, adopt matching orphans,
    release owned objects whose labels stopped matching."""

    def __init__(self, control: _ObjectControl, job: dict, selector: Dict[str, str],
                 owner_ref: dict):
        self.control = control
        self.job = job
        self.selector = selector
        self.owner_ref = owner_ref

    def claim(self, objs: List[dict]) -> List[dict]:
        uid = self.job["metadata"]["uid"]
        deleting = bool(self.job["metadata"].get("deletionTimestamp"))
        out = []
        for o in objs:
            ref = controller_of(o)
            md = o["metadata"]
            match = _matches(md.get("labels") or {}, self.selector)
            if ref is not None:
                if ref.get("uid") != uid:
                    continue  # someone else's
                if match:
                    out.append(o)
                elif not md.get("deletionTimestamp"):
                    self._release(o)
                continue
            if not match or deleting or md.get("deletionTimestamp"):
                continue
            adopted = self._adopt(o)
            if adopted is not None:
                out.append(adopted)
        return out

    def _adopt(self, o: dict) -> Optional[dict]:
        ref = dict(self.owner_ref)

        def add(obj):
            refs = obj["metadata"].setdefault("ownerReferences", [])
            if controller_of(obj) is None:
                refs.append(ref)
        try:
            return self.control.patch(o["metadata"]["namespace"], o["metadata"]["name"], add)
        except NotFound:
            return None

    def _release(self, o: dict) -> None:
        uid = self.job["metadata"]["uid"]

        def drop(obj):
            obj["metadata"]["ownerReferences"] = [r for r in obj["metadata"].get("ownerReferences") or []
                                                  if r.get("uid") != uid]
        try:
            self.control.patch(o["metadata"]["namespace"], o["metadata"]["name"], drop)
        except NotFound:
            pass
