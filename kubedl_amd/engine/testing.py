"""Test doubles for the job engine (``service_control.go:163-234``,
``test_job_controller.go:14-128``, ``pkg/test_job``, ``pkg/test_util``).

* ``FakePodControl`` / ``FakeServiceControl`` record every create/delete/patch
  instead of touching the store, with the reference's ``err`` injection and
  ``create_limit`` (create calls beyond the limit fail);
* ``TestWorkload`` is a minimal ``WorkloadController`` (``test-operator``,
  replica types Master/Worker, port ``default-port-name``/9999, no
  cluster-spec injection, status: Succeeded when every replica succeeded);
* ``new_test_job`` builds a TestJob-shaped object and ``new_job_controller``
  wires a ``JobController`` around fakes and an in-memory store.
"""
from __future__ import annotations

import copy
import threading
import uuid
from typing import Callable, Dict, List, Optional

from kubedl_amd.api import common as c
from kubedl_amd.engine.job_controller import JobController, JobControllerConfig, WorkloadController
from kubedl_amd.store import EventRecorder, NotFound, Store

TEST_GROUP = "test.kubedl.io"
TEST_KIND = "TestJob"


class _FakeControl:
    def __init__(self, store: Optional[Store] = None):
        self._lock = threading.Lock()
        self.store = store  # only used to serve patch() of adoption against real objects
        self.clear()

    def clear(self) -> None:
        with self._lock:
            self.templates: List[dict] = []
            self.controller_refs: List[dict] = []
            self.deleted: List[str] = []
            self.patches: List[str] = []
            self.err: Optional[Exception] = None
            self.create_limit = 0
            self.create_calls = 0

    def create(self, job: dict, obj: dict) -> dict:
        with self._lock:
            self.create_calls += 1
            if self.create_limit and self.create_calls > self.create_limit:
                raise RuntimeError(f"not creating {obj.get('kind', 'object').lower()}, limit {self.create_limit} "
                                   f"already reached (create call {self.create_calls})")
            self.templates.append(copy.deepcopy(obj))
            for ref in obj["metadata"].get("ownerReferences") or []:
                if ref.get("controller"):
                    self.controller_refs.append(dict(ref))
            if self.err is not None:
                raise self.err
            return obj

    def delete(self, job: dict, namespace: str, name: str) -> None:
        with self._lock:
            self.deleted.append(name)
            if self.err is not None:
                raise self.err

    def patch(self, namespace: str, name: str, fn: Callable[[dict], None]) -> dict:
        with self._lock:
            self.patches.append(f"{namespace}/{name}")
            if self.err is not None:
                raise self.err
        if self.store is None:
            raise NotFound(f"{namespace}/{name}")
        return self.store.patch(self.KIND, namespace, name, fn)


class FakePodControl(_FakeControl):
    KIND = "Pod"


class FakeServiceControl(_FakeControl):
    KIND = "Service"


class TestWorkload(WorkloadController):
    __test__ = False  # not a pytest class

    def controller_name(self) -> str:
        return "test-operator"

    def get_api_group_version_kind(self):
        return TEST_GROUP, "v1", TEST_KIND

    def get_group_name_label_value(self) -> str:
        return TEST_GROUP

    def get_default_container_name(self) -> str:
        return "default-container"

    def get_default_container_port_name(self) -> str:
        return "default-port-name"

    def get_default_container_port_number(self) -> int:
        return 9999

    def get_reconcile_orders(self):
        return ("Master", "Worker")

    def is_master_role(self, replicas, rtype, index) -> bool:
        return rtype == "Master"

    def set_cluster_spec(self, job, pod_template, rtype, index) -> None:
        return None

    def update_job_status(self, job, replicas, status, restart) -> None:
        done = all(c.rs_get((status.get("replicaStatuses") or {}).get(rt) or {}, "succeeded") == c.replicas_of(spec)
                   for rt, spec in replicas.items())
        if done:
            c.update_job_conditions(status, c.JOB_SUCCEEDED, c.JOB_SUCCEEDED_REASON, "done")
        else:
            c.update_job_conditions(status, c.JOB_RUNNING, c.JOB_RUNNING_REASON, "running")


def new_test_job(name: str = "test-job", namespace: str = "default", workers: int = 1, master: bool = True,
                 restart_policy: str = c.RESTART_POLICY_NEVER) -> dict:
    """``pkg/test_job/v1``-shaped job: Master (optional) + ``workers`` Workers."""
    def rs(n):
        return {"replicas": n, "restartPolicy": restart_policy, "template": {"spec": {"containers": [
            {"name": "default-container", "image": "test-image",
             "ports": [{"name": "default-port-name", "containerPort": 9999}]}]}}}
    specs: Dict[str, dict] = {}
    if master:
        specs["Master"] = rs(1)
    if workers:
        specs["Worker"] = rs(workers)
    return {"apiVersion": f"{TEST_GROUP}/v1", "kind": TEST_KIND,
            "metadata": {"name": name, "namespace": namespace, "uid": str(uuid.uuid4())},
            "spec": {"testReplicaSpecs": specs}, "status": {"conditions": [], "replicaStatuses": {}}}


def new_job_controller(store: Optional[Store] = None, config: Optional[JobControllerConfig] = None,
                       metrics=None):
    """(JobController, FakePodControl, FakeServiceControl) around an in-memory store."""
    store = store or Store()
    rec = EventRecorder(store, "test-operator")
    pods, svcs = FakePodControl(store), FakeServiceControl(store)
    jc = JobController(TestWorkload(), store, rec, metrics, config=config, pod_control=pods, service_control=svcs)
    return jc, pods, svcs
