"""Shared reconciler scaffold for the four workload controllers.

Every reference controller (``controllers/<fw>/<fw>job_controller.go``) has
the same shape, reproduced once here:

1. ``on_owner_create`` (the create predicate, e.g.
   ``controllers/tensorflow/status.go:33-53``): default the job, append the
   ``Created`` condition, bump ``kubedl_jobs_created``.  [NEW] the condition
   is written to the store at submission instead of mutating a cache copy.
2. ``reconcile(key)``: get the job (NotFound => ``kubedl_jobs_deleted``++
   and expectation cleanup), deep copy, gate on ``SatisfyExpectations``,
   apply defaults, ``ReconcileJobs``.
3. Pod/Service watch predicates resolve the owning job, mark expectations
   observed and enqueue it (``pkg/job_controller/pod.go:53-163``,
   ``service.go:39-137``).
"""
from __future__ import annotations

import copy
import logging
from typing import Dict, Optional

from kubedl_amd.api import common as c
from kubedl_amd.api import kinds as K
from kubedl_amd.engine.job_controller import (JobController, JobControllerConfig, ReconcileResult,
                                              WorkloadController, controller_of)
from kubedl_amd.store import ADDED, DELETED, MODIFIED, NotFound

log = logging.getLogger("kubedl_amd.controllers")


class BaseReconciler(WorkloadController):
    info: K.KindInfo
    # [NEW] ranks share one communicator (RCCL / gloo / rabit / XDL's PS mesh):
    # a retryable failure of one restarts the whole gang (JobController.restart_gang)
    collective: bool = False

    def __init__(self, store, recorder, metrics_registry, config: Optional[JobControllerConfig] = None,
                 gang=None):
        self.store = store
        self.recorder = recorder
        self.metrics = metrics_registry.job_metrics(self.info.kind)
        self.ctrl = JobController(self, store, recorder, self.metrics, config, gang)

    # ------------------------------------------------------------ helpers
    @property
    def kind(self) -> str:
        return self.info.kind

    def replica_specs(self, job: dict) -> Dict[str, dict]:
        return K.replica_specs(job)

    def get_pods_for_job(self, job: dict):
        return self.ctrl.get_pods_for_job(job)

    # ------------------------------------------------------------ create predicate
    def on_owner_create(self, job: dict) -> bool:
        st = (job.get("status") or {})
        if c.has_condition(st, c.JOB_CREATED):
            return True
        job = copy.deepcopy(job)
        K.set_defaults(job)
        status = c.ensure_status(job)
        msg = f"{self.created_msg_kind()} {job['metadata']['name']} is created."
        c.update_job_conditions(status, c.JOB_CREATED, c.JOB_CREATED_REASON, msg)
        try:
            self.store.update_status(job)
        except NotFound:
            return False
        log.info(msg)
        self.metrics.created_inc()
        return True

    def created_msg_kind(self) -> str:
        return self.kind

    def restart_whole_gang(self, replicas) -> bool:
        return self.collective and c.total_replicas(replicas) > 1

    # ------------------------------------------------------------ reconcile
    def reconcile(self, namespace: str, name: str) -> ReconcileResult:
        try:
            shared = self.store.get(self.kind, namespace, name)
        except NotFound:
            log.info("%s %s/%s has been deleted", self.kind, namespace, name)
            self.metrics.deleted_inc()
            self.ctrl.expectations.delete_prefix(f"{namespace}/{name}/")
            return ReconcileResult()
        job = copy.deepcopy(shared)
        if not self.ctrl.satisfy_expectations(job):
            log.debug("expectations not satisfied for %s/%s", namespace, name)
            return ReconcileResult()
        K.set_defaults(job)
        status = c.ensure_status(job)
        return self.ctrl.reconcile_jobs(job, self.replica_specs(job), status, K.run_policy(job))

    # ------------------------------------------------------------ watch predicates
    def owner_of(self, obj: dict) -> Optional[dict]:
        ref = controller_of(obj)
        if ref is None or ref.get("kind") != self.kind:
            return None
        ns = obj["metadata"].get("namespace", "default")
        job = self.store.try_get(self.kind, ns, ref.get("name"))
        if job is None or job["metadata"].get("uid") != ref.get("uid"):
            return None
        return job

    def on_dependent_event(self, etype: str, obj: dict) -> Optional[str]:
        """Return the owning job's ``ns/name`` to enqueue, after updating expectations."""
        ref = controller_of(obj)
        if ref is None or ref.get("kind") != self.kind:
            return None
        ns = obj["metadata"].get("namespace", "default")
        key = f"{ns}/{ref.get('name')}"
        rtype = (obj["metadata"].get("labels") or {}).get(c.REPLICA_TYPE_LABEL)
        if rtype is None:
            return None
        what = "pods" if obj["kind"] == "Pod" else "services"
        exp_key = f"{key}/{rtype}/{what}"
        if etype == ADDED:
            if obj["metadata"].get("deletionTimestamp"):
                return None
            self.ctrl.expectations.creation_observed(exp_key)
        elif etype == DELETED:
            self.ctrl.expectations.deletion_observed(exp_key)
        elif etype != MODIFIED:
            return None
        return key

    # ------------------------------------------------------------ status helpers
    def _set_completion(self, status: dict) -> None:
        if not status.get("completionTime"):
            status["completionTime"] = c.now()

    def _failed_or_restarting(self, job: dict, status: dict, rtype: str, failed: int, restart: bool,
                              prev_restarting: bool, prev_failed: bool, display: str) -> None:
        name = job["metadata"]["name"]
        # The reference captures previousRestarting/previousFailed once per pass,
        # so two replica types failing in the same pass count the job twice
        # (found by tests/test_stress.py).  Here the transition is counted once:
        # "already" also covers an earlier replica type of this pass.
        if restart:
            msg = f"{display} {name} is restarting because {failed} {rtype} replica(s) failed."
            self.recorder.event(job, "Warning", c.JOB_RESTARTING_REASON, msg)
            already = prev_restarting or c.is_restarting(status)
            c.update_job_conditions(status, c.JOB_RESTARTING, c.JOB_RESTARTING_REASON, msg)
            if not already:
                self.metrics.failure_inc()
                self.metrics.restart_inc()
        else:
            msg = f"{display} {name} is failed because {failed} {rtype} replica(s) failed."
            self.recorder.event(job, "Normal", c.JOB_FAILED_REASON, msg)
            self._set_completion(status)
            already = prev_failed or c.is_failed(status)
            c.update_job_conditions(status, c.JOB_FAILED, c.JOB_FAILED_REASON, msg)
            if not already:
                self.metrics.failure_inc()

    def _succeeded(self, job: dict, status: dict, msg: str) -> None:
        self.recorder.event(job, "Normal", c.JOB_SUCCEEDED_REASON, msg)
        self._set_completion(status)
        already = c.is_succeeded(status)
        c.update_job_conditions(status, c.JOB_SUCCEEDED, c.JOB_SUCCEEDED_REASON, msg)
        if not already:
            # the reference increments on every pass that sees success; count
            # the transition once so the counter means "jobs", not "passes"
            self.metrics.success_inc()

    # ------------------------------------------------------------ cluster-spec helpers
    @staticmethod
    def _append_env(container: dict, name: str, value: str) -> None:
        container.setdefault("env", []).append({"name": name, "value": value})
