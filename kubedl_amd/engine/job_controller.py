"""The common job engine (``pkg/job_controller``): ``ReconcileJobs`` and the
pod/service reconcilers shared by every workload kind.

A ``WorkloadController`` (``kubedl_amd.controllers.*``) supplies the
per-framework parts -- the ``ControllerInterface`` of the reference
(``pkg/job_controller/api/v1/interface.go:10-76``): cluster-spec injection,
status state machine, reconcile order, master role, default container/port.

Faithful to the reference (``pkg/job_controller/job.go:56-345``,
``pod.go:212-442``, ``service.go:188-330``):

* backoff: ``exceedsBackoffLimit`` (a new failure while not all replicas are
  active and ``previousRetry + 1 > backoffLimit``, previousRetry = the work
  queue's requeue count) or ``pastBackoffLimit`` (sum of restartCounts over
  RUNNING pods of OnFailure/Always replica types; limit 0 => any restart);
* ``activeDeadlineSeconds`` measured from ``status.startTime``;
* terminal jobs: pods/services cleaned per ``cleanPodPolicy`` (None keeps all,
  Running deletes only Running pods, All deletes all), TTL cleanup deletes
  the job ``ttlSecondsAfterFinished`` after ``completionTime`` (else requeue
  after the remainder), gang deleted, Failed condition appended when a limit
  was exceeded, active counts folded into succeeded on success;
* pods are named ``<job>-<rtype>-<index>`` with labels group-name/job-name/
  replica-type/replica-index (+ job-role=master), the ExitCode restart policy
  becomes pod restartPolicy Never, and a Failed pod with a retryable exit code
  (``common.is_retryable_exit_code``) of an ExitCode replica is deleted and
  recreated (``restart=True`` -> Restarting condition);
* one headless Service per replica index (PyTorch: Master only);
* launch-delay metrics: first-pod on Created->Running, all-pods when the
  active count first reaches the total and the job was not Restarting.
"""
from __future__ import annotations

import copy
import logging
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from kubedl_amd.api import common as c
from kubedl_amd.api import kinds as K
from kubedl_amd import code_sync
from kubedl_amd.engine.control import (ControllerRefManager, PodControl, ServiceControl,  # noqa: F401
                                       controller_of)
from kubedl_amd.engine.expectations import Expectations
from kubedl_amd.engine.workqueue import RateLimitingQueue
from kubedl_amd.store import NORMAL, WARNING, AlreadyExists, EventRecorder, NotFound, Store

log = logging.getLogger("kubedl_amd.engine")

from kubedl_amd.utils.log import logger_for_job, logger_for_replica  # noqa: E402

# event reasons (pkg/job_controller/pod_control.go, service_control.go, pod.go)
from kubedl_amd.engine.control import (FAILED_CREATE_POD, FAILED_CREATE_SERVICE, FAILED_DELETE_POD,  # noqa: F401,E402
                                       SUCCESSFUL_CREATE_POD, SUCCESSFUL_CREATE_SERVICE,
                                       SUCCESSFUL_DELETE_POD, SUCCESSFUL_DELETE_SERVICE)
EXITED_WITH_CODE = "ExitedWithCode"
POD_TEMPLATE_RESTART_POLICY = "SettedPodTemplateRestartPolicy"
EXIT_CODE_SENTINEL = 0xBEEF


@dataclass
class ReconcileResult:
    requeue: bool = False
    requeue_after: float = 0.0


@dataclass
class JobControllerConfig:
    enable_gang_scheduling: bool = False
    gang_scheduler_name: str = ""
    max_concurrent_reconciles: int = 1
    # declared but unused by the reference (job_controller.go:36-42); kept for parity
    reconciler_sync_loop_period: float = 0.0


def job_key(job: dict) -> str:
    md = job["metadata"]
    return f"{md['namespace']}/{md['name']}"


def gen_owner_reference(job: dict) -> dict:
    """GenOwnerReference: controller=true, blockOwnerDeletion=true."""
    md = job["metadata"]
    return {"apiVersion": job["apiVersion"], "kind": job["kind"], "name": md["name"],
            "uid": md["uid"], "controller": True, "blockOwnerDeletion": True}


def pod_phase(pod: dict) -> str:
    return (pod.get("status") or {}).get("phase", "Pending") or "Pending"


def filter_active_pods(pods: List[dict]) -> List[dict]:
    """k8sutil.FilterActivePods: not Succeeded, not Failed, not being deleted."""
    return [p for p in pods if pod_phase(p) not in ("Succeeded", "Failed")
            and not p["metadata"].get("deletionTimestamp")]


def filter_pod_count(pods: List[dict], phase: str) -> int:
    return sum(1 for p in pods if pod_phase(p) == phase)


class WorkloadController:
    """The ControllerInterface each workload kind implements."""

    info: K.KindInfo

    def controller_name(self) -> str:
        return f"{self.info.kind}Controller"

    def get_api_group_version_kind(self) -> Tuple[str, str, str]:
        return self.info.group, self.info.version, self.info.kind

    def get_group_name_label_value(self) -> str:
        return self.info.group_label

    def get_default_container_name(self) -> str:
        return self.info.default_container

    def get_default_container_port_name(self) -> str:
        return self.info.default_port_name

    def get_default_container_port_number(self) -> int:
        return self.info.default_port

    def get_reconcile_orders(self) -> Tuple[str, ...]:
        return self.info.reconcile_order

    def is_master_role(self, replicas: Dict[str, dict], rtype: str, index: int) -> bool:
        return False

    def set_cluster_spec(self, job: dict, pod_template: dict, rtype: str, index: str) -> None:
        raise NotImplementedError

    def update_job_status(self, job: dict, replicas: Dict[str, dict], status: dict,
                          restart: bool) -> None:
        raise NotImplementedError

    def reconcile_services_for(self, rtype: str) -> bool:
        """Whether ReconcileServices runs for this replica type (PyTorch: Master only)."""
        return True

    def restart_whole_gang(self, replicas: Dict[str, dict]) -> bool:
        """[NEW] Whether a retryable failure of one replica restarts EVERY pod of
        the job.  True for collective jobs (the ranks share an RCCL/gloo
        communicator, which cannot survive a dead peer: the survivors would
        block in their next collective until the process-group timeout);
        False keeps the reference's per-pod restart (``pod.go:281-307``)."""
        return False


class JobController:
    def __init__(self, controller: WorkloadController, store: Store, recorder: EventRecorder,
                 metrics, config: Optional[JobControllerConfig] = None, gang=None,
                 queue: Optional[RateLimitingQueue] = None, pod_control=None, service_control=None):
        self.controller = controller
        self.store = store
        self.recorder = recorder
        self.pod_control = pod_control or PodControl(store, recorder)
        self.service_control = service_control or ServiceControl(store, recorder)
        self.metrics = metrics
        self.config = config or JobControllerConfig()
        self.gang = gang
        self.expectations = Expectations()
        # BackoffStatesQueue: only used to count retries per job (job.go:78-88,119)
        self.backoff_queue = queue or RateLimitingQueue()
        self._lock = threading.Lock()
        self._launch_marks: Dict[str, set] = {}

    # ------------------------------------------------------------ labels/names
    def gen_labels(self, job_name: str) -> Dict[str, str]:
        return {c.GROUP_NAME_LABEL: self.controller.get_group_name_label_value(),
                c.JOB_NAME_LABEL: job_name.replace("/", "-")}

    def expectation_keys(self, job: dict) -> List[str]:
        key = job_key(job)
        out = []
        for rtype in K.replica_specs(job):
            out.append(c.gen_expectation_pods_key(key, rtype))
            out.append(c.gen_expectation_services_key(key, rtype))
        return out

    def satisfy_expectations(self, job: dict) -> bool:
        return self.expectations.satisfied(self.expectation_keys(job))

    # ------------------------------------------------------------ object access
    def get_pods_for_job(self, job: dict) -> List[dict]:
        """List by label selector, then claim (keep owned, adopt orphans)."""
        md = job["metadata"]
        sel = self.gen_labels(md["name"])
        pods = self.store.list("Pod", md["namespace"], sel)
        return ControllerRefManager(self.pod_control, job, sel, gen_owner_reference(job)).claim(pods)

    def get_services_for_job(self, job: dict) -> List[dict]:
        md = job["metadata"]
        sel = self.gen_labels(md["name"])
        svcs = self.store.list("Service", md["namespace"], sel)
        return ControllerRefManager(self.service_control, job, sel, gen_owner_reference(job)).claim(svcs)

    @staticmethod
    def filter_for_replica_type(objs: List[dict], rt: str) -> List[dict]:
        return [o for o in objs if (o["metadata"].get("labels") or {}).get(c.REPLICA_TYPE_LABEL) == rt]

    @staticmethod
    def get_slices(objs: List[dict], replicas: int) -> List[List[dict]]:
        """GetPodSlices / GetServiceSlices: bucket by replica-index label."""
        slices: List[List[dict]] = [[] for _ in range(replicas)]
        for o in objs:
            idx = (o["metadata"].get("labels") or {}).get(c.REPLICA_INDEX_LABEL)
            if idx is None:
                log.warning("object %s has no index label", o["metadata"]["name"])
                continue
            try:
                i = int(idx)
            except ValueError:
                log.warning("bad index label on %s", o["metadata"]["name"])
                continue
            if 0 <= i < replicas:
                slices[i].append(o)
            else:
                log.warning("unexpected index label %d on %s", i, o["metadata"]["name"])
        return slices

    # ------------------------------------------------------------ gang glue
    def create_gang(self, job: dict, replicas: Dict[str, dict]):
        return self.gang.create_gang(job, replicas)

    def delete_gang(self, job: dict) -> None:
        md = job["metadata"]
        self.gang.delete_gang(md["namespace"], md["name"])

    # ------------------------------------------------------------ pod/service control
    def create_pod(self, job: dict, pod: dict) -> dict:
        return self.pod_control.create(job, pod)

    def delete_pod(self, job: dict, pod: dict) -> None:
        md = pod["metadata"]
        rt = (md.get("labels") or {}).get(c.REPLICA_TYPE_LABEL, "")
        key = c.gen_expectation_pods_key(job_key(job), rt)
        self.expectations.expect_deletions(key, 1)
        try:
            self.pod_control.delete(job, md["namespace"], md["name"])
        except NotFound:
            self.expectations.deletion_observed(key)
        except Exception:
            self.expectations.deletion_observed(key)
            raise

    def delete_service(self, job: dict, name: str, namespace: str) -> None:
        try:
            svc = self.store.get("Service", namespace, name)
        except NotFound:
            return
        rt = (svc["metadata"].get("labels") or {}).get(c.REPLICA_TYPE_LABEL, "")
        key = c.gen_expectation_services_key(job_key(job), rt)
        self.expectations.expect_deletions(key, 1)
        try:
            self.service_control.delete(job, namespace, name)
        except NotFound:
            self.expectations.deletion_observed(key)
        except Exception:
            self.expectations.deletion_observed(key)
            raise

    def update_job_status_in_store(self, job: dict, status: dict) -> dict:
        cur = copy.deepcopy(job)
        cur["status"] = status
        return self.store.update_status(cur)

    def delete_job(self, job: dict) -> None:
        md = job["metadata"]
        try:
            self.store.delete(job["kind"], md["namespace"], md["name"])
        except NotFound:
            return
        self.recorder.event(job, NORMAL, "SuccessfulDeleteJob", f"Deleted job: {md['name']}")

    # ------------------------------------------------------------ ReconcileJobs
    def reconcile_jobs(self, job: dict, replicas: Dict[str, dict], job_status: dict,
                       run_policy: dict) -> ReconcileResult:
        key = job_key(job)
        job_name = job["metadata"]["name"]
        result = ReconcileResult()
        err: Optional[BaseException] = None
        try:
            result = self._reconcile_jobs(job, replicas, job_status, run_policy, key, job_name)
            return result
        except BaseException as e:
            err = e
            raise
        finally:
            if result.requeue or err is not None:
                self.backoff_queue.when(key)  # AddRateLimited: counts the retry
            else:
                self.backoff_queue.forget(key)

    def _reconcile_jobs(self, job, replicas, job_status, run_policy, key, job_name) -> ReconcileResult:
        result = ReconcileResult()
        if self.config.enable_gang_scheduling and self.gang is not None:
            self.create_gang(job, replicas)

        old_status = copy.deepcopy(job_status)
        code_sync.inject_code_sync_init_containers(job["metadata"], replicas)

        pods = self.get_pods_for_job(job)
        services = self.get_services_for_job(job)

        previous_retry = self.backoff_queue.num_requeues(key)
        active_pods = filter_active_pods(pods)
        active = len(active_pods)
        failed = filter_pod_count(pods, "Failed")
        total_replicas = c.total_replicas(replicas)
        prev_failed = c.total_failed(job_status.get("replicaStatuses"))

        failure_message = ""
        job_exceeds_limit = False
        exceeds_backoff = past_backoff = False
        if run_policy.get("backoffLimit") is not None:
            limit = int(run_policy["backoffLimit"])
            has_new_failure = failed > prev_failed
            exceeds_backoff = has_new_failure and (active != total_replicas) and (previous_retry + 1 > limit)
            past_backoff = self.past_backoff_limit(job_name, run_policy, replicas, pods)
        if exceeds_backoff or past_backoff:
            job_exceeds_limit = True
            failure_message = f"Job {job_name} has failed because it has reached the specified backoff limit"
        elif self.past_active_deadline(run_policy, job_status):
            failure_message = f"Job {job_name} has failed because it was active longer than specified deadline"
            job_exceeds_limit = True
            job_status["completionTime"] = c.now()

        if c.is_succeeded(job_status) or c.is_failed(job_status) or job_exceeds_limit:
            self.delete_pods_and_services(run_policy, job, pods)
            result = self.cleanup_job(run_policy, job_status, job)
            if self.config.enable_gang_scheduling and self.gang is not None:
                self.recorder.event(job, NORMAL, "JobTerminated", "Job has been terminated. Deleting PodGroup")
                self.delete_gang(job)
                self.recorder.event(job, NORMAL, "SuccessfulDeletePodGroup", f"Deleted PodGroup: {job_name}")
            if job_exceeds_limit:
                self.recorder.event(job, NORMAL, c.JOB_FAILED_REASON, failure_message)
                if not job_status.get("completionTime"):
                    job_status["completionTime"] = c.now()
                c.update_job_conditions(job_status, c.JOB_FAILED, c.JOB_FAILED_REASON, failure_message)
            if c.is_succeeded(job_status):
                for rs in (job_status.get("replicaStatuses") or {}).values():
                    c.rs_set(rs, "succeeded", c.rs_get(rs, "succeeded") + c.rs_get(rs, "active"))
                    c.rs_set(rs, "active", 0)
            if old_status != job_status:
                self.update_job_status_in_store(job, job_status)
            return result

        restart = [False]
        deleted: set = set()
        for rtype in self.controller.get_reconcile_orders():
            spec = replicas.get(rtype)
            if spec is None:
                continue
            self.reconcile_pods(job, job_status, pods, rtype, spec, replicas, restart, deleted)
            if not self.controller.reconcile_services_for(rtype):
                continue
            self.reconcile_services(job, services, rtype, spec)
        if deleted and self.controller.restart_whole_gang(replicas):
            self.restart_gang(job, pods, deleted)

        self.controller.update_job_status(job, replicas, job_status, restart[0])

        # Launch-delay metrics (job.go:242-259).  The reference observes on the
        # Created->Running / all-active transitions and reads whatever PodReady
        # condition exists; a rank here becomes Ready only once its process
        # group is up, which can be after the phase flips, so each histogram is
        # observed exactly once per job, on the first reconcile where its
        # condition holds with Ready=True pods (never after a Restarting phase
        # for all-pods, as in the reference).
        uid = job["metadata"].get("uid")
        marks = self._launch_marks.setdefault(uid, set())
        if "first" not in marks and c.is_created(job_status) and (
                c.is_running(job_status) or c.is_succeeded(job_status)):
            # every pod of the job, not only active ones: a short rank may already
            # have finished (its readyTime survives) when the job first reads Running
            if self.metrics.first_pod_launch_delay(pods, job, job_status) is not None:
                marks.add("first")
        if "all" not in marks and not c.is_restarting(old_status) and not c.is_restarting(job_status):
            if c.total_active(job_status.get("replicaStatuses")) == total_replicas:
                if self.metrics.all_pods_launch_delay(self.get_pods_for_job(job), job, job_status) is not None:
                    marks.add("all")
        elif c.is_restarting(job_status):
            marks.add("all")

        if old_status != job_status:
            self.update_job_status_in_store(job, job_status)
        # [NEW] wake up when the active deadline expires (the reference only
        # notices a passed deadline on the next pod/job event)
        dl = run_policy.get("activeDeadlineSeconds")
        st = c.to_epoch(job_status.get("startTime"))
        if dl is not None and st is not None:
            result.requeue_after = max(0.01, st + float(dl) - time.time())
        return result

    # ------------------------------------------------------------ limits
    def past_active_deadline(self, run_policy: dict, status: dict) -> bool:
        dl = run_policy.get("activeDeadlineSeconds")
        st = c.to_epoch(status.get("startTime"))
        if dl is None or st is None:
            return False
        return time.time() - st >= float(dl)

    def past_backoff_limit(self, job_name: str, run_policy: dict, replicas: Dict[str, dict],
                           pods: List[dict]) -> bool:
        limit = run_policy.get("backoffLimit")
        if limit is None:
            return False
        total = 0
        for rtype, spec in replicas.items():
            if spec.get("restartPolicy") not in (c.RESTART_POLICY_ON_FAILURE, c.RESTART_POLICY_ALWAYS):
                continue
            for p in self.filter_for_replica_type(pods, rtype.lower()):
                if pod_phase(p) != "Running":
                    continue
                st = p.get("status") or {}
                for cs in (st.get("initContainerStatuses") or []) + (st.get("containerStatuses") or []):
                    total += int(cs.get("restartCount", 0))
        if int(limit) == 0:
            return total > 0
        return total >= int(limit)

    def cleanup_job(self, run_policy: dict, status: dict, job: dict) -> ReconcileResult:
        ttl = run_policy.get("ttlSecondsAfterFinished")
        if ttl is None:
            return ReconcileResult()
        ct = c.to_epoch(status.get("completionTime"))
        if ct is None:
            raise RuntimeError(f"cleanup Job {job['metadata']['name']}, but job has CompletionTime not set")
        delete_at = ct + float(ttl)
        now = time.time()
        if now > delete_at:
            self.delete_job(job)
            return ReconcileResult()
        return ReconcileResult(requeue=True, requeue_after=delete_at - now)

    def delete_pods_and_services(self, run_policy: dict, job: dict, pods: List[dict]) -> None:
        if not pods:
            return
        policy = run_policy.get("cleanPodPolicy", c.CLEAN_POD_POLICY_UNDEFINED)
        if policy == c.CLEAN_POD_POLICY_NONE:
            return
        for p in pods:
            if policy == c.CLEAN_POD_POLICY_RUNNING and pod_phase(p) != "Running":
                continue
            self.delete_pod(job, p)
            self.delete_service(job, p["metadata"]["name"], p["metadata"]["namespace"])

    # ------------------------------------------------------------ pods
    def restart_gang(self, job: dict, pods: List[dict], deleted: set) -> None:
        """[NEW] Gang-wide teardown for collective jobs (failure
        detection): a retryable failure of one rank deletes every other pod of
        the job as well, so all ranks are recreated together and rendezvous
        afresh (resuming from the job's checkpoint) instead of the survivors
        hanging in a collective with a dead peer.  The kubelet starts the new
        pods only after the old rank processes have exited and the scheduler
        returns the old pods' GPUs only then, so the gang's re-admission is
        all-or-nothing against exactly the GPUs it held."""
        others = [p for p in pods if p["metadata"]["name"] not in deleted
                  and not p["metadata"].get("deletionTimestamp")]
        if not others:
            return
        # A peer that failed with a PERMANENT code in the same pass keeps its pod
        # (and its failure record): no teardown, so the next reconcile fails the
        # job exactly as the reference's per-pod ExitCode handling would.
        # Succeeded peers ARE recreated: restarted ranks cannot rendezvous
        # without them, and they resume from the job's checkpoint.
        dc = self.controller.get_default_container_name()
        for p in others:
            if pod_phase(p) != "Failed":
                continue
            code = next((int(((cs.get("state") or {}).get("terminated") or {}).get("exitCode", 0))
                         for cs in (p.get("status") or {}).get("containerStatuses") or []
                         if cs.get("name") == dc and (cs.get("state") or {}).get("terminated") is not None),
                        EXIT_CODE_SENTINEL)
            if not c.is_retryable_exit_code(code):
                logger_for_job(job, log).info("no gang restart: %s failed permanently (exit %d)",
                                              p["metadata"]["name"], code)
                return
        msg = (f"Restarting all {len(others) + len(deleted)} ranks of {job['metadata']['name']}: "
               f"{', '.join(sorted(deleted))} failed with a retryable exit code")
        logger_for_job(job, log).info(msg)
        self.recorder.event(job, NORMAL, "GangRestart", msg)
        for p in others:
            try:
                self.delete_pod(job, p)
            except NotFound:
                pass

    def reconcile_pods(self, job: dict, job_status: dict, pods: List[dict], rtype: str, spec: dict,
                       replicas: Dict[str, dict], restart: List[bool], deleted: Optional[set] = None) -> None:
        rt = rtype.lower()
        rlog = logger_for_replica(job, rt, log)
        pods = self.filter_for_replica_type(pods, rt)
        num = c.replicas_of(spec)
        # initializeReplicaStatuses: reset this type's counts every pass
        job_status.setdefault("replicaStatuses", {})[rtype] = {}
        rs = job_status["replicaStatuses"][rtype]
        for index, sl in enumerate(self.get_slices(pods, num)):
            if len(sl) > 1:
                rlog.warning("too many pods for %s %d", rt, index)
            elif len(sl) == 0:
                master = self.controller.is_master_role(replicas, rtype, index)
                try:
                    self.create_new_pod(job, rt, str(index), spec, master, replicas)
                except AlreadyExists:
                    key = job_key(job)
                    self.expectations.creation_observed(c.gen_expectation_pods_key(key, rt))
                    self.expectations.creation_observed(c.gen_expectation_services_key(key, rt))
                    raise
            else:
                pod = sl[0]
                exit_code = EXIT_CODE_SENTINEL
                for cs in (pod.get("status") or {}).get("containerStatuses") or []:
                    term = (cs.get("state") or {}).get("terminated")
                    if cs.get("name") == self.controller.get_default_container_name() and term is not None:
                        exit_code = int(term.get("exitCode", 0))
                        self.recorder.event(job, NORMAL, EXITED_WITH_CODE,
                                            f"Pod: {pod['metadata']['namespace']}.{pod['metadata']['name']} "
                                            f"exited with code {exit_code}")
                        break
                if spec.get("restartPolicy") == c.RESTART_POLICY_EXIT_CODE:
                    if pod_phase(pod) == "Failed" and c.is_retryable_exit_code(exit_code):
                        rlog.info("need to restart pod %s", pod["metadata"]["name"])
                        self.delete_pod(job, pod)
                        restart[0] = True
                        if deleted is not None:
                            deleted.add(pod["metadata"]["name"])
                phase = pod_phase(pod)
                if phase == "Running":
                    c.rs_inc(rs, "active")
                elif phase == "Succeeded":
                    c.rs_inc(rs, "succeeded")
                elif phase == "Failed":
                    c.rs_inc(rs, "failed")

    def create_new_pod(self, job: dict, rt: str, index: str, spec: dict, master: bool,
                       replicas: Dict[str, dict]) -> None:
        key = job_key(job)
        exp_key = c.gen_expectation_pods_key(key, rt)
        self.expectations.expect_creations(exp_key, 1)
        labels = self.gen_labels(job["metadata"]["name"])
        labels[c.REPLICA_TYPE_LABEL] = rt
        labels[c.REPLICA_INDEX_LABEL] = index
        if master:
            labels[c.JOB_ROLE_LABEL] = "master"
        tmpl = copy.deepcopy(spec.get("template") or {})
        tmd = tmpl.setdefault("metadata", {})
        tmd["name"] = c.gen_general_name(job["metadata"]["name"], rt, index)
        tmd.setdefault("labels", {}).update(labels)
        self.controller.set_cluster_spec(job, tmpl, rt, index)
        pspec = tmpl.setdefault("spec", {})
        if pspec.get("restartPolicy"):
            msg = "Restart policy in pod template will be overwritten by restart policy in replica spec"
            logger_for_job(job, log).warning(msg)
            self.recorder.event(job, WARNING, POD_TEMPLATE_RESTART_POLICY, msg)
        # setRestartPolicy: ExitCode is implemented by the controller => pod Never
        rp = spec.get("restartPolicy", "")
        pspec["restartPolicy"] = c.RESTART_POLICY_NEVER if rp == c.RESTART_POLICY_EXIT_CODE else rp
        if self.config.enable_gang_scheduling and self.gang is not None:
            md = job["metadata"]
            entity = self.gang.get_gang(md["namespace"], md["name"])
            if entity is None:
                entity = self.gang.create_gang(job, replicas)
            self.gang.bind_pod_to_gang(tmpl, entity)
        annotations = dict(tmd.get("annotations") or {})
        # [NEW] FIFO position of the job (a restarted gang keeps its place)
        annotations.setdefault("kubedl.io/queue-time", job["metadata"].get("creationTimestamp") or c.now())
        pod = {"apiVersion": "v1", "kind": "Pod",
               "metadata": {"name": tmd["name"], "namespace": job["metadata"]["namespace"],
                            "labels": dict(tmd.get("labels") or {}),
                            "annotations": annotations,
                            "ownerReferences": [gen_owner_reference(job)]},
               "spec": pspec,
               "status": {"phase": "Pending"}}
        try:
            self.create_pod(job, pod)
        except Exception:
            self.expectations.creation_observed(exp_key)
            raise

    # ------------------------------------------------------------ services
    def reconcile_services(self, job: dict, services: List[dict], rtype: str, spec: dict) -> None:
        rt = rtype.lower()
        svcs = self.filter_for_replica_type(services, rt)
        for index, sl in enumerate(self.get_slices(svcs, c.replicas_of(spec))):
            if len(sl) > 1:
                log.warning("too many services for %s %d", rt, index)
            elif len(sl) == 0:
                self.create_new_service(job, rtype, spec, str(index))

    def port_from_spec(self, spec: dict) -> int:
        for ctr in c.containers_of(spec):
            if ctr.get("name") == self.controller.get_default_container_name():
                for p in ctr.get("ports") or []:
                    if p.get("name") == self.controller.get_default_container_port_name():
                        return int(p["containerPort"])
        raise LookupError("failed to find the port")

    def create_new_service(self, job: dict, rtype: str, spec: dict, index: str) -> None:
        key = job_key(job)
        rt = rtype.lower()
        exp_key = c.gen_expectation_services_key(key, rt)
        self.expectations.expect_creations(exp_key, 1)
        labels = self.gen_labels(job["metadata"]["name"])
        labels[c.REPLICA_TYPE_LABEL] = rt
        labels[c.REPLICA_INDEX_LABEL] = index
        try:
            port = self.port_from_spec(spec)
        except LookupError:
            self.expectations.creation_observed(exp_key)
            raise
        name = c.gen_general_name(job["metadata"]["name"], rt, index)
        ns = job["metadata"]["namespace"]
        svc = {"apiVersion": "v1", "kind": "Service",
               "metadata": {"name": name, "namespace": ns, "labels": labels,
                            "ownerReferences": [gen_owner_reference(job)]},
               "spec": {"clusterIP": "None", "selector": dict(labels),
                        "ports": [{"name": self.controller.get_default_container_port_name(),
                                   "port": port}]}}
        # local "DNS": the service name resolves to 127.0.0.1:<hostPort>
        host_port = self.store.host_port(ns, name, port)
        svc["metadata"]["annotations"] = {"kubedl.io/host-port": str(host_port)}
        try:
            self.service_control.create(job, svc)
        except AlreadyExists:
            self.expectations.creation_observed(exp_key)
            return
        except Exception:
            self.expectations.creation_observed(exp_key)
            raise
