"""XDLJob controller (``controllers/xdl/``).

Cluster spec (``xdljob_controller.go:191-217``): for every container, append
``/<job-UID>`` to ``ZK_ADDR`` (no double slash) and add ``TASK_NAME`` =
lower-cased replica type and ``TASK_INDEX`` = index.  ``XDL_CONFIG`` /
``genXDLConfigJSON`` are dead code in the reference and not reproduced.
Reconcile order PS, Scheduler, Worker, ExtendRole; no master role.

Status (``status.go:61-160``): failures are checked first and return at the
first failed type; ``startTime`` is set when a type is fully active;
Succeeded when succeeded(Worker + ExtendRole) >= ``ceil(n * minFinishWorkRate
/ 100)`` (rate wins when both are set) or ``minFinishWorkNum``; else Running.

[NEW] With no ZooKeeper on the node, the bundled CTR worker
(``kubedl_amd.workers.xdl_ctr``) rendezvouses through ``ZK_ADDR`` when it
is a ``host:port`` it can reach, else through ``KDL_RDZV_*`` set by the runtime.
"""
from __future__ import annotations

import math

from kubedl_amd.api import common as c
from kubedl_amd.api import kinds as K
from kubedl_amd.controllers.base import BaseReconciler

ZK_ADDR = "ZK_ADDR"
TASK_NAME = "TASK_NAME"
TASK_INDEX = "TASK_INDEX"


def calculate_min_finish(job: dict, workers: int) -> int:
    spec = job.get("spec") or {}
    if spec.get("minFinishWorkRate") is not None:
        return int(math.ceil(workers * int(spec["minFinishWorkRate"]) / 100.0))
    if spec.get("minFinishWorkNum") is not None:
        return int(spec["minFinishWorkNum"])
    return workers


class XDLJobReconciler(BaseReconciler):
    info = K.XDLJOB
    collective = True

    def created_msg_kind(self) -> str:
        return "XdlJob"

    def set_cluster_spec(self, job: dict, pod_template: dict, rtype: str, index: str) -> None:
        uid = job["metadata"]["uid"]
        rdzv = self._rendezvous_env(job, rtype, int(index))
        for ctr in (pod_template.setdefault("spec", {}).get("containers") or []):
            env = ctr.setdefault("env", [])
            for e in env:
                if e.get("name") == ZK_ADDR:
                    v = e.get("value", "")
                    e["value"] = v + uid if v.endswith("/") else v + "/" + uid
            env.append({"name": TASK_NAME, "value": rtype.lower()})
            env.append({"name": TASK_INDEX, "value": index})
            env.extend(rdzv)

    @staticmethod
    def _rendezvous_env(job: dict, rtype: str, index: int):
        """[NEW] collective rendezvous for the bundled CTR worker (no ZooKeeper on
        the node): PS, Worker, ExtendRole ranks form one process group in that
        order; the Scheduler is not a member.  The endpoint is the first
        member's Service, resolved to 127.0.0.1:<hostPort> by the runtime."""
        specs = K.replica_specs(job)
        order = [t for t in (K.XDL_PS, K.XDL_WORKER, K.XDL_EXTEND) if t in specs]
        base, rank = 0, -1
        for t in order:
            if t.lower() == rtype.lower():
                rank = base + index
            base += c.replicas_of(specs[t])
        if not order:
            return []
        first = order[0]
        try:
            port = c.port_from_job(specs, first, "xdl", "xdljob-port")
        except LookupError:
            port = 2222
        host = c.gen_general_name(job["metadata"]["name"], first.lower(), "0")
        n_ps = c.replicas_of(specs[K.XDL_PS]) if K.XDL_PS in specs else 0
        return [{"name": "KDL_RANK", "value": str(rank)}, {"name": "KDL_WORLD_SIZE", "value": str(base)},
                {"name": "KDL_NUM_PS", "value": str(n_ps)},
                {"name": "KDL_RDZV_ENDPOINT", "value": f"{host}:{port}"}]

    def update_job_status(self, job, replicas, status, restart) -> None:
        name = job["metadata"]["name"]
        prev_restarting = c.is_restarting(status)
        prev_failed = c.is_failed(status)
        workers = succeeded = 0
        for rtype, spec in replicas.items():
            rs = (status.get("replicaStatuses") or {}).get(rtype)
            if rs is None:
                continue
            n = c.replicas_of(spec)
            failed = c.rs_get(rs, "failed")
            if rtype in (K.XDL_WORKER, K.XDL_EXTEND):
                workers += n
                succeeded += c.rs_get(rs, "succeeded")
            if c.rs_get(rs, "active") == n and not status.get("startTime"):
                status["startTime"] = c.now()
            if failed > 0:
                self._failed_or_restarting(job, status, rtype, failed, restart, prev_restarting,
                                           prev_failed, "XDLJob")
                return
        if succeeded >= calculate_min_finish(job, workers):
            self._set_completion(status)
            already = c.is_succeeded(status)
            c.update_job_conditions(status, c.JOB_SUCCEEDED, c.JOB_SUCCEEDED_REASON,
                                    f"XDLJob {name} is successfully completed.")
            if not already:
                self.metrics.success_inc()
            return
        c.update_job_conditions(status, c.JOB_RUNNING, c.JOB_RUNNING_REASON, f"XDLJob {name} is running.")
