"""XGBoostJob controller (``controllers/xgboost/``).

Cluster spec (``pod.go:106-152``; test ``pod_test.go:69-124``): the same five
env vars as PyTorch, but ``RANK = index`` WITHOUT the +1 offset (so master-0
and worker-0 both get RANK 0 -- a reference quirk kept for API parity; rabit
assigns real ranks through its tracker) and ``MASTER_ADDR`` is always
``<job>-master-0`` (no ``localhost`` on the master).  [NEW] ``KDL_RANK``
carries a collision-free rank (master 0, worker i -> i + 1) that the bundled
GBDT worker uses for its RCCL process group.

Status (``job.go:89-190``): ``startTime`` is set when some replica type is
fully active; Master running => Running; Master done => Succeeded (early
return); failures => Restarting/Failed; otherwise the function falls through
to an UNCONDITIONAL Running condition (quirk kept).  The group-name label is
``kubeflow.org`` (not the API group).
"""
from __future__ import annotations

from kubedl_amd.api import common as c
from kubedl_amd.api import kinds as K
from kubedl_amd.controllers.base import BaseReconciler


class XGBoostJobReconciler(BaseReconciler):
    info = K.XGBOOSTJOB
    collective = True

    def created_msg_kind(self) -> str:
        return "xgboostJob"  # reference message spelling (job.go:218)

    def is_master_role(self, replicas, rtype, index) -> bool:
        return rtype == K.XGB_MASTER

    def set_cluster_spec(self, job: dict, pod_template: dict, rtype: str, index: str) -> None:
        specs = K.replica_specs(job)
        rank = int(index)
        master_addr = c.gen_general_name(job["metadata"]["name"], K.XGB_MASTER.lower(), "0")
        master_port = c.port_from_job(specs, K.XGB_MASTER, "xgboostjob", "xgboostjob-port")
        world = c.total_replicas(specs)
        kdl_rank = rank if rtype == K.XGB_MASTER.lower() else rank + (
            c.replicas_of(specs[K.XGB_MASTER]) if K.XGB_MASTER in specs else 0)
        for ctr in (pod_template.setdefault("spec", {}).get("containers") or []):
            self._append_env(ctr, "MASTER_PORT", str(master_port))
            self._append_env(ctr, "MASTER_ADDR", master_addr)
            self._append_env(ctr, "WORLD_SIZE", str(world))
            self._append_env(ctr, "RANK", str(rank))
            self._append_env(ctr, "PYTHONUNBUFFERED", "0")
            self._append_env(ctr, "KDL_RANK", str(kdl_rank))

    def update_job_status(self, job, replicas, status, restart) -> None:
        name = job["metadata"]["name"]
        prev_restarting = c.is_restarting(status)
        prev_failed = c.is_failed(status)
        for rtype, spec in replicas.items():
            rs = (status.get("replicaStatuses") or {}).get(rtype)
            if rs is None:
                continue
            succeeded = c.rs_get(rs, "succeeded")
            expected = c.replicas_of(spec) - succeeded
            running = c.rs_get(rs, "active")
            failed = c.rs_get(rs, "failed")
            if running == c.replicas_of(spec) and not status.get("startTime"):
                status["startTime"] = c.now()
            if rtype == K.XGB_MASTER:
                if running > 0:
                    c.update_job_conditions(status, c.JOB_RUNNING, c.JOB_RUNNING_REASON,
                                            f"XGBoostJob {name} is running.")
                if expected == 0:
                    self._succeeded(job, status, f"XGBoostJob {name} is successfully completed.")
                    return
            if failed > 0:
                self._failed_or_restarting(job, status, rtype, failed, restart, prev_restarting,
                                           prev_failed, "XGBoostJob")
        c.update_job_conditions(status, c.JOB_RUNNING, c.JOB_RUNNING_REASON,
                                f"XGBoostJob {name} is running.")
