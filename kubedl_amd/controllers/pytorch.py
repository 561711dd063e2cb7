"""PyTorchJob controller (``controllers/pytorch/``).

Cluster spec (``pytorchjob_controller.go:180-233``): on EVERY container
``MASTER_PORT`` = the Master's ``pytorchjob-port``, ``MASTER_ADDR`` =
``<job>-master-0`` (``localhost`` on the master itself), ``WORLD_SIZE`` =
sum of replicas, ``RANK`` = 0 for the master and ``index + 1`` for workers,
``PYTHONUNBUFFERED=0``.  A master with index != 0 is an error.  Services are
created for the Master only (``pkg/job_controller/job.go:224-227``).

Status (``status.go:34-125``): Master running => Running; Master
``replicas - succeeded == 0`` => Succeeded; any failed replica => Restarting
(when a pod is being restarted) or Failed; a job without a Master spec is
``invalid config``.

On the MI355X runtime each rank is one process on its gang-allocated GPU;
``MASTER_ADDR``/``MASTER_PORT`` are resolved by the runtime to
``127.0.0.1:<service host port>`` and the worker binds RCCL over xGMI.
"""
from __future__ import annotations

from kubedl_amd.api import common as c
from kubedl_amd.api import kinds as K
from kubedl_amd.controllers.base import BaseReconciler


class PyTorchJobReconciler(BaseReconciler):
    info = K.PYTORCHJOB
    collective = True

    def created_msg_kind(self) -> str:
        return "PytorchJob"  # reference message spelling (status.go:137)

    def is_master_role(self, replicas, rtype, index) -> bool:
        return K.PT_MASTER in replicas and rtype == K.PT_MASTER

    def reconcile_services_for(self, rtype: str) -> bool:
        return rtype == K.PT_MASTER

    def set_cluster_spec(self, job: dict, pod_template: dict, rtype: str, index: str) -> None:
        specs = K.replica_specs(job)
        rank = int(index)
        master_port = c.port_from_job(specs, K.PT_MASTER, "pytorch", "pytorchjob-port")
        master_addr = c.gen_general_name(job["metadata"]["name"], K.PT_MASTER.lower(), "0")
        if rtype == K.PT_MASTER.lower():
            if rank != 0:
                raise ValueError("invalid config: There should be only a single master with index=0")
            master_addr = "localhost"
        else:
            rank += 1
        world = c.total_replicas(specs)
        for ctr in (pod_template.setdefault("spec", {}).get("containers") or []):
            self._append_env(ctr, "MASTER_PORT", str(master_port))
            self._append_env(ctr, "MASTER_ADDR", master_addr)
            self._append_env(ctr, "WORLD_SIZE", str(world))
            self._append_env(ctr, "RANK", str(rank))
            self._append_env(ctr, "PYTHONUNBUFFERED", "0")

    def update_job_status(self, job, replicas, status, restart) -> None:
        if not status.get("startTime"):
            status["startTime"] = c.now()
        prev_restarting = c.is_restarting(status)
        prev_failed = c.is_failed(status)
        name = job["metadata"]["name"]
        for rtype, spec in replicas.items():
            rs = (status.get("replicaStatuses") or {}).get(rtype)
            if rs is None:
                continue
            expected = c.replicas_of(spec) - c.rs_get(rs, "succeeded")
            running = c.rs_get(rs, "active")
            failed = c.rs_get(rs, "failed")
            if K.PT_MASTER not in replicas:
                raise ValueError("invalid config: Job must contain master replica spec")
            if rtype == K.PT_MASTER:
                if running > 0:
                    c.update_job_conditions(status, c.JOB_RUNNING, c.JOB_RUNNING_REASON,
                                            f"PyTorchJob {name} is running.")
                if expected == 0:
                    self._succeeded(job, status, f"PyTorchJob {name} is successfully completed.")
            if failed > 0:
                self._failed_or_restarting(job, status, rtype, failed, restart, prev_restarting,
                                           prev_failed, "PyTorchJob")
