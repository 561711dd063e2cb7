"""TFJob controller (``controllers/tensorflow/``).

Cluster spec (``tfjob_controller.go:187-245``, ``tensorflow.go:30-142``):
``TF_CONFIG`` = ``{"cluster": {<rt>: ["<job>-<rt>-<i>.<ns>.svc[.$CUSTOM_CLUSTER_DOMAIN]:<port>", ...]},
"task": {"type": <rt>, "index": <i>}, "environment": "cloud"}`` is added to
the ``tensorflow`` container only when the job is distributed (total
replicas != 1).  Evaluator replicas are left out of the cluster spec, and
Evaluator pods are never created (absent from the reconcile order: a
reference quirk we keep).

Status (``status.go:56-212``): with a Chief/Master, chief running =>
Running and chief ``replicas - succeeded == 0`` => Succeeded; otherwise for
Worker: all succeeded OR worker-0 exited 0 => Succeeded, any running =>
Running.  Failures => Restarting/Failed.

The TF data plane itself (gRPC PS/worker) is not on the MI355X path; the
bundled TF worker (``kubedl_amd.workers.tf_stub``) parses ``TF_CONFIG``,
opens its server port and rendezvouses with its peers -- the plumbing the
``tf_job_mnist.yaml`` example needs.
"""
from __future__ import annotations

import json
import os

from kubedl_amd.api import common as c
from kubedl_amd.api import kinds as K
from kubedl_amd.controllers.base import BaseReconciler

ENV_CUSTOM_CLUSTER_DOMAIN = "CUSTOM_CLUSTER_DOMAIN"
TF_CONFIG = "TF_CONFIG"


def contain_chief_or_master(job: dict) -> bool:
    specs = K.replica_specs(job)
    return K.TF_CHIEF in specs or K.TF_MASTER in specs


def is_distributed(job: dict) -> bool:
    specs = K.replica_specs(job)
    n = 0
    for t in (K.TF_CHIEF, K.TF_EVAL, K.TF_MASTER, K.TF_PS, K.TF_WORKER):
        s = specs.get(t)
        if s is not None:
            n += 1 if s.get("replicas") is None else int(s["replicas"])
    return n != 1


def gen_cluster_spec(job: dict) -> dict:
    cluster = {}
    md = job["metadata"]
    specs = K.replica_specs(job)
    domain = os.environ.get(ENV_CUSTOM_CLUSTER_DOMAIN, "")
    for rtype, spec in specs.items():
        if rtype == K.TF_EVAL:
            continue
        rt = rtype.lower()
        port = c.port_from_job(specs, rtype, "tensorflow", "tfjob-port")
        names = []
        for i in range(c.replicas_of(spec)):
            svc = f"{c.gen_general_name(md['name'], rt, i)}.{md['namespace']}.svc"
            if domain:
                svc += "." + domain
            names.append(f"{svc}:{port}")
        cluster[rt] = names
    return cluster


def gen_tf_config(job: dict, rtype: str, index: str) -> str:
    cfg = {"cluster": gen_cluster_spec(job), "task": {"type": rtype, "index": int(index, 0)},
           "environment": "cloud"}
    return json.dumps(cfg, separators=(",", ":"))


class TFJobReconciler(BaseReconciler):
    info = K.TFJOB

    def is_master_role(self, replicas, rtype, index) -> bool:
        return K.tf_is_chief_or_master(rtype)

    def set_cluster_spec(self, job: dict, pod_template: dict, rtype: str, index: str) -> None:
        if not is_distributed(job):
            return
        cfg = gen_tf_config(job, rtype, index)
        for ctr in (pod_template.setdefault("spec", {}).get("containers") or []):
            if ctr.get("name") == "tensorflow":
                self._append_env(ctr, TF_CONFIG, cfg)
                break

    def update_job_status(self, job, replicas, status, restart) -> None:
        name = job["metadata"]["name"]
        prev_restarting = c.is_restarting(status)
        prev_failed = c.is_failed(status)
        worker0_completed = False
        pods = self.ctrl.filter_for_replica_type(self.get_pods_for_job(job), K.TF_WORKER.lower())
        for pod in pods:
            try:
                idx = int((pod["metadata"].get("labels") or {}).get(c.REPLICA_INDEX_LABEL, ""))
            except ValueError:
                continue
            if idx == 0:
                code = 0xBEEF
                for cs in (pod.get("status") or {}).get("containerStatuses") or []:
                    term = (cs.get("state") or {}).get("terminated")
                    if cs.get("name") == "tensorflow" and term is not None:
                        code = int(term.get("exitCode", 0))
                        break
                if code == 0 and (pod.get("status") or {}).get("phase") == "Succeeded":
                    worker0_completed = True
                break
        if not status.get("startTime"):
            status["startTime"] = c.now()
        has_chief = contain_chief_or_master(job)
        for rtype, spec in replicas.items():
            rs = (status.get("replicaStatuses") or {}).get(rtype)
            if rs is None:
                continue
            expected = c.replicas_of(spec) - c.rs_get(rs, "succeeded")
            running = c.rs_get(rs, "active")
            failed = c.rs_get(rs, "failed")
            if has_chief:
                if K.tf_is_chief_or_master(rtype):
                    if running > 0:
                        c.update_job_conditions(status, c.JOB_RUNNING, c.JOB_RUNNING_REASON,
                                                f"TFJob {name} is running.")
                    if expected == 0:
                        self._succeeded(job, status, f"TFJob {name} successfully completed.")
            elif rtype == K.TF_WORKER:
                if expected == 0 or worker0_completed:
                    self._succeeded(job, status, f"TFJob {name} successfully completed.")
                elif running > 0:
                    c.update_job_conditions(status, c.JOB_RUNNING, c.JOB_RUNNING_REASON,
                                            f"TFJob {name} is running.")
            if failed > 0:
                self._failed_or_restarting(job, status, rtype, failed, restart, prev_restarting,
                                           prev_failed, "TFJob")
