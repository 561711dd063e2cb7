"""Launch-delay benchmark through the full control plane (BASELINE.md metric).

Submits ``--jobs`` concurrent PyTorchJobs, each ``--gpus`` ranks (1 Master +
gpus-1 Workers, ``amd.com/gpu: 1`` per rank) running the ResNet-50 DDP worker
(``kubedl_amd.workers.resnet50``), through store -> reconcile -> gang
allocator -> kubelet -> rank processes, and reports per job:

* ``first_pod_launch_delay_s`` / ``all_pods_launch_delay_s`` -- exactly the
  reference histograms' values (``pkg/metrics/job_metrics.go:139-194``):
  earliest / latest rank Ready time minus job creation; a rank is Ready when
  its process group is initialised (``KDL_READY_FILE``);
* ``steps_per_sec`` / ``images_per_sec`` as reported by rank 0;
* ``job_wall_s`` -- creation to Succeeded.

With ``--jobs 2 --gpus 4 --gang`` this is BASELINE.json's "2x concurrent
PyTorchJob 4-GPU each, gang-scheduled" config.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import time


def add_args(p) -> None:
    p.add_argument("--jobs", type=int, default=1)
    p.add_argument("--gpus", type=int, default=1, help="ranks (GPUs) per job")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--image", type=int, default=224)
    p.add_argument("--tiny", action="store_true")
    p.add_argument("--cpu", action="store_true", help="CPU/gloo ranks (plumbing test)")
    p.add_argument("--gang", action="store_true")
    p.add_argument("--node-gpus", type=int, default=None)
    p.add_argument("--timeout", type=float, default=1800)
    p.add_argument("--home", default=None)


def make_job(name: str, ranks: int, args) -> dict:
    cmd = [sys.executable, "-u", "-m", "kubedl_amd.workers.resnet50", "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--batch", str(args.batch), "--image", str(args.image)]
    if args.tiny:
        cmd.append("--tiny")
    if args.cpu:
        cmd.append("--cpu")
    res = {"resources": {"limits": {"cpu": "2"}}} if args.cpu else {"resources": {"limits": {"amd.com/gpu": 1}}}

    def tmpl():
        return {"spec": {"containers": [dict({"name": "pytorch", "image": "kubedl-amd/resnet50",
                                               "command": list(cmd)}, **res)]}}
    specs = {"Master": {"replicas": 1, "restartPolicy": "Never", "template": tmpl()}}
    if ranks > 1:
        specs["Worker"] = {"replicas": ranks - 1, "restartPolicy": "Never", "template": tmpl()}
    return {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
            "metadata": {"name": name, "namespace": "default"},
            "spec": {"cleanPodPolicy": "None", "pytorchReplicaSpecs": specs}}


def _last_json(path: str):
    try:
        for line in reversed(open(path, errors="replace").read().splitlines()):
            line = line.strip()
            if line.startswith("{") and line.endswith("}"):
                return json.loads(line)
    except (OSError, ValueError):
        pass
    return None


def main(args) -> int:
    from kubedl_amd.api import common as c
    from kubedl_amd.engine.manager import Manager, ManagerOptions
    home = args.home or tempfile.mkdtemp(prefix="kdl-bench-")
    mgr = Manager(ManagerOptions(home=home, gpus=args.node_gpus,
                                 gang_scheduler_name="kdl-gang" if args.gang else "")).start()
    out = {"metric": "job launch delay (s) + steps/sec", "jobs": []}
    try:
        names = [f"resnet50-j{i}" for i in range(args.jobs)]
        t0 = time.time()
        for n in names:
            mgr.apply(make_job(n, args.gpus, args))
        for n in names:
            job = mgr.wait_for_condition("PyTorchJob", "default", n, ["Succeeded", "Failed"], timeout=args.timeout)
            st = job["status"]
            uid = job["metadata"]["uid"]
            created = c.to_epoch(job["metadata"]["creationTimestamp"])
            res = _last_json(mgr.kubelet.log_path("default", f"{n}-master-0")) or {}
            if c.last_condition_type(st) != "Succeeded":
                # a diagnosable tail per rank: which rank died, and how
                print(f"[bench_launch] job {n} ended {c.last_condition_type(st)!r}; rank logs:", file=sys.stderr)
                for p in mgr.store.list("Pod", "default"):
                    pn = p["metadata"]["name"]
                    if not pn.startswith(n + "-"):
                        continue
                    lp = mgr.kubelet.log_path("default", pn)
                    tail = ""
                    if lp and os.path.exists(lp):
                        with open(lp, errors="replace") as f:
                            tail = "".join(f.readlines()[-30:])
                    print(f"---- {pn} ----\n{tail}", file=sys.stderr, flush=True)
            out["jobs"].append({
                "name": n, "state": c.last_condition_type(st), "ranks": args.gpus,
                "first_pod_launch_delay_s": mgr.metrics.observed["first"].get(uid),
                "all_pods_launch_delay_s": mgr.metrics.observed["all"].get(uid),
                "job_wall_s": round(c.to_epoch(st.get("completionTime")) - created, 3)
                if st.get("completionTime") else None,
                "steps_per_sec": res.get("steps_per_sec"), "images_per_sec": res.get("images_per_sec"),
                "gpus": sorted({g for p in mgr.store.list("Pod") if p["metadata"]["name"].startswith(n + "-")
                                for g in (p["metadata"].get("annotations") or {}).get("kubedl.io/gpus", "").split(",")
                                if g}),
            })
        out["total_wall_s"] = round(time.time() - t0, 3)
        out["config"] = {"jobs": args.jobs, "gpus_per_job": args.gpus, "gang": bool(args.gang),
                         "batch": args.batch, "image": args.image, "tiny": bool(args.tiny), "cpu": bool(args.cpu)}
    finally:
        mgr.stop()
    print(json.dumps(out), flush=True)
    return 0 if all(j["state"] == "Succeeded" for j in out["jobs"]) else 1
