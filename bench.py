#!/usr/bin/env python3
"""Headline benchmark: PyTorchJob ResNet-50 DDP bf16 training on MI355X.

Metric/config from BASELINE.json ("Job launch delay (s) + steps/sec, PyTorchJob
ResNet-50 at 1/2/4/8 MI355X"; config "PyTorchJob ResNet-50 DDP bf16, 8 workers").
The reference publishes no number, so ``vs_baseline`` is null.

Driver contract: ``python bench.py --gpus N --steps K --warmup W``.  Two ways in:

* **No ``WORLD_SIZE`` in the environment** (the default, any N >= 1): this
  process is a kdl control plane.  It starts an in-process ``Manager`` (store,
  PyTorchJob controller, all-or-nothing gang allocator, node scheduler,
  kubelet with the pre-warmed rank zygote), submits ONE PyTorchJob of N ranks
  (1 Master + N-1 Workers, ``amd.com/gpu: 1`` each), waits for it to succeed
  and prints rank 0's result plus the controller-path launch delays
  (``first_pod_launch_delay_s`` / ``all_pods_launch_delay_s``: job creation ->
  first / last rank Ready, the reference's histograms; measured warm -- ranks
  forked from the running node's pre-imported zygote -- with ``cold_*`` from a
  ready-only probe job submitted before the zygote is up; ``comm_init_s`` =
  the first collective, where the lazy RCCL communicator bootstraps;
  ``pkg/metrics/job_metrics.go:139-194``, observed at
  ``pkg/job_controller/job.go:242-259``).  This process never touches the GPU
  (it does not even import torch): the ranks are forked from the zygote or
  spawned by the kubelet before any GPU call.  Exit status is non-zero if the
  job did not succeed with N Ready ranks or rank 0's world size is not N.
* **``WORLD_SIZE`` set** (``torch.distributed.run``, or ``--direct``): this
  process IS a rank (``kubedl_amd.workers.resnet_bench.run``).

Either way the timed region is the ranks' own: W untimed warm-up steps, then
exactly K steps between a barrier + ``synchronize`` on both sides, MAX over
ranks; ``value`` is whole-job images/s (weak scaling, fixed per-GPU batch).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from kubedl_amd.workers import resnet_bench  # noqa: E402  (no torch import at module level)

JOB_NAME = "resnet50-bench"


def _rank_args(args) -> list:
    out = ["--gpus", str(args.gpus), "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--batch", str(args.batch), "--image", str(args.image), "--bn-backend", args.bn_backend,
           "--conv-benchmark", str(args.conv_benchmark), "--engine", args.engine,
           "--allreduce", args.allreduce]
    if args.cpu:
        out.append("--cpu")
    if args.tiny:
        out.append("--tiny")
    return out


def make_job(args, name: str = JOB_NAME, ready_only: bool = False) -> dict:
    """One PyTorchJob, N ranks, one GPU each (the BASELINE.json job spec);
    ``ready_only``: the same ranks exit right after signalling Ready (the cold
    launch-delay probe)."""
    cmd = [sys.executable, "-u", "-m", "kubedl_amd.workers.resnet_bench"] + _rank_args(args)
    if ready_only:
        cmd.append("--ready-only")
    res = {"limits": {"cpu": "2"}} if args.cpu else {"limits": {"amd.com/gpu": 1}}
    env = [{"name": "KDL_BENCH_LAUNCHER", "value": "kdl-pytorchjob"}]
    if os.environ.get("KDL_FAULT"):  # fault-injection rehearsal (the kubelet never leaks it by itself)
        env.append({"name": "KDL_FAULT", "value": os.environ["KDL_FAULT"]})

    def tmpl():
        return {"spec": {"containers": [{"name": "pytorch", "image": "kubedl-amd/resnet50",
                                         "command": list(cmd), "env": list(env), "resources": res}]}}
    specs = {"Master": {"replicas": 1, "restartPolicy": "Never", "template": tmpl()}}
    if args.gpus > 1:
        specs["Worker"] = {"replicas": args.gpus - 1, "restartPolicy": "Never", "template": tmpl()}
    return {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
            "metadata": {"name": name, "namespace": "default"},
            "spec": {"cleanPodPolicy": "None", "pytorchReplicaSpecs": specs}}


def _last_json(path):
    try:
        for line in reversed(open(path, errors="replace").read().splitlines()):
            line = line.strip()
            if line.startswith("{") and line.endswith("}"):
                return json.loads(line)
    except (OSError, TypeError, ValueError):
        pass
    return None


def _tail(path, n=40) -> str:
    try:
        return "\n".join(open(path, errors="replace").read().splitlines()[-n:])
    except (OSError, TypeError):
        return "<no log>"


def launch_job(args) -> int:
    from kubedl_amd.api import common as c
    from kubedl_amd.engine.manager import Manager, ManagerOptions
    from kubedl_amd.gang.allocator import detect_gpus

    if not args.cpu:
        have = detect_gpus().count
        if have < args.gpus:
            print(f"[bench] --gpus {args.gpus} but this node has {have} GPU(s)", file=sys.stderr)
            return 2
    home = tempfile.mkdtemp(prefix="kdl-bench-")
    mgr = Manager(ManagerOptions(home=home, gang_scheduler_name="kdl-gang")).start()
    rc = 1
    cold = {}
    try:
        # 1. cold launch delay: a ready-only job of the same N ranks submitted the
        #    moment the node runtime is up, before the rank zygote can serve it
        #    (every rank is a fresh interpreter importing torch) -- a node's first job
        if not args.no_cold_probe:
            probe = mgr.apply(make_job(args, JOB_NAME + "-cold", ready_only=True))
            try:
                pj = mgr.wait_for_condition("PyTorchJob", "default", JOB_NAME + "-cold", ["Succeeded", "Failed"],
                                            timeout=min(args.timeout, 600))
                if c.last_condition_type(pj.get("status") or {}) == "Succeeded":
                    puid = probe["metadata"]["uid"]
                    for k, key in (("first", "cold_first_pod_launch_delay_s"), ("all", "cold_all_pods_launch_delay_s")):
                        v = mgr.metrics.observed[k].get(puid)
                        cold[key] = round(v, 3) if v is not None else None
            except TimeoutError as e:
                print(f"[bench] cold probe: {e}", file=sys.stderr)
        # 2. warm: a running node's steady state (the reference's long-lived
        #    operator) -- ranks forked from the pre-imported zygote
        z = mgr.kubelet.zygote if mgr.kubelet is not None else None
        zygote_ready = bool(z is not None and z.ready.wait(timeout=min(args.timeout, 300)))
        # ... its device libraries in the page cache and the node warm-up done
        # (runtime/zygote.py, runtime/node_warm.py: the code-object cache the
        # first communicator of a fresh node otherwise fills, ~2.6 s)
        if z is not None:
            z.prefetched.wait(timeout=min(args.timeout, 240))
        t_submit = time.time()
        job = mgr.apply(make_job(args))
        uid = job["metadata"]["uid"]
        try:
            job = mgr.wait_for_condition("PyTorchJob", "default", JOB_NAME, ["Succeeded", "Failed"],
                                         timeout=args.timeout)
        except TimeoutError as e:
            print(f"[bench] {e}", file=sys.stderr)
            job = mgr.get("PyTorchJob", "default", JOB_NAME)
        st = job.get("status") or {}
        state = c.last_condition_type(st)
        pods = [p for p in mgr.store.list("Pod", "default")
                if (p["metadata"].get("labels") or {}).get(c.JOB_NAME_LABEL) == JOB_NAME]
        ready = [p for p in pods if any(x.get("type") == "Ready" and x.get("status") == "True"
                                        for x in (p.get("status") or {}).get("conditions") or [])
                 or (p.get("status") or {}).get("phase") == "Succeeded"]
        master_log = mgr.kubelet.log_path("default", f"{JOB_NAME}-master-0")
        res = _last_json(master_log)
        if state != "Succeeded" or res is None:
            print(f"[bench] job {JOB_NAME} ended {state!r}; rank logs:", file=sys.stderr)
            for p in sorted(pods, key=lambda p: p["metadata"]["name"]):
                lp = mgr.kubelet.log_path("default", p["metadata"]["name"])
                print(f"---- {p['metadata']['name']} ----\n{_tail(lp)}", file=sys.stderr)
            return 1
        if res.get("n_gpus") != args.gpus or len(pods) != args.gpus:
            print(f"[bench] world size mismatch: rank 0 reports {res.get('n_gpus')}, "
                  f"{len(pods)} pods, --gpus {args.gpus}", file=sys.stderr)
            return 1
        created = c.to_epoch(job["metadata"]["creationTimestamp"])
        first = mgr.metrics.observed["first"].get(uid)
        alld = mgr.metrics.observed["all"].get(uid)
        res["first_pod_launch_delay_s"] = round(first, 3) if first is not None else None
        res["all_pods_launch_delay_s"] = round(alld, 3) if alld is not None else None
        res["job_wall_s"] = (round(c.to_epoch(st["completionTime"]) - created, 3)
                             if st.get("completionTime") else None)
        res["submit_to_done_s"] = round(time.time() - t_submit, 3)
        if res.get("t_first_step_unix"):
            # job creation -> every rank has finished its first training step:
            # launch delay + model build + communicator bootstrap + step 1
            res["time_to_first_step_s"] = round(res["t_first_step_unix"] - created, 3)
        res["ranks_ready"] = len(ready)
        res["launch"] = "warm (zygote)" if zygote_ready else "cold (no zygote)"
        if z is not None and z.prefetch_s is not None:
            res["node_prefetch_s"] = round(z.prefetch_s, 3)
        if z is not None and z.warm is not None:
            res["node_warm"] = z.warm
        res.update(cold)
        if os.environ.get("KDL_BENCH_KEEP"):
            res["home"] = home
        res["gpus"] = sorted({int(g) for p in pods
                              for g in ((p["metadata"].get("annotations") or {}).get("kubedl.io/gpus") or "")
                              .split(",") if g})
        print(json.dumps(res), flush=True)
        rc = 0 if len(ready) == args.gpus else 1
        if rc:
            print(f"[bench] only {len(ready)}/{args.gpus} ranks became Ready", file=sys.stderr)
        return rc
    finally:
        mgr.stop()
        if not os.environ.get("KDL_BENCH_KEEP"):
            shutil.rmtree(home, ignore_errors=True)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    resnet_bench.add_args(ap)
    ap.add_argument("--direct", action="store_true",
                    help="run as a single in-process rank (no control plane); WORLD_SIZE forces this too")
    ap.add_argument("--timeout", type=float, default=1800.0, help="job-path wait limit (s)")
    ap.add_argument("--no-cold-probe", action="store_true",
                    help="job path: skip the cold (pre-zygote) ready-only probe job")
    args = ap.parse_args(argv)
    if "WORLD_SIZE" in os.environ or args.direct:
        if "WORLD_SIZE" not in os.environ:
            os.environ.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
        ws = int(os.environ["WORLD_SIZE"])
        if ws != args.gpus and int(os.environ.get("RANK", "0")) == 0:
            print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={ws}", file=sys.stderr)
        return resnet_bench.run(args, "direct" if args.direct else "torchrun")
    return launch_job(args)


if __name__ == "__main__":
    sys.exit(main())
