"""Rank-process supervisor: runs bound pods as local process trees ("kubelet").

For every pod bound to this node (``spec.nodeName``, GPUs in the
``kubedl.io/gpus`` annotation) a pod worker thread:

1. builds a sandbox ``<root>/pods/<ns>_<name>_<uid8>/`` with ``volumes/``
   (emptyDir; hostPath maps to the host path), a ``root/`` tree where every
   ``volumeMount`` appears as a symlink (``subPath`` honoured) and ``logs/``;
2. runs ``initContainers`` one after another (e.g. ``git-sync-code``), then
   all ``containers``, each as its own session/process group through the
   native spawner (``kubedl_amd._native.spawn``: PR_SET_PDEATHSIG, log
   redirection, exec-failure -> 127/126);
3. renders the environment: the container's ``env`` (``value`` and
   ``valueFrom.fieldRef``), service DNS names ``<svc>[.<ns>[.svc[.<domain>]]]``
   rewritten to ``127.0.0.1`` with each ``<svc>:<port>`` mapped to the
   store's host port (so two jobs can both use 23456), ``MASTER_PORT``
   remapped along with ``MASTER_ADDR``, ``HIP_VISIBLE_DEVICES`` from the gang
   allocation -- a gang member's own GPU is ``cuda:0`` as in a pod, with the
   rest of the gang's GPUs visible behind it for the xGMI P2P transports
   (runtime/gpu_env.py) -- and ``KDL_*`` sandbox variables;
4. reports status like a kubelet: ``phase`` Pending -> Running ->
   Succeeded/Failed, ``containerStatuses`` (``state.running|terminated``,
   ``exitCode``, ``restartCount``, ``lastState``), and the ``Initialized`` /
   ``ContainersReady`` / ``Ready`` conditions.  "Ready" is the rank's own
   signal (``$KDL_READY_FILE``, written once its process group is up) for
   bundled workers, process start otherwise -- the timestamp the launch-delay
   metrics use;
5. applies the pod ``restartPolicy``: Always / OnFailure restart the container
   in place with exponential back-off (``restartCount``++, pod stays Running,
   which is what ``pastBackoffLimit`` counts); Never leaves it terminated;
6. on pod deletion sends SIGTERM to the process group, waits
   ``terminationGracePeriodSeconds`` (default 5 s locally), then SIGKILL;
7. [NEW] gang teardown barrier: a new pod of a job does not start its
   containers while another pod of the same job is still terminating (a gang
   restart deletes every rank; the replacements must not race the old ranks
   for the master port or the GPU), and the scheduler keeps a deleted pod's
   GPUs reserved until its processes are gone (``holds``).
"""
from __future__ import annotations

import json
import logging
import os
import re
import shutil
import signal
import threading
import time
from typing import Dict, List, Optional, Tuple

from kubedl_amd.api import common as c
from kubedl_amd.runtime import images
from kubedl_amd.runtime import zygote as zygote_mod
from kubedl_amd.runtime.gpu_env import rank_gpu_env
from kubedl_amd.runtime.scheduler import GANG_GPUS_ANNOTATION, GPU_ANNOTATION, HBM_ANNOTATION
from kubedl_amd.store import ADDED, DELETED, MODIFIED, NotFound, Store

log = logging.getLogger("kubedl_amd.kubelet")

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# variables of the runtime process that must never leak into a rank
_ENV_DENY = {"RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
             "TF_CONFIG", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
             "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID", "KDL_FAULT", "KDL_READY_FILE",
             "KDL_PROGRESS_FILE", "PYTEST_CURRENT_TEST"}


def _spawner():
    from kubedl_amd.runtime import native  # KDL_NATIVE_SO: e.g. the sanitizer build
    return native.load()


class _Container:
    __slots__ = ("spec", "name", "pid", "started_at", "restart_count", "last_term", "term",
                 "next_start", "ready_file", "readiness", "ready_at", "log_path", "dns_wait_logged")

    def __init__(self, spec: dict, ready_file: str, log_path: str):
        self.spec = spec
        self.name = spec.get("name", "main")
        self.pid: Optional[int] = None
        self.started_at: Optional[str] = None
        self.restart_count = 0
        self.last_term: Optional[dict] = None
        self.term: Optional[dict] = None
        self.next_start = 0.0
        self.ready_file = ready_file
        self.readiness = "start"
        self.ready_at: Optional[str] = None
        self.log_path = log_path
        self.dns_wait_logged = False


class PodWorker(threading.Thread):
    def __init__(self, kubelet: "Kubelet", pod: dict):
        super().__init__(name=f"pod-{pod['metadata']['name']}", daemon=True)
        self.k = kubelet
        self.pod = pod
        md = pod["metadata"]
        self.ns, self.name, self.uid = md["namespace"], md["name"], md.get("uid", "")
        self.sandbox = os.path.join(kubelet.root, "pods", f"{self.ns}_{self.name}_{self.uid[:8]}")
        self.deleted = threading.Event()
        self.grace = float((pod.get("spec") or {}).get("terminationGracePeriodSeconds",
                                                      kubelet.default_grace))
        self.gpus = [g for g in ((md.get("annotations") or {}).get(GPU_ANNOTATION) or "").split(",") if g]
        self.job_label = (md.get("labels") or {}).get(c.JOB_NAME_LABEL, "")
        self.containers: List[_Container] = []
        self.start_time = c.now()
        self.unresolved: List[str] = []
        # how long a container waits for an unknown <svc>.<ns>.svc peer to appear
        self.dns_hold_until = time.monotonic() + kubelet.dns_hold_s

    # ------------------------------------------------------------ helpers
    def _patch_status(self, fn) -> bool:
        def mutate(o):
            if o["metadata"].get("uid") != self.uid:
                raise NotFound("pod replaced")
            fn(o.setdefault("status", {}))
        try:
            self.k.store.patch("Pod", self.ns, self.name, mutate)
            return True
        except NotFound:
            self.deleted.set()
            return False

    def _volumes(self) -> Dict[str, str]:
        vols = {}
        for v in (self.pod.get("spec") or {}).get("volumes") or []:
            name = v.get("name")
            if "hostPath" in v:
                path = v["hostPath"].get("path")
                if v["hostPath"].get("type") in ("DirectoryOrCreate", None, ""):
                    try:
                        os.makedirs(path, exist_ok=True)
                    except OSError:
                        pass
                vols[name] = path
            else:  # emptyDir / configMap / secret / anything else: a sandbox dir
                d = os.path.join(self.sandbox, "volumes", name)
                os.makedirs(d, exist_ok=True)
                vols[name] = d
        return vols

    def _mount(self, ctr: dict, vols: Dict[str, str]) -> Dict[str, str]:
        """Materialise the container's volumeMounts under sandbox/root; returns
        mountPath -> host path."""
        root = os.path.join(self.sandbox, "root")
        out = {}
        for m in ctr.get("volumeMounts") or []:
            src = vols.get(m.get("name"))
            if src is None:
                continue
            if m.get("subPath"):
                src = os.path.join(src, m["subPath"])
                os.makedirs(src, exist_ok=True)
            mp = m.get("mountPath") or ""
            link = os.path.join(root, mp.lstrip("/"))
            os.makedirs(os.path.dirname(link) or root, exist_ok=True)
            if os.path.islink(link) or os.path.exists(link):
                if os.path.islink(link):
                    os.unlink(link)
                else:
                    shutil.rmtree(link, ignore_errors=True)
            os.symlink(src, link)
            out[mp] = src
            if mp.startswith("/"):
                out[mp.rstrip("/")] = src
        return out

    # ------------------------------------------------------------ env
    def _container_hbm(self, ctr: dict) -> float:
        """This container's HBM cap in GB: its own ``kubedl.io/hbm-gb`` request,
        else an equal share of what is left of the pod's scheduled slice (the
        annotation is the SUM over containers, so exporting it whole to every
        container would let them together exceed the reservation)."""
        own = c.hbm_requested(ctr)
        if own:
            return own
        slice_gb = (self.pod["metadata"].get("annotations") or {}).get(HBM_ANNOTATION)
        if not slice_gb:
            return 0.0
        ctrs = (self.pod.get("spec") or {}).get("containers") or []
        asked = [c.hbm_requested(x) for x in ctrs]
        unset = sum(1 for a in asked if not a)
        return max(0.0, float(slice_gb) - sum(asked)) / max(1, unset)

    def _env(self, ctr: dict, mounts: Dict[str, str], cidx: str) -> Tuple[Dict[str, str], str]:
        env = {k: v for k, v in os.environ.items() if k not in _ENV_DENY}
        pp = env.get("PYTHONPATH", "")
        env["PYTHONPATH"] = REPO_ROOT + (os.pathsep + pp if pp else "")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        # node-level MIOpen perf/find db + kernel cache shared by every rank:
        # without it each job recompiles its conv kernels (~35 s of a 40 s job)
        env.setdefault("MIOPEN_USER_DB_PATH", os.path.join(REPO_ROOT, "miopen_db", "user"))
        env.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(REPO_ROOT, "miopen_db", "cache"))
        raw: Dict[str, str] = {}
        for e in ctr.get("env") or []:
            if "value" in e:
                raw[e["name"]] = str(e.get("value", ""))
            elif "valueFrom" in e:
                fr = ((e["valueFrom"] or {}).get("fieldRef") or {}).get("fieldPath", "")
                md = self.pod["metadata"]
                raw[e["name"]] = {"metadata.name": md["name"], "metadata.namespace": md["namespace"],
                                  "metadata.uid": md.get("uid", ""), "status.podIP": "127.0.0.1",
                                  "status.hostIP": "127.0.0.1",
                                  "spec.nodeName": self.pod["spec"].get("nodeName", "")}.get(fr, "")
        raw = self.k.resolver.resolve(self.ns, self.name, raw, self.pod)
        self.unresolved = self.k.resolver.unresolved(self.ns, raw)
        # paths that are mount points of this container -> their host directories
        for k, v in list(raw.items()):
            if v in mounts:
                raw[k] = mounts[v]
        env.update(raw)
        # GPU visibility: own GPU first (cuda:0, as in a pod), then the rest of
        # the gang's set (runtime/gpu_env.py); outside a gang only its own GPUs
        gang = [g for g in ((self.pod["metadata"].get("annotations") or {}).get(GANG_GPUS_ANNOTATION) or "")
                .split(",") if g]
        for k, v in rank_gpu_env(self.gpus, gang).items():
            if k == "HIP_VISIBLE_DEVICES" or k not in raw:  # an explicit container env LOCAL_* wins
                env[k] = v
        cpu = str(((ctr.get("resources") or {}).get("limits") or {}).get("cpu", ""))
        if cpu:  # honour a CPU limit the way a cgroup quota would bound intra-op threads
            n = float(cpu[:-1]) / 1000.0 if cpu.endswith("m") else float(cpu)
            env["OMP_NUM_THREADS"] = str(max(1, int(n)))
        md = self.pod["metadata"]
        labels = md.get("labels") or {}
        env["KDL_POD_NAME"] = self.name
        env["KDL_POD_NAMESPACE"] = self.ns
        env["KDL_POD_UID"] = self.uid
        env["KDL_JOB_NAME"] = labels.get(c.JOB_NAME_LABEL, "")
        env["KDL_REPLICA_TYPE"] = labels.get(c.REPLICA_TYPE_LABEL, "")
        env["KDL_REPLICA_INDEX"] = labels.get(c.REPLICA_INDEX_LABEL, "")
        env["KDL_SANDBOX"] = self.sandbox
        env["KDL_NUM_GPUS"] = str(len(self.gpus))
        # HBM slice of a shared GPU (scheduler annotation) or a per-process cap
        # asked on an exclusive GPU: the rank caps its caching allocator to it
        hbm = self._container_hbm(ctr)
        if hbm:
            env["KDL_HBM_LIMIT_GB"] = f"{hbm:g}"
        ready = os.path.join(self.sandbox, f"ready.{cidx}")
        env["KDL_READY_FILE"] = ready
        env["KDL_PROGRESS_FILE"] = os.path.join(self.sandbox, f"progress.{cidx}")
        # the node warm-up's lock: a rank waits on it after its Ready, before its
        # first communicator build (parallel/dist.py wait_node_warm) -- pods are
        # never held back from starting by the warm-up
        z = self.k.zygote
        if z is not None and z.warm_gpu is not None:
            env["KDL_NODE_WARM_LOCK"] = z.warm_lock
        return env, ready

    # ------------------------------------------------------------ process control
    def _spawn(self, cs: _Container, ctr: dict, vols: Dict[str, str], cidx: str) -> bool:
        mounts = self._mount(ctr, vols)
        root = os.path.join(self.sandbox, "root")
        wd = ctr.get("workingDir") or ""
        cwd = os.path.join(root, wd.lstrip("/")) if wd else root
        if wd and wd in mounts:
            cwd = mounts[wd]
        os.makedirs(cwd, exist_ok=True)
        env, ready = self._env(ctr, mounts, cidx)
        if self.unresolved and time.monotonic() < self.dns_hold_until:
            # a peer name no Service, Pod or replica spec of this job accounts for:
            # the rank would start with an address nothing on the node answers
            if not cs.dns_wait_logged:
                with open(cs.log_path, "a") as f:
                    f.write(f"[kdl-kubelet] {c.now()} holding {cs.name}: unresolved {self.unresolved}\n")
                cs.dns_wait_logged = True
            cs.next_start = time.monotonic() + 0.05
            return False
        if self.unresolved:
            with open(cs.log_path, "a") as f:
                f.write(f"[kdl-kubelet] {c.now()} starting {cs.name} with unresolved {self.unresolved}\n")
        try:
            os.unlink(ready)
        except FileNotFoundError:
            pass
        cs.ready_file = ready
        cs.ready_at = None
        nat = self.k.native
        try:
            argv, cs.readiness = images.resolve_argv(ctr, cwd, env.get("PATH", ""))
            # $(VAR) references in command/args (k8s dependent-variable expansion)
            argv = [images.expand_env_refs(a, env) for a in argv]
            with open(cs.log_path, "a") as f:
                f.write(f"[kdl-kubelet] {c.now()} start {cs.name} (restart {cs.restart_count}): "
                        f"{' '.join(argv)}\n")
            envl = [f"{k}={v}" for k, v in env.items()]
            pid = None
            z = self.k.zygote
            if z is not None and zygote_mod.eligible(argv) is not None:
                pid = z.launch(argv, env, cwd, cs.log_path)
                if pid is not None:
                    with open(cs.log_path, "a") as f:
                        f.write(f"[kdl-kubelet] forked from the pre-warmed zygote as pid {pid}\n")
            if pid is not None:
                cs.pid = pid
            elif nat is not None:
                cs.pid = nat.spawn(argv, envl, cwd, cs.log_path, cs.log_path)
            else:  # pragma: no cover
                import subprocess
                lf = open(cs.log_path, "a")
                cs.pid = subprocess.Popen(argv, env=env, cwd=cwd, stdout=lf, stderr=lf,
                                          start_new_session=True).pid
        except (OSError, ValueError) as e:
            code = 127 if isinstance(e, (FileNotFoundError, ValueError)) or getattr(e, "errno", 0) == 2 else 126
            with open(cs.log_path, "a") as f:
                f.write(f"[kdl-kubelet] {c.now()} failed to start {cs.name}: {e}\n")
            cs.pid = None
            cs.term = {"exitCode": code, "reason": "StartError", "message": str(e),
                       "startedAt": c.now(), "finishedAt": c.now()}
            return False
        cs.started_at = c.now()
        cs.term = None
        if cs.readiness == "start":
            cs.ready_at = cs.started_at
        return True

    def _kill(self, cs: _Container, sig: int) -> None:
        if cs.pid is not None and self.k.native is not None:
            self.k.native.kill_group(cs.pid, sig)
        elif cs.pid is not None:  # pragma: no cover
            try:
                os.killpg(cs.pid, sig)
            except ProcessLookupError:
                pass

    def _reap(self, conts: List[_Container]) -> List[Tuple[_Container, int]]:
        live = [cs for cs in conts if cs.pid is not None]
        if not live:
            return []
        by_pid = {cs.pid: cs for cs in live}
        out = []
        if self.k.native is not None:
            for pid, code in self.k.native.reap(list(by_pid)):
                out.append((by_pid[pid], code))
        else:  # pragma: no cover
            for pid, cs in by_pid.items():
                r, st = os.waitpid(pid, os.WNOHANG)
                if r == pid:
                    out.append((cs, os.waitstatus_to_exitcode(st) if st else 0))
        return out

    # ------------------------------------------------------------ status rendering
    def _container_status(self, cs: _Container) -> dict:
        st = {"name": cs.name, "image": cs.spec.get("image", ""), "restartCount": cs.restart_count,
              "ready": cs.term is None and cs.pid is not None and cs.ready_at is not None}
        if cs.term is not None:
            st["state"] = {"terminated": dict(cs.term)}
        elif cs.pid is not None:
            st["state"] = {"running": {"startedAt": cs.started_at}}
        else:
            st["state"] = {"waiting": {"reason": "ContainerCreating" if cs.restart_count == 0
                                       else "CrashLoopBackOff"}}
        if cs.last_term is not None:
            st["lastState"] = {"terminated": dict(cs.last_term)}
        return st

    def _publish(self, phase: str, init_done: bool, reason: Optional[str] = None,
                 init_statuses: Optional[List[dict]] = None) -> None:
        conts = self.containers
        all_ready = bool(conts) and all(self._container_status(cs)["ready"] for cs in conts)
        ready_times = [cs.ready_at for cs in conts if cs.ready_at]
        ready_ts = max(ready_times) if ready_times and all_ready else None

        def fn(st):
            st["phase"] = phase
            st["hostIP"] = "127.0.0.1"
            st["podIP"] = "127.0.0.1"
            st.setdefault("startTime", self.start_time)
            if reason:
                st["reason"] = reason
            st["containerStatuses"] = [self._container_status(cs) for cs in conts]
            if init_statuses is not None:
                st["initContainerStatuses"] = init_statuses
            conds = {x["type"]: x for x in st.get("conditions") or []}

            def setc(t, ok, ts=None):
                old = conds.get(t)
                s = "True" if ok else "False"
                if old is None or old.get("status") != s:
                    conds[t] = {"type": t, "status": s, "lastTransitionTime": ts or c.now()}
            setc("Initialized", init_done)
            setc("ContainersReady", all_ready, ready_ts)
            setc("Ready", all_ready, ready_ts)
            if all_ready and ready_ts:
                # first time every container was Ready: kept after the pod ends, so a
                # rank that finishes before the controller looks still has a launch time
                st.setdefault("readyTime", ready_ts)
            order = ["PodScheduled", "Initialized", "ContainersReady", "Ready"]
            st["conditions"] = [conds[t] for t in order if t in conds]
        self._patch_status(fn)

    # ------------------------------------------------------------ main
    def run(self) -> None:
        try:
            self._run()
        except Exception:
            log.exception("pod worker %s/%s crashed", self.ns, self.name)
        finally:
            self.k._worker_done(self)

    def _wait_peers_gone(self) -> None:
        """Gang teardown barrier: wait (bounded) until no other pod of this job
        is still terminating."""
        t_end = time.monotonic() + self.k.default_grace + 15.0
        while self.k.terminating_peers(self) and time.monotonic() < t_end:
            if self.deleted.wait(self.k.poll_interval * 5):
                return

    def _run(self) -> None:
        self._wait_peers_gone()
        if self.deleted.is_set():
            return
        os.makedirs(os.path.join(self.sandbox, "logs"), exist_ok=True)
        os.makedirs(os.path.join(self.sandbox, "root"), exist_ok=True)
        spec = self.pod.get("spec") or {}
        policy = spec.get("restartPolicy") or "Always"
        vols = self._volumes()
        logs = os.path.join(self.sandbox, "logs")
        self.containers = [_Container(ct, "", os.path.join(logs, f"{ct.get('name', i)}.log"))
                           for i, ct in enumerate(spec.get("containers") or [])]
        # ---- init containers (sequential, to completion)
        init_statuses = []
        for i, ict in enumerate(spec.get("initContainers") or []):
            ics = _Container(ict, "", os.path.join(logs, f"init-{ict.get('name', i)}.log"))
            while not self.deleted.is_set():
                ok = self._spawn(ics, ict, vols, f"init{i}")
                if not ok and ics.term is None:  # held on an unresolved peer name
                    self.deleted.wait(self.k.poll_interval)
                    continue
                code = ics.term["exitCode"] if not ok else self._wait_one(ics)
                if code is None:
                    return  # deleted while running
                term = {"exitCode": code, "reason": "Completed" if code == 0 else "Error",
                        "startedAt": ics.started_at or c.now(), "finishedAt": c.now()}
                if code == 0:
                    init_statuses.append({"name": ics.name, "ready": True, "restartCount": ics.restart_count,
                                          "state": {"terminated": term}})
                    break
                ics.last_term = term
                if policy == "Never":
                    init_statuses.append({"name": ics.name, "ready": False,
                                          "restartCount": ics.restart_count, "state": {"terminated": term}})
                    self._publish("Failed", False, reason="Init:Error", init_statuses=init_statuses)
                    return
                ics.restart_count += 1
                if self.deleted.wait(self.k.backoff(ics.restart_count)):
                    return
            if self.deleted.is_set():
                return
        # ---- main containers
        for i, cs in enumerate(self.containers):
            self._spawn(cs, cs.spec, vols, str(i))
        phase = "Running"
        self._publish(phase, True, init_statuses=init_statuses or None)
        last_pub = None
        while True:
            if self.deleted.is_set():
                self._terminate()
                return
            changed = False
            for cs, code in self._reap(self.containers):
                cs.pid = None
                reason = "Completed" if code == 0 else ("OOMKilled" if code == 137 else "Error")
                cs.term = {"exitCode": code, "reason": reason, "startedAt": cs.started_at,
                           "finishedAt": c.now()}
                if policy == "Always" or (policy == "OnFailure" and code != 0):
                    cs.last_term = cs.term
                    cs.restart_count += 1
                    cs.next_start = time.monotonic() + self.k.backoff(cs.restart_count)
                    cs.term = None
                changed = True
            for cs in self.containers:
                if cs.pid is None and cs.term is None and time.monotonic() >= cs.next_start:
                    self._spawn(cs, cs.spec, vols, str(self.containers.index(cs)))
                    changed = True
                if cs.pid is not None and cs.ready_at is None and cs.readiness == "file":
                    t = _read_ready(cs.ready_file)
                    if t is not None:
                        cs.ready_at = t
                        changed = True
            if all(cs.term is not None for cs in self.containers) and self.containers:
                ok = all(cs.term["exitCode"] == 0 for cs in self.containers)
                self._publish("Succeeded" if ok else "Failed", True)
                return
            if changed or last_pub is None:
                self._publish(phase, True)
                last_pub = time.monotonic()
            self.deleted.wait(self.k.poll_interval)

    def _wait_one(self, cs: _Container) -> Optional[int]:
        while not self.deleted.is_set():
            r = self._reap([cs])
            if r:
                cs.pid = None
                return r[0][1]
            self.deleted.wait(self.k.poll_interval)
        self._kill(cs, signal.SIGKILL)
        self._reap([cs])
        return None

    def _terminate(self) -> None:
        live = [cs for cs in self.containers if cs.pid is not None]
        for cs in live:
            self._kill(cs, signal.SIGTERM)
        deadline = time.monotonic() + self.grace
        while live and time.monotonic() < deadline:
            for cs, _ in self._reap(live):
                cs.pid = None
            live = [cs for cs in live if cs.pid is not None]
            if live:
                time.sleep(self.k.poll_interval)
        for cs in live:
            self._kill(cs, signal.SIGKILL)
        t_end = time.monotonic() + 5
        while live and time.monotonic() < t_end:
            for cs, _ in self._reap(live):
                cs.pid = None
            live = [cs for cs in live if cs.pid is not None]
            if live:
                time.sleep(self.k.poll_interval)


def _read_ready(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            d = json.load(f)
        t = d.get("ready_time")
        if t is None:
            return c.format_time(__import__("datetime").datetime.fromtimestamp(os.path.getmtime(path)))
        import datetime as _dt
        return c.format_time(_dt.datetime.fromtimestamp(float(t), _dt.timezone.utc))
    except (OSError, ValueError):
        return None


class ServiceResolver:
    """Local DNS: ``<svc>[.<ns>[.svc[.<domain>]]][:<port>]`` -> ``127.0.0.1[:<hostPort>]``.

    The reference's cluster-spec endpoints are headless-Service DNS names
    (``controllers/tensorflow/tensorflow.go:120-139``,
    ``pkg/job_controller/service.go:263-276``) that resolve whenever the peer's
    Service exists, however late.  Here a rank's env is rendered once, at spawn,
    so the names cannot depend on which Services / Pods happen to be in the
    store at that moment: every ``<job>-<rtype>-<i>`` of the owning job's replica
    specs (``i < replicas``; the names GenGeneralName gives its pods and
    services) is resolvable from the job object alone, and ``store.host_port``
    hands each ``(ns, name, port)`` one stable port whoever asks first -- the
    peer's Service or a rank that names it."""

    def __init__(self, store: Store, domain: Optional[str] = None):
        self.store = store
        self.domain = domain if domain is not None else os.environ.get("CUSTOM_CLUSTER_DOMAIN", "")

    def job_names(self, ns: str, pod: Optional[dict]) -> set:
        """Deterministic endpoint names of ``pod``'s controlling job."""
        if not pod:
            return set()
        from kubedl_amd.api import kinds as _kinds
        for ref in (pod.get("metadata") or {}).get("ownerReferences") or []:
            if not ref.get("controller"):
                continue
            job = self.store.try_get(ref.get("kind", ""), ns, ref.get("name", ""))
            if job is None:
                return set()
            jname = job["metadata"]["name"]
            out = set()
            for rt, spec in _kinds.replica_specs(job).items():
                n = (spec or {}).get("replicas")
                for i in range(1 if n is None else int(n)):
                    out.add(c.gen_general_name(jname, rt.lower(), i))
            return out
        return set()

    def _names(self, ns: str, pod: Optional[dict] = None) -> List[str]:
        names = {s["metadata"]["name"] for s in self.store.list("Service", ns)}
        names |= {p["metadata"]["name"] for p in self.store.list("Pod", ns)}
        names |= self.job_names(ns, pod)
        return sorted(names, key=len, reverse=True)

    def unresolved(self, ns: str, env: Dict[str, str]) -> List[str]:
        """Service DNS names (``<name>.<ns>.svc...``) still left in a rendered env:
        a peer this node cannot map to a port."""
        pat = re.compile("(?<![\\w.-])[a-z0-9]([-a-z0-9]*[a-z0-9])?\\." + re.escape(ns) + "\\.svc(?![\\w-])")
        return sorted({m.group(0) for k, v in env.items() if isinstance(v, str) for m in pat.finditer(v)})

    def resolve(self, ns: str, pod_name: str, env: Dict[str, str], pod: Optional[dict] = None) -> Dict[str, str]:
        names = self._names(ns, pod)
        if not names:
            return dict(env)
        alts = []
        for n in names:
            en = re.escape(n)
            variants = []
            if self.domain:
                variants.append(f"{en}\\.{re.escape(ns)}\\.svc\\.{re.escape(self.domain)}")
            variants += [f"{en}\\.{re.escape(ns)}\\.svc", f"{en}\\.{re.escape(ns)}", en]
            alts.append((n, "|".join(variants)))
        pat = re.compile("(?<![\\w.-])(" + "|".join(f"(?P<n{i}>{v})" for i, (_, v) in enumerate(alts))
                         + ")(?::(?P<port>\\d+))?(?![\\w.-])")

        def sub(m):
            idx = next(i for i in range(len(alts)) if m.group(f"n{i}") is not None)
            svc = alts[idx][0]
            if m.group("port"):
                return f"127.0.0.1:{self.store.host_port(ns, svc, int(m.group('port')))}"
            return "127.0.0.1"

        out = {}
        for k, v in env.items():
            out[k] = pat.sub(sub, v) if isinstance(v, str) and k != "MASTER_PORT" else v
        # MASTER_ADDR/MASTER_PORT travel together (PyTorch/XGBoost env)
        addr = env.get("MASTER_ADDR")
        if addr is not None and env.get("MASTER_PORT", "").isdigit():
            svc = None
            if addr in ("localhost", "127.0.0.1"):
                svc = pod_name
            else:
                host = addr.split(".", 1)[0]
                if host in names:
                    svc = host
            if svc is not None:
                out["MASTER_ADDR"] = "127.0.0.1"
                out["MASTER_PORT"] = str(self.store.host_port(ns, svc, int(env["MASTER_PORT"])))
        return out


class Kubelet:
    def __init__(self, store: Store, root: str, node_name: str = "localhost",
                 poll_interval: float = 0.01, default_grace: float = 5.0,
                 backoff_base: float = 1.0, backoff_max: float = 30.0, zygote: Optional[bool] = None,
                 gpus: Optional[int] = None):
        """``gpus``: the node's GPU inventory size (None: unknown, warm-up on GPU
        0); the node warm-up runs on its LAST GPU -- the allocator hands GPUs
        out from 0 (``warm_gpu``).  No pod waits for it to start: every rank
        gets ``KDL_NODE_WARM_LOCK`` and waits on it after its Ready, before
        its first communicator build."""
        self.store = store
        self.root = root
        self.node = node_name
        self.poll_interval = poll_interval
        self.default_grace = default_grace
        self.backoff_base = float(os.environ.get("KDL_RESTART_BACKOFF_BASE", backoff_base))
        self.backoff_max = backoff_max
        self.dns_hold_s = 30.0
        self.native = _spawner()
        self.resolver = ServiceResolver(store)
        self._workers: Dict[str, PodWorker] = {}
        self._lock = threading.Lock()
        self.on_worker_done = None  # callback(uid) once a pod's processes are gone
        os.makedirs(os.path.join(root, "pods"), exist_ok=True)
        self._cancel = None
        if zygote is None:
            zygote = os.environ.get("KDL_ZYGOTE", "1") != "0"
        self.warm_gpu = (gpus - 1 if gpus > 0 else None) if gpus is not None else 0
        self.zygote = zygote_mod.ZygoteClient(root, self.native, warm_gpu=self.warm_gpu) \
            if (zygote and self.native is not None) else None

    def backoff(self, n: int) -> float:
        return min(self.backoff_base * (2 ** max(0, n - 1)), self.backoff_max)

    def start(self) -> None:
        if self.zygote is not None:
            env = {k: v for k, v in os.environ.items() if k not in _ENV_DENY}
            env["PYTHONPATH"] = REPO_ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
            self.zygote.start(env)
        self._cancel = self.store.watch(self._on_event, kind="Pod")
        for p in self.store.list("Pod"):
            self._maybe_start(p)

    def stop(self, kill: bool = True) -> None:
        if self._cancel:
            self._cancel()
        with self._lock:
            workers = list(self._workers.values())
        if kill:
            for w in workers:
                w.grace = min(w.grace, 2.0)
                w.deleted.set()
            for w in workers:
                w.join(timeout=10)
        if self.zygote is not None:
            self.zygote.stop()

    def _on_event(self, etype: str, pod: dict) -> None:
        if etype == DELETED:
            with self._lock:
                w = self._workers.get(pod["metadata"].get("uid", ""))
            if w is not None:
                w.deleted.set()
            return
        if etype in (ADDED, MODIFIED):
            self._maybe_start(pod)

    def _maybe_start(self, pod: dict) -> None:
        if (pod.get("spec") or {}).get("nodeName") != self.node:
            return
        if (pod.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
            return
        uid = pod["metadata"].get("uid", "")
        with self._lock:
            if uid in self._workers or uid in getattr(self, "_done", set()):
                return
            w = PodWorker(self, pod)
            self._workers[uid] = w
        w.start()

    def _worker_done(self, w: PodWorker) -> None:
        with self._lock:
            self._workers.pop(w.uid, None)
            if not hasattr(self, "_done"):
                self._done = set()
            self._done.add(w.uid)
        cb = self.on_worker_done
        if cb is not None:
            cb(w.uid)

    def holds(self, uid: str) -> bool:
        """Whether the pod ``uid`` still has a worker (live or terminating processes)."""
        with self._lock:
            return uid in self._workers

    def terminating_peers(self, w: PodWorker) -> List[str]:
        if not w.job_label:
            return []
        with self._lock:
            return [o.name for o in self._workers.values()
                    if o is not w and o.deleted.is_set() and o.ns == w.ns and o.job_label == w.job_label]

    def running_pods(self) -> List[str]:
        with self._lock:
            return [f"{w.ns}/{w.name}" for w in self._workers.values()]

    def log_path(self, ns: str, name: str, container: Optional[str] = None) -> Optional[str]:
        pod = self.store.try_get("Pod", ns, name)
        if pod is None:
            return None
        sb = os.path.join(self.root, "pods", f"{ns}_{name}_{pod['metadata'].get('uid', '')[:8]}", "logs")
        ctrs = (pod.get("spec") or {}).get("containers") or []
        cname = container or (ctrs[0].get("name") if ctrs else "main")
        return os.path.join(sb, f"{cname}.log")
