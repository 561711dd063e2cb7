"""Node scheduler: binds pending pods to this MI355X node's GPUs.

Replaces kube-scheduler + kube-batch for one node:

* a pod requests ``amd.com/gpu`` (or ``nvidia.com/gpu`` for unchanged
  specs) per container; 0-GPU pods always fit;
* pods bound to a gang (``spec.schedulerName`` = a registered gang scheduler
  and the ``scheduling.k8s.io/group-name`` annotation) are admitted
  all-or-nothing: only when ``PodGroup.spec.minMember`` members exist AND the
  allocator can reserve every member's GPUs at once (``GPUAllocator``);
  otherwise nothing is reserved and the pods stay Pending with
  ``PodScheduled=False, reason=Unschedulable``;
* queue order is FIFO by creation time with backfill: a later gang that fits
  in the currently free GPUs may start while the head waits, until the head
  has waited ``starvation_s`` -- then backfill stops so big gangs cannot starve;
* a pod asking for ``kubedl.io/hbm-gb`` and no whole GPU gets an HBM slice
  of a shared GPU (``GPUAllocator``); its binding also carries
  ``kubedl.io/hbm-gb``;
* binding writes ``spec.nodeName``, the ``kubedl.io/gpus`` annotation and the
  ``PodScheduled`` condition; GPUs return to the pool when the pod reaches a
  terminal phase, or when it is deleted AND the kubelet no longer holds its
  processes (``holder``): a rank being torn down keeps its GPU until it has
  exited, so a gang restart never overlaps old and new ranks on one device;
* a scheduling unit's queue age is the owning job's creation time
  (``kubedl.io/queue-time``), so a gang re-admitted after a restart keeps its
  place in the FIFO instead of queueing behind later jobs.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Dict, List, Optional, Tuple

from kubedl_amd.api import common as c
from kubedl_amd.gang import interface as gang_iface
from kubedl_amd.gang.allocator import GPUAllocator
from kubedl_amd.gang.local import GROUP_ANNOTATION
from kubedl_amd.store import ADDED, DELETED, MODIFIED, NotFound, Store

log = logging.getLogger("kubedl_amd.scheduler")

GPU_ANNOTATION = "kubedl.io/gpus"
GANG_GPUS_ANNOTATION = "kubedl.io/gang-gpus"  # the gang's GPU set on this node (runtime/gpu_env.py)
HBM_ANNOTATION = "kubedl.io/hbm-gb"
NODE_NAME = "localhost"


def pod_key(pod: dict) -> str:
    md = pod["metadata"]
    return f"{md['namespace']}/{md['name']}/{md.get('uid', '')}"


def pod_gpus(pod: dict) -> int:
    return c.pod_template_gpus({"spec": pod.get("spec") or {}})


def pod_hbm(pod: dict) -> float:
    return c.pod_template_hbm({"spec": pod.get("spec") or {}})


QUEUE_TIME_ANNOTATION = "kubedl.io/queue-time"


def _queue_age(pod: dict) -> float:
    md = pod["metadata"]
    t = c.to_epoch((md.get("annotations") or {}).get(QUEUE_TIME_ANNOTATION))
    return t if t is not None else (c.to_epoch(md.get("creationTimestamp")) or 0)


def is_terminal(pod: dict) -> bool:
    return (pod.get("status") or {}).get("phase") in ("Succeeded", "Failed")


class NodeScheduler:
    def __init__(self, store: Store, allocator: GPUAllocator, node_name: str = NODE_NAME,
                 starvation_s: float = 30.0, metrics=None):
        self.store = store
        self.alloc = allocator
        self.node = node_name
        self.starvation_s = starvation_s
        self.metrics = metrics
        self._wake = threading.Event()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._owner_of_pod: Dict[str, str] = {}
        self._unsched_marked: set = set()
        self._lock = threading.Lock()
        # uid -> still has processes (kubelet.holds); deleted pods' GPUs wait for it
        self.holder = None
        self._deferred: Dict[str, dict] = {}
        self._cancel = store.watch(self._on_event)

    # ------------------------------------------------------------ lifecycle
    def start(self) -> None:
        self._thread = threading.Thread(target=self._loop, name="kdl-scheduler", daemon=True)
        self._thread.start()
        self._wake.set()

    def stop(self) -> None:
        self._stop.set()
        self._wake.set()
        self._cancel()
        if self._thread:
            self._thread.join(timeout=5)

    def _on_event(self, etype: str, obj: dict) -> None:
        kind = obj.get("kind")
        if kind == "Pod":
            if etype == DELETED and self.holder is not None and self.holder(obj["metadata"].get("uid", "")):
                with self._lock:
                    self._deferred[pod_key(obj)] = obj
            elif etype == DELETED or (etype == MODIFIED and is_terminal(obj)):
                self._release(obj)
            self._wake.set()
        elif kind == "PodGroup":
            self._wake.set()

    def _release(self, pod: dict) -> None:
        k = pod_key(pod)
        with self._lock:
            owner = self._owner_of_pod.pop(k, None)
            self._unsched_marked.discard(k)
        if owner is not None:
            self.alloc.release(owner, k)
            if self.metrics is not None:
                self.metrics.gpus_allocated.set(self.alloc.used())
            self._wake.set()

    def wake(self, uid: str = "") -> None:
        """Kubelet callback: a pod's processes are gone (its deferred GPUs can go back)."""
        self._wake.set()

    def _release_deferred(self) -> None:
        with self._lock:
            items = list(self._deferred.items())
        for k, pod in items:
            if self.holder is None or not self.holder(pod["metadata"].get("uid", "")):
                with self._lock:
                    self._deferred.pop(k, None)
                self._release(pod)

    def _loop(self) -> None:
        while not self._stop.is_set():
            self._wake.wait(timeout=1.0)
            self._wake.clear()
            if self._stop.is_set():
                break
            self._release_deferred()
            try:
                self.schedule_once()
            except Exception:
                log.exception("schedule pass failed")

    # ------------------------------------------------------------ one pass
    def _units(self) -> List[Tuple[float, str, List[dict], int]]:
        """Pending scheduling units: (age key, owner, pods-to-bind, min members)."""
        pods = self.store.list("Pod")
        gangs: Dict[str, List[dict]] = {}
        singles: List[dict] = []
        for p in pods:
            if p["metadata"].get("deletionTimestamp") or is_terminal(p):
                continue
            sched = (p.get("spec") or {}).get("schedulerName")
            grp = (p["metadata"].get("annotations") or {}).get(GROUP_ANNOTATION)
            if grp and sched and gang_iface.get(sched) is not None:
                gangs.setdefault(f"{p['metadata']['namespace']}/{grp}", []).append(p)
            elif not (p.get("spec") or {}).get("nodeName"):
                singles.append(p)
        units = []
        for gkey, members in gangs.items():
            unbound = [p for p in members if not (p.get("spec") or {}).get("nodeName")]
            if not unbound:
                continue
            ns, name = gkey.split("/", 1)
            pg = self.store.try_get("PodGroup", ns, name)
            min_member = int(((pg or {}).get("spec") or {}).get("minMember", len(members)))
            age = min(_queue_age(p) for p in members)
            units.append((age, "gang:" + gkey, unbound, min_member if len(members) < min_member else 0))
        for p in singles:
            age = _queue_age(p)
            units.append((age, "pod:" + pod_key(p), [p], 0))
        units.sort(key=lambda u: u[0])
        return units

    def schedule_once(self) -> int:
        bound = 0
        units = self._units()
        head_blocked_since = None
        now = time.time()
        for age, owner, pods, missing in units:
            if missing:
                # gang incomplete: wait for all minMember pods to exist
                self._mark_unschedulable(pods, f"PodGroup has fewer than {missing} members")
                continue
            if head_blocked_since is not None and now - head_blocked_since > self.starvation_s:
                self._mark_unschedulable(pods, "waiting behind an older gang (FIFO after starvation)")
                continue
            try:
                req = {pod_key(p): pod_gpus(p) for p in pods}
                hbm = {pod_key(p): pod_hbm(p) for p in pods}
                alloc = self.alloc.allocate(owner, req, hbm)
            except (ValueError, TypeError) as e:
                # a malformed request (e.g. kubedl.io/hbm-gb: "lots") fails only its
                # own unit; the rest of the pass keeps scheduling
                self._mark_unschedulable(pods, f"invalid resource request: {e}")
                continue
            if alloc is None:
                free = len(self.alloc.free)
                want_hbm = sum(v for k, v in hbm.items() if not req[k])
                self._mark_unschedulable(
                    pods, f"0/1 nodes available: insufficient amd.com/gpu (need {sum(req.values())}, "
                          f"{free}/{self.alloc.inv.count} free)"
                          + (f" or kubedl.io/hbm-gb (need {want_hbm:g} GB in slices, "
                             f"max free on a GPU {max(self.alloc.hbm_free().values(), default=0):g} GB)"
                             if want_hbm else ""))
                if head_blocked_since is None:
                    head_blocked_since = age
                continue
            gang_gpus = None
            if owner.startswith("gang:"):
                gang_gpus = sorted({g for k in alloc.pods for g in alloc.pods[k]})
                if len(gang_gpus) < 2:
                    gang_gpus = None
            for p in pods:
                k = pod_key(p)
                if self._bind(p, alloc.pods.get(k, []), alloc.slices.get(k), gang_gpus):
                    with self._lock:
                        self._owner_of_pod[k] = owner
                        self._unsched_marked.discard(k)
                    bound += 1
                else:
                    self.alloc.release(owner, k)
            if owner.startswith("gang:"):
                ns, name = owner[5:].split("/", 1)
                self._set_group_phase(ns, name, "Running")
        if self.metrics is not None:
            self.metrics.gpus_allocated.set(self.alloc.used())
        return bound

    def _bind(self, pod: dict, gpus: List[int], hbm_slice: Optional[float] = None,
              gang_gpus: Optional[List[int]] = None) -> bool:
        md = pod["metadata"]
        ts = c.now()

        def mutate(o):
            if o["metadata"].get("uid") != md.get("uid"):
                raise NotFound("pod replaced")
            o.setdefault("spec", {})["nodeName"] = self.node
            ann = o["metadata"].setdefault("annotations", {})
            ann[GPU_ANNOTATION] = ",".join(map(str, gpus))
            if hbm_slice is not None:
                ann[HBM_ANNOTATION] = f"{hbm_slice:g}"
            if gang_gpus is not None and len(gpus) == 1:
                ann[GANG_GPUS_ANNOTATION] = ",".join(map(str, gang_gpus))
            else:
                ann.pop(GANG_GPUS_ANNOTATION, None)
            st = o.setdefault("status", {})
            conds = [x for x in st.get("conditions") or [] if x.get("type") != "PodScheduled"]
            conds.append({"type": "PodScheduled", "status": "True", "lastTransitionTime": ts})
            st["conditions"] = conds
        try:
            self.store.patch("Pod", md["namespace"], md["name"], mutate)
            return True
        except NotFound:
            return False

    def _mark_unschedulable(self, pods: List[dict], msg: str) -> None:
        for p in pods:
            k = pod_key(p)
            with self._lock:
                if k in self._unsched_marked:
                    continue
                self._unsched_marked.add(k)
            md = p["metadata"]
            ts = c.now()

            def mutate(o, msg=msg, ts=ts):
                st = o.setdefault("status", {})
                conds = [x for x in st.get("conditions") or [] if x.get("type") != "PodScheduled"]
                conds.append({"type": "PodScheduled", "status": "False", "reason": "Unschedulable",
                              "message": msg, "lastTransitionTime": ts})
                st["conditions"] = conds
            try:
                self.store.patch("Pod", md["namespace"], md["name"], mutate)
            except NotFound:
                pass

    def _set_group_phase(self, ns: str, name: str, phase: str) -> None:
        def mutate(o):
            o.setdefault("status", {})["phase"] = phase
        try:
            self.store.patch("PodGroup", ns, name, mutate)
        except NotFound:
            pass
