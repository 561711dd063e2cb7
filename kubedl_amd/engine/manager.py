"""Controller manager: wires store, controllers, gang scheduling, metrics,
persistence and the local MI355X node runtime into one process.

Reference ``main.go:48-115``: parse flags, build the manager, register
schemes, gang schedulers, workload controllers (gated by ``--workloads``),
storage backends and persist controllers, start the metrics endpoint, run.
Controller-runtime's informers + work queues become store watches feeding a
``RateLimitingQueue`` per workload kind with ``max_concurrent_reconciles``
worker threads (one key is never reconciled by two workers at once).
"""
from __future__ import annotations

import logging
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from kubedl_amd.api import common as c
from kubedl_amd.api import kinds as K
from kubedl_amd.controllers import RECONCILERS
from kubedl_amd.controllers.workloadgate import is_workload_enable
from kubedl_amd.engine.job_controller import JobControllerConfig
from kubedl_amd.engine.workqueue import RateLimitingQueue
from kubedl_amd.gang import interface as gang_iface
from kubedl_amd.gang.allocator import GPUAllocator, GPUInventory, detect_gpus
from kubedl_amd.metrics.job_metrics import MetricsRegistry
from kubedl_amd.store import ADDED, DELETED, MODIFIED, EventRecorder, Store
from kubedl_amd.utils.log import logger_for_key
from kubedl_amd.utils.trace import trace_range

log = logging.getLogger("kubedl_amd.manager")


@dataclass
class ManagerOptions:
    home: str = field(default_factory=lambda: os.environ.get("KDL_HOME", os.path.expanduser("~/.kubedl_amd")))
    durable: bool = False                 # sqlite-backed store under home
    workloads: str = "auto"               # --workloads
    gang_scheduler_name: str = ""         # --gang-scheduler-name (enables gang when non-empty)
    max_reconciles: int = 1               # --max-reconciles (<=0 -> 1)
    metrics_port: int = 0                 # --metrics-addr port (0 = no HTTP endpoint)
    metrics_host: str = "127.0.0.1"       # --metrics-addr host part ("" = every interface, as Go's ":8443")
    controller_metrics_port: int = 0      # --controller-metrics-addr port (controller-runtime metrics)
    controller_metrics_host: str = "127.0.0.1"
    leader_election: bool = False         # --enable-leader-election (the CLI defaults it on, main.go:56)
    leader_wait_s: Optional[float] = None  # standby: how long to wait for leadership (None = forever)
    run_node: bool = True                 # run the local node runtime (scheduler + kubelet)
    gpus: Optional[int] = None            # override GPU inventory
    object_storage: str = ""              # --object-storage (e.g. "sqlite")
    event_storage: str = ""               # --event-storage (e.g. "jsonl")
    region: str = field(default_factory=lambda: os.environ.get("REGION", ""))
    starvation_s: float = 30.0


class _KindLoop:
    def __init__(self, mgr: "Manager", reconciler, workers: int):
        self.mgr = mgr
        self.r = reconciler
        self.name = reconciler.kind.lower()  # controller-runtime names the controller after the kind
        self.queue = RateLimitingQueue()
        cm = mgr.controller_metrics
        cm.queues[self.name] = lambda: len(self.queue)
        self.threads = [threading.Thread(target=self._work, name=f"reconcile-{reconciler.kind}-{i}",
                                         daemon=True) for i in range(max(1, workers))]
        self.errors: List[str] = []

    def start(self):
        for t in self.threads:
            t.start()

    def _work(self):
        while True:
            key, shutdown = self.queue.get()
            if shutdown:
                return
            if key is None:
                continue
            ns, name = key.split("/", 1)
            cm = self.mgr.controller_metrics
            t0 = time.perf_counter()
            try:
                with trace_range(f"reconcile {self.r.kind} {key}"):
                    res = self.r.reconcile(ns, name)
                self.queue.forget(key)
                if res.requeue_after > 0:
                    self.queue.add_after(key, res.requeue_after)
                    result = "requeue_after"
                elif res.requeue:
                    self.queue.add_rate_limited(key)
                    cm.queue_retries.labels(self.name).inc()
                    result = "requeue"
                else:
                    result = "success"
            except Exception as e:  # reconcile error -> rate-limited retry (controller-runtime)
                logger_for_key(key, log).warning("reconcile %s failed: %s", self.r.kind, e)
                self.errors.append(f"{key}: {e}")
                self.queue.add_rate_limited(key)
                cm.queue_retries.labels(self.name).inc()
                result = "error"
            finally:
                self.queue.done(key)
            cm.observe_reconcile(self.name, time.perf_counter() - t0, result)

    def add(self, key: str) -> None:
        self.mgr.controller_metrics.queue_adds.labels(self.name).inc()
        self.queue.add(key)


class Manager:
    def __init__(self, opts: Optional[ManagerOptions] = None, store: Optional[Store] = None,
                 metrics: Optional[MetricsRegistry] = None):
        self.opts = opts or ManagerOptions()
        os.makedirs(self.opts.home, exist_ok=True)
        # leader election first: a standby opens neither the store nor the node
        # runtime until it holds the lease (engine/leader.py)
        self.leader = None
        if self.opts.leader_election:
            from kubedl_amd.engine.leader import LeaderLock
            self.leader = LeaderLock(self.opts.home)
            if not self.leader.acquire(timeout=self.opts.leader_wait_s):
                raise TimeoutError(f"not leader: {self.leader.path} held by "
                                   f"{self.leader.holder().get('holderIdentity', '?')}")
        from kubedl_amd.metrics.controller_metrics import ControllerMetrics
        self.controller_metrics = ControllerMetrics()
        db = os.path.join(self.opts.home, "store.db") if self.opts.durable else None
        self.store = store or Store(db)
        self.recorder = EventRecorder(self.store)
        self.metrics = metrics or MetricsRegistry()
        self.metrics.lister = lambda kind: self.store.list(kind)
        # gang schedulers (registry.RegisterGangSchedulers)
        gang_iface.register_gang_schedulers(self.store)
        gang = gang_iface.get(self.opts.gang_scheduler_name) if self.opts.gang_scheduler_name else None
        if self.opts.gang_scheduler_name and gang is None:
            raise ValueError(f"unknown gang scheduler {self.opts.gang_scheduler_name!r}; "
                             f"registered: {gang_iface.names()}")
        cfg = JobControllerConfig(enable_gang_scheduling=gang is not None,
                                  gang_scheduler_name=self.opts.gang_scheduler_name,
                                  max_concurrent_reconciles=max(1, self.opts.max_reconciles))
        self.loops: Dict[str, _KindLoop] = {}
        self.reconcilers = {}
        for info in K.ALL_KINDS:
            if not is_workload_enable(info.kind, self.opts.workloads):
                log.info("workload %s disabled", info.kind)
                continue
            r = RECONCILERS[info.kind](self.store, self.recorder, self.metrics, cfg, gang)
            self.reconcilers[info.kind] = r
            self.loops[info.kind] = _KindLoop(self, r, cfg.max_concurrent_reconciles)
        self._cancel = self.store.watch(self._on_event)
        # node runtime
        self.allocator = None
        self.scheduler = None
        self.kubelet = None
        if self.opts.run_node:
            from kubedl_amd.runtime.kubelet import Kubelet
            from kubedl_amd.runtime.scheduler import NodeScheduler
            inv = GPUInventory(self.opts.gpus) if self.opts.gpus is not None else detect_gpus()
            self.allocator = GPUAllocator(inv)
            self.scheduler = NodeScheduler(self.store, self.allocator, starvation_s=self.opts.starvation_s,
                                           metrics=self.metrics)
            self.kubelet = Kubelet(self.store, os.path.join(self.opts.home, "node"), gpus=inv.count)
            self.scheduler.holder = self.kubelet.holds
            self.kubelet.on_worker_done = self.scheduler.wake
        # persistence (controllers/persist)
        self.persist = None
        if self.opts.object_storage or self.opts.event_storage:
            from kubedl_amd.persist.controller import PersistController
            self.persist = PersistController(self.store, self.opts.home, self.opts.object_storage,
                                             self.opts.event_storage, self.opts.region)
        self.http = None
        self.ctrl_http = None
        self._started = False

    # ------------------------------------------------------------ events -> queues
    def _on_event(self, etype: str, obj: dict) -> None:
        kind = obj.get("kind")
        if kind in self.loops:
            md = obj["metadata"]
            key = f"{md['namespace']}/{md['name']}"
            if etype == ADDED:
                self.reconcilers[kind].on_owner_create(obj)
            self.loops[kind].add(key)
        elif kind in ("Pod", "Service"):
            for k, r in self.reconcilers.items():
                key = r.on_dependent_event(etype, obj)
                if key is not None:
                    self.loops[k].add(key)

    # ------------------------------------------------------------ lifecycle
    def start(self) -> "Manager":
        if self._started:
            return self
        self._started = True
        for loop in self.loops.values():
            loop.start()
        # reconcile everything already in a durable store
        for kind, loop in self.loops.items():
            for j in self.store.list(kind):
                if not c.is_created(j.get("status") or {}):
                    self.reconcilers[kind].on_owner_create(j)
                loop.add(f"{j['metadata']['namespace']}/{j['metadata']['name']}")
        if self.scheduler:
            self.scheduler.start()
        if self.kubelet:
            self.kubelet.start()
        if self.persist:
            self.persist.start()
        from kubedl_amd.metrics import start_monitoring
        if self.opts.metrics_port:
            self.http = start_monitoring(self.opts.metrics_port, self.metrics, self.opts.metrics_host)
        if self.opts.controller_metrics_port:
            self.ctrl_http = start_monitoring(self.opts.controller_metrics_port, self.controller_metrics,
                                              self.opts.controller_metrics_host)
        return self

    def stop(self) -> None:
        for loop in self.loops.values():
            loop.queue.shutdown()
        if self.kubelet:
            self.kubelet.stop()
        if self.scheduler:
            self.scheduler.stop()
        if self.persist:
            self.persist.stop()
        self._cancel()
        for srv in (self.http, self.ctrl_http):
            if srv is not None:
                try:
                    srv.shutdown()
                    srv.server_close()
                except Exception:
                    pass
        self.store.close()
        if self.leader is not None:
            self.leader.release()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # ------------------------------------------------------------ client API
    def apply(self, manifest: dict) -> dict:
        """Create a job (kubectl apply of a new object); validates and defaults."""
        import copy as _copy
        obj = _copy.deepcopy(manifest)
        if obj.get("kind") in K.BY_KIND:
            errs = K.validate(obj)
            if errs:
                raise ValueError("; ".join(errs))
            # [NEW] persist the defaulted spec (the reference defaults a cached
            # copy on every reconcile and never stores it)
            K.set_defaults(obj)
        obj.setdefault("metadata", {}).setdefault("namespace", "default")
        return self.store.create(obj)

    def get(self, kind: str, namespace: str, name: str) -> dict:
        return self.store.get(K.lookup(kind).kind if kind not in ("Pod", "Service", "Event", "PodGroup")
                              else kind, namespace, name)

    def delete(self, kind: str, namespace: str, name: str) -> None:
        k = K.lookup(kind).kind if kind not in ("Pod", "Service", "Event", "PodGroup") else kind
        self.store.delete(k, namespace, name)

    def wait_for(self, kind: str, namespace: str, name: str,
                 pred: Callable[[dict], bool], timeout: float = 60.0, interval: float = 0.02) -> dict:
        deadline = time.time() + timeout
        last = None
        while time.time() < deadline:
            last = self.store.try_get(kind, namespace, name)
            if last is not None and pred(last):
                return last
            time.sleep(interval)
        raise TimeoutError(f"{kind} {namespace}/{name} did not reach the expected state in {timeout}s; "
                           f"last status: {(last or {}).get('status')}")

    def wait_for_condition(self, kind: str, namespace: str, name: str, ctypes, timeout: float = 60.0):
        if isinstance(ctypes, str):
            ctypes = (ctypes,)
        return self.wait_for(kind, namespace, name,
                             lambda j: any(c.has_condition(j.get("status") or {}, t) for t in ctypes),
                             timeout=timeout)

    def idle(self) -> bool:
        return all(loop.queue.idle() for loop in self.loops.values())
