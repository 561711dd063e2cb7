"""Prometheus job metrics with the reference's names and labels.

``pkg/metrics/job_metrics.go:32-194`` + ``status_counter.go:31-84``:

=========================================  =========  =================================
metric                                      type       labels
=========================================  =========  =================================
kubedl_jobs_created                         counter    kind (lower-cased)
kubedl_jobs_deleted                         counter    kind
kubedl_jobs_successful                      counter    kind
kubedl_jobs_failed                          counter    kind
kubedl_jobs_restarted                       counter    kind
kubedl_jobs_running                         gauge      kind (const label; computed on scrape)
kubedl_jobs_pending                         gauge      kind (Created is the only condition)
kubedl_jobs_first_pod_launch_delay_seconds  histogram  kind (NOT lower-cased), name, namespace, uid
kubedl_jobs_all_pods_launch_delay_seconds   histogram  kind, name, namespace, uid
=========================================  =========  =================================

[NEW] ``kdl_job_steps_per_second`` gauge (per job, from rank progress files)
and ``kdl_gpus_allocated`` gauge (gang allocator).

Launch delay: "pod Ready" is the rank process having signalled readiness
(``KDL_READY_FILE`` written after its process group is up); the histogram
value is ``ready_time - job.creationTimestamp`` exactly like the reference's
``PodReady.lastTransitionTime - creationTimestamp``.
"""
from __future__ import annotations

import threading
from typing import Callable, Dict, List, Optional

from prometheus_client import CollectorRegistry, Gauge, Histogram
from prometheus_client.core import GaugeMetricFamily

from kubedl_amd.api import common as c
from kubedl_amd.metrics.exposition import BareCounterVec

# The reference's two launch-delay histograms use the Go client's default
# buckets (prometheus.DefBuckets; pkg/metrics/job_metrics.go:53-60 sets none);
# their ``le`` boundaries are visible to scrapers, so they are kept exactly.
# (Python's client default adds .075/.75/7.5 -- not the same set.)
GO_DEF_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, float("inf"))
# Finer local-node buckets (rank launch is sub-second warm, seconds cold, up to
# minutes for a gang waiting on GPUs) under a separately named kdl_* metric
# with bounded labels {kind, phase}.
FINE_DELAY_BUCKETS = (0.05, 0.1, 0.2, 0.3, 0.5, 0.75, 1.0, 1.5, 2.0, 3.0, 5.0, 7.5, 10.0, 15.0, 30.0, 60.0,
                      120.0, 300.0, float("inf"))


class _StatusGauges:
    """Custom collector: running/pending computed on scrape by listing jobs
    (JobStatusCounter semantics: a full list per kind per scrape)."""

    def __init__(self, owner: "MetricsRegistry"):
        self.owner = owner

    def collect(self):
        running = GaugeMetricFamily("kubedl_jobs_running", "Counts number of jobs running currently",
                                    labels=["kind"])
        pending = GaugeMetricFamily("kubedl_jobs_pending", "Counts number of jobs pending currently",
                                    labels=["kind"])
        for kind in sorted(self.owner.kinds):
            lister = self.owner.lister
            jobs = lister(kind) if lister else []
            nrun = sum(1 for j in jobs if c.is_running(j.get("status") or {}))
            npend = sum(1 for j in jobs
                        if c.is_created(j.get("status") or {})
                        and len((j.get("status") or {}).get("conditions") or []) == 1)
            running.add_metric([kind.lower()], nrun)
            pending.add_metric([kind.lower()], npend)
        yield running
        yield pending


class MetricsRegistry:
    def __init__(self, registry: Optional[CollectorRegistry] = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        # client_golang CounterVecs: exported under these exact names (no _total / _created)
        self.created = BareCounterVec("kubedl_jobs_created", "Counts number of jobs created", ["kind"], registry=r)
        self.deleted = BareCounterVec("kubedl_jobs_deleted", "Counts number of jobs deleted", ["kind"], registry=r)
        self.success = BareCounterVec("kubedl_jobs_successful", "Counts number of jobs successfully finished",
                                      ["kind"], registry=r)
        self.failure = BareCounterVec("kubedl_jobs_failed", "Counts number of jobs failed", ["kind"], registry=r)
        self.restart = BareCounterVec("kubedl_jobs_restarted", "Counts number of jobs restarted", ["kind"],
                                      registry=r)
        self.first_pod_delay = Histogram(
            "kubedl_jobs_first_pod_launch_delay_seconds",
            "Histogram for recording launch delay duration(from job created to first pod running).",
            ["kind", "name", "namespace", "uid"], registry=r, buckets=GO_DEF_BUCKETS)
        self.all_pods_delay = Histogram(
            "kubedl_jobs_all_pods_launch_delay_seconds",
            "Histogram for recording sync launch delay duration(from job created to all pods running).",
            ["kind", "name", "namespace", "uid"], registry=r, buckets=GO_DEF_BUCKETS)
        self.launch_delay_fine = Histogram(
            "kdl_jobs_launch_delay_seconds",
            "Launch delay (job created -> first / all ranks Ready) in local-node buckets; phase = first | all.",
            ["kind", "phase"], registry=r, buckets=FINE_DELAY_BUCKETS)
        self.steps_per_sec = Gauge("kdl_job_steps_per_second", "Training steps/s reported by rank 0",
                                   ["kind", "name", "namespace"], registry=r)
        self.gpus_allocated = Gauge("kdl_gpus_allocated", "GPUs held by gang allocations", registry=r)
        self.kinds: set = set()
        self.lister: Optional[Callable[[str], List[dict]]] = None
        r.register(_StatusGauges(self))
        # last observed values, for tests/CLI (prometheus histograms hide them)
        self._lock = threading.Lock()
        self.observed: Dict[str, Dict[str, float]] = {"first": {}, "all": {}}

    def job_metrics(self, kind: str) -> "JobMetrics":
        self.kinds.add(kind)
        return JobMetrics(self, kind)


class JobMetrics:
    """Per-kind facade matching ``JobMetrics`` in the reference."""

    def __init__(self, reg: MetricsRegistry, kind: str):
        self.reg = reg
        self.kind = kind
        lk = kind.lower()
        self._created = reg.created.labels(lk)
        self._deleted = reg.deleted.labels(lk)
        self._success = reg.success.labels(lk)
        self._failure = reg.failure.labels(lk)
        self._restart = reg.restart.labels(lk)

    def created_inc(self):
        self._created.inc()

    def deleted_inc(self):
        self._deleted.inc()

    def success_inc(self):
        self._success.inc()

    def failure_inc(self):
        self._failure.inc()

    def restart_inc(self):
        self._restart.inc()

    def first_pod_launch_delay(self, active_pods: List[dict], job: dict, status: dict) -> Optional[float]:
        # Running, or Succeeded in the same reconcile that first saw a ready rank
        if not (c.is_running(status) or c.is_succeeded(status)):
            return None
        earliest = None
        for pod in active_pods:
            if (pod.get("status") or {}).get("phase") not in ("Running", "Succeeded"):
                continue
            t = _ready_time(pod)
            if t is None:
                continue
            if earliest is None or t < earliest:
                earliest = t
        if earliest is None:
            return None
        md = job["metadata"]
        delay = earliest - c.to_epoch(md["creationTimestamp"])
        self.reg.first_pod_delay.labels(self.kind, md["name"], md["namespace"], md["uid"]).observe(delay)
        self.reg.launch_delay_fine.labels(self.kind, "first").observe(delay)
        with self.reg._lock:
            self.reg.observed["first"][md["uid"]] = delay
        return delay

    def all_pods_launch_delay(self, pods: List[dict], job: dict, status: dict) -> Optional[float]:
        if not c.is_running(status) or not status.get("startTime"):
            return None
        md = job["metadata"]
        created = c.to_epoch(md["creationTimestamp"])
        final = created
        for pod in pods:
            if (pod.get("status") or {}).get("phase") != "Running":
                return None
            t = _ready_time(pod)
            if t is None:
                return None  # not every rank is Ready yet: observe later
            if t > final:
                final = t
        delay = final - created
        self.reg.all_pods_delay.labels(self.kind, md["name"], md["namespace"], md["uid"]).observe(delay)
        self.reg.launch_delay_fine.labels(self.kind, "all").observe(delay)
        with self.reg._lock:
            self.reg.observed["all"][md["uid"]] = delay
        return delay


def _ready_time(pod: dict) -> Optional[float]:
    """lastTransitionTime of a TRUE Ready condition (a False one means the rank
    has not signalled readiness yet and is not a launch-complete time); for a
    pod that already ran to completion, the time it first became Ready
    (``status.readyTime``, kept by the kubelet after Ready turns False)."""
    st = pod.get("status") or {}
    for cond in st.get("conditions") or []:
        if cond.get("type") == "Ready" and cond.get("status") == "True":
            return c.to_epoch(cond.get("lastTransitionTime"))
    if st.get("phase") == "Succeeded" and st.get("readyTime"):
        return c.to_epoch(st["readyTime"])
    return None


def pod_ready(pod: dict) -> bool:
    return _ready_time(pod) is not None


_default: Optional[MetricsRegistry] = None


def default_registry() -> MetricsRegistry:
    global _default
    if _default is None:
        _default = MetricsRegistry()
    return _default
