"""Controller-runtime metrics served on ``--controller-metrics-addr``.

Reference: ``main.go:54,72`` binds controller-runtime's metrics endpoint to
``:8080``; controller-runtime v0.4 registers there (on its own registry, apart
from the default registry KubeDL's ``kubedl_jobs_*`` live in on ``:8443``) the
reconcile counters/histogram of every controller and the client-go workqueue
metrics of every controller's queue.  Same names and labels here, fed by the
manager's per-kind reconcile loops (``engine/manager.py`` ``_KindLoop``).
"""
from __future__ import annotations

from typing import Callable, Dict

from prometheus_client import CollectorRegistry, Counter, Histogram
from prometheus_client.core import GaugeMetricFamily


class _QueueGauges:
    """workqueue_depth / workqueue_unfinished_work_seconds computed on scrape."""

    def __init__(self, owner: "ControllerMetrics"):
        self.owner = owner

    def collect(self):
        depth = GaugeMetricFamily("workqueue_depth", "Current depth of workqueue", labels=["name"])
        for name, q in sorted(self.owner.queues.items()):
            depth.add_metric([name], float(q()))
        yield depth


class ControllerMetrics:
    def __init__(self):
        self.registry = CollectorRegistry()
        r = self.registry
        self.reconcile_total = Counter("controller_runtime_reconcile_total",
                                       "Total number of reconciliations per controller",
                                       ["controller", "result"], registry=r)
        self.reconcile_errors = Counter("controller_runtime_reconcile_errors_total",
                                        "Total number of reconciliation errors per controller", ["controller"],
                                        registry=r)
        self.reconcile_time = Histogram("controller_runtime_reconcile_time_seconds",
                                        "Length of time per reconciliation per controller", ["controller"],
                                        registry=r)
        self.queue_adds = Counter("workqueue_adds_total", "Total number of adds handled by workqueue", ["name"],
                                  registry=r)
        self.queue_retries = Counter("workqueue_retries_total", "Total number of retries handled by workqueue",
                                     ["name"], registry=r)
        self.queue_latency = Histogram("workqueue_work_duration_seconds",
                                       "How long in seconds processing an item from workqueue takes.", ["name"],
                                       registry=r)
        self.queues: Dict[str, Callable[[], int]] = {}
        r.register(_QueueGauges(self))

    def observe_reconcile(self, controller: str, seconds: float, result: str) -> None:
        """result: success | error | requeue | requeue_after (controller-runtime's labels)."""
        self.reconcile_total.labels(controller, result).inc()
        if result == "error":
            self.reconcile_errors.labels(controller).inc()
        self.reconcile_time.labels(controller).observe(seconds)
        self.queue_latency.labels(controller).observe(seconds)

    def render(self) -> str:
        from kubedl_amd.metrics.exposition import generate_text
        return generate_text(self.registry).decode()
