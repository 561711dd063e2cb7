"""Prometheus metrics (``pkg/metrics``) + the ``/metrics`` HTTP endpoint."""
from __future__ import annotations

from kubedl_amd.metrics.job_metrics import JobMetrics, MetricsRegistry, default_registry  # noqa: F401


def start_monitoring(port: int, registry: MetricsRegistry | None = None, addr: str = "127.0.0.1"):
    """StartMonitoringForDefaultRegistry (``pkg/metrics/monitor.go:27-36``):
    serve ``/metrics`` on ``addr:port`` in a daemon thread.  Returns the server."""
    from prometheus_client import start_http_server
    reg = registry or default_registry()
    server, _thread = start_http_server(port, addr=addr, registry=reg.registry)
    return server


def render(registry: MetricsRegistry | None = None) -> str:
    from prometheus_client import generate_latest
    reg = registry or default_registry()
    return generate_latest(reg.registry).decode()
