"""Prometheus metrics (``pkg/metrics``) + the ``/metrics`` HTTP endpoint."""
from __future__ import annotations

from kubedl_amd.metrics.job_metrics import JobMetrics, MetricsRegistry, default_registry  # noqa: F401


def start_monitoring(port: int, registry=None, addr: str = "127.0.0.1"):
    """StartMonitoringForDefaultRegistry (``pkg/metrics/monitor.go:27-36``):
    serve ``/metrics`` on ``addr:port`` in a daemon thread.  Returns the server,
    or None when the port cannot be bound -- like the reference, which logs
    "monitoring default registry failed" and keeps the manager running.
    ``registry``: anything with a ``.registry`` CollectorRegistry."""
    import logging
    from kubedl_amd.metrics.exposition import serve
    reg = registry or default_registry()
    try:
        server = serve(port, addr or "0.0.0.0", reg.registry)
    except OSError as e:
        logging.getLogger("kubedl_amd.metrics").error("monitoring registry on %s:%d failed, err: %s", addr, port, e)
        return None
    return server


def parse_addr(v, default_host: str = "") -> tuple:
    """``--metrics-addr`` / ``--controller-metrics-addr`` value -> (host, port).
    Accepts the reference's int form (``8443``) and Go's ``[host]:port``
    (``:8443`` = every interface); ``0``, ``""`` or ``:0`` turn it off (port 0)."""
    s = str(v if v is not None else "").strip()
    if not s:
        return default_host, 0
    host, _, port = s.rpartition(":")
    return (host if ":" in s else default_host), int(port or 0)


def render(registry: MetricsRegistry | None = None) -> str:
    from kubedl_amd.metrics.exposition import generate_text
    reg = registry or default_registry()
    return generate_text(reg.registry).decode()
