"""Prometheus text exposition with Go client_golang's counter naming.

Python's ``prometheus_client`` renames every counter ``<name>_total`` in the
text format and adds a ``<name>_created`` series; Go's client_golang (what the
reference links, ``pkg/metrics/job_metrics.go:32-61``) exports a counter under
exactly the name it was registered with and no creation-time series.  Scrapers
and dashboards written against KubeDL read ``kubedl_jobs_created{kind=...}``,
so the job counters here are :class:`BareCounterVec` collectors and the
registry is rendered by :func:`generate_text`, which keeps a counter's name as
its samples carry it.  Everything else (gauges, histograms, controller-runtime
``*_total`` counters) renders exactly as ``generate_latest`` would.
"""
from __future__ import annotations

import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, Iterable, Tuple

from prometheus_client.core import Metric
from prometheus_client.utils import floatToGoString


class _Child:
    __slots__ = ("_vec", "_key")

    def __init__(self, vec: "BareCounterVec", key: Tuple[str, ...]):
        self._vec = vec
        self._key = key

    def inc(self, amount: float = 1.0) -> None:
        if amount < 0:
            raise ValueError("counters can only increase")
        with self._vec._lock:
            self._vec._values[self._key] = self._vec._values.get(self._key, 0.0) + amount

    def get(self) -> float:
        with self._vec._lock:
            return self._vec._values.get(self._key, 0.0)


class BareCounterVec:
    """A labelled counter exported as ``name{labels} value`` (no ``_total``,
    no ``_created``): client_golang's ``CounterVec`` exposition."""

    def __init__(self, name: str, documentation: str, labelnames: Iterable[str], registry=None):
        self.name = name
        self.documentation = documentation
        self.labelnames = tuple(labelnames)
        self._lock = threading.Lock()
        self._values: Dict[Tuple[str, ...], float] = {}
        if registry is not None:
            registry.register(self)

    def labels(self, *values: str) -> _Child:
        if len(values) != len(self.labelnames):
            raise ValueError(f"{self.name}: expected labels {self.labelnames}, got {values}")
        key = tuple(str(v) for v in values)
        with self._lock:
            self._values.setdefault(key, 0.0)
        return _Child(self, key)

    def describe(self):
        return [Metric(self.name, self.documentation, "counter")]

    def collect(self):
        m = Metric(self.name, self.documentation, "counter")
        with self._lock:
            items = sorted(self._values.items())
        for key, v in items:
            m.add_sample(self.name, dict(zip(self.labelnames, key)), v)
        yield m


def _labels(d: dict) -> str:
    if not d:
        return ""
    parts = []
    for k, v in sorted(d.items()):
        v = str(v).replace("\\", r"\\").replace("\n", r"\n").replace('"', r"\"")
        parts.append(f'{k}="{v}"')
    return "{" + ",".join(parts) + "}"


_TYPES = {"info": "gauge", "stateset": "gauge", "gaugehistogram": "histogram", "unknown": "untyped"}


def generate_text(registry) -> bytes:
    """Text format 0.0.4 of ``registry``; a counter whose samples carry its bare
    name keeps it in HELP/TYPE (client_golang), any other counter gets the
    ``_total`` family name ``generate_latest`` gives it.  The python client's
    ``*_created`` series are dropped (client_golang has none)."""
    out = []
    for metric in registry.collect():
        mname, mtype = metric.name, metric.type
        if mtype == "counter":
            if not any(s.name == metric.name for s in metric.samples):
                mname = mname + "_total"
        elif mtype == "info":
            mname = mname + "_info"
        mtype = _TYPES.get(mtype, mtype)
        doc = metric.documentation.replace("\\", r"\\").replace("\n", r"\n")
        out.append(f"# HELP {mname} {doc}\n")
        out.append(f"# TYPE {mname} {mtype}\n")
        for s in metric.samples:
            if s.name == metric.name + "_created" and metric.type in ("counter", "histogram", "summary"):
                continue  # python-client creation timestamps: client_golang has none
            ts =f" {int(float(s.timestamp) * 1000):d}" if s.timestamp is not None else ""
            out.append(f"{s.name}{_labels(s.labels)} {floatToGoString(s.value)}{ts}\n")
    return "".join(out).encode()


CONTENT_TYPE = "text/plain; version=0.0.4; charset=utf-8"


def serve(port: int, addr: str, registry) -> ThreadingHTTPServer:
    """``/metrics`` (any path, like promhttp's handler mounted at the root mux)
    on ``addr:port`` in a daemon thread."""

    class _H(BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            body = generate_text(registry)
            self.send_response(200)
            self.send_header("Content-Type", CONTENT_TYPE)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = ThreadingHTTPServer((addr, port), _H)
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, name=f"metrics:{port}", daemon=True).start()
    return srv
