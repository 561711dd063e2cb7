"""HTTP API of the manager daemon (the API-server endpoint ``kdl`` talks to).

A small JSON REST surface over the store, mirroring what ``kubectl`` needs:

====================================================  ==========================================
``POST   /api/apply``                                  create a job (manifest JSON body)
``GET    /api/objects/<kind>[?namespace=ns]``          list (``kind`` may be an alias: tfjobs...)
``GET    /api/objects/<kind>/<ns>/<name>``             get
``DELETE /api/objects/<kind>/<ns>/<name>``             delete (cascades to pods/services)
``GET    /api/events?namespace=&uid=``                 events
``GET    /api/logs/<ns>/<pod>?container=&tail=N``      container log
``GET    /api/node``                                   GPU inventory + gang allocations
``GET    /api/summary``                                one row per job: state, age, replicas, launch delays
``GET    /dashboard``                                  the same as an auto-refreshing HTML page (the
                                                      reference's "job dashboard", README.md:100-105)
``GET    /metrics``                                    Prometheus exposition (kubedl_jobs_*)
====================================================  ==========================================
"""
from __future__ import annotations

import html
import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional
from urllib.parse import parse_qs, urlparse

from kubedl_amd.api import kinds as K
from kubedl_amd.store import AlreadyExists, NotFound

CORE_KINDS = {"pod": "Pod", "pods": "Pod", "po": "Pod", "service": "Service", "services": "Service",
              "svc": "Service", "event": "Event", "events": "Event", "podgroup": "PodGroup",
              "podgroups": "PodGroup"}


def resolve_kind(k: str) -> str:
    if k in ("Pod", "Service", "Event", "PodGroup"):
        return k
    if k.lower() in CORE_KINDS:
        return CORE_KINDS[k.lower()]
    return K.lookup(k).kind


def job_summary(mgr) -> list:
    """Dashboard rows: every job of every kind with its state and timings."""
    from kubedl_amd.api import common as c
    rows = []
    now = time.time()
    for kind in sorted(K.BY_KIND):
        for j in mgr.store.list(kind):
            md, st = j["metadata"], j.get("status") or {}
            conds = [x for x in st.get("conditions") or [] if x.get("status") == "True"]
            created = c.to_epoch(md.get("creationTimestamp")) or now
            done = c.to_epoch(st.get("completionTime"))
            reps = {rt: {k: int(v) for k, v in (rs or {}).items()} for rt, rs in (st.get("replicaStatuses") or {}).items()}
            uid = md.get("uid", "")
            obs = getattr(mgr.metrics, "observed", {"first": {}, "all": {}})
            rows.append({"kind": kind, "namespace": md.get("namespace", ""), "name": md["name"],
                         "state": conds[-1]["type"] if conds else "", "age_s": round(now - created, 1),
                         "duration_s": round((done or now) - created, 1), "replicas": reps,
                         "first_pod_launch_delay_s": obs["first"].get(uid), "all_pods_launch_delay_s": obs["all"].get(uid)})
    return rows


def dashboard_html(rows) -> str:
    def cell(v):
        return html.escape("" if v is None else (json.dumps(v) if isinstance(v, dict) else str(v)))
    cols = ["kind", "namespace", "name", "state", "age_s", "duration_s", "replicas", "first_pod_launch_delay_s",
            "all_pods_launch_delay_s"]
    head = "".join(f"<th>{c}</th>" for c in cols)
    body = "".join("<tr>" + "".join(f"<td>{cell(r.get(c))}</td>" for c in cols) + "</tr>" for r in rows)
    return ("<!doctype html><html><head><meta charset='utf-8'><meta http-equiv='refresh' content='5'>"
            "<title>kdl jobs</title><style>body{font-family:sans-serif}table{border-collapse:collapse}"
            "td,th{border:1px solid #bbb;padding:3px 8px;font-size:13px}</style></head><body>"
            f"<h3>kdl jobs ({len(rows)})</h3><table><tr>{head}</tr>{body}</table></body></html>")


def make_handler(mgr):
    class Handler(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, fmt, *args):  # quiet
            pass

        def _send(self, code: int, body, ctype="application/json"):
            data = body.encode() if isinstance(body, str) else json.dumps(body).encode()
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def _err(self, code, msg):
            self._send(code, {"error": msg})

        def do_GET(self):
            u = urlparse(self.path)
            q = {k: v[0] for k, v in parse_qs(u.query).items()}
            parts = [p for p in u.path.split("/") if p]
            try:
                if u.path == "/metrics":
                    from kubedl_amd.metrics import render
                    return self._send(200, render(mgr.metrics), "text/plain; version=0.0.4")
                if parts[:2] == ["api", "objects"] and len(parts) == 3:
                    return self._send(200, {"items": mgr.store.list(resolve_kind(parts[2]), q.get("namespace"))})
                if parts[:2] == ["api", "objects"] and len(parts) == 5:
                    return self._send(200, mgr.store.get(resolve_kind(parts[2]), parts[3], parts[4]))
                if parts[:2] == ["api", "events"]:
                    evs = mgr.store.list("Event", q.get("namespace"))
                    if q.get("uid"):
                        evs = [e for e in evs if (e.get("involvedObject") or {}).get("uid") == q["uid"]]
                    evs.sort(key=lambda e: e.get("firstTimestamp", ""))
                    return self._send(200, {"items": evs})
                if parts[:2] == ["api", "logs"] and len(parts) == 4:
                    if mgr.kubelet is None:
                        return self._err(404, "no node runtime")
                    path = mgr.kubelet.log_path(parts[2], parts[3], q.get("container"))
                    if path is None:
                        return self._err(404, "pod not found")
                    try:
                        text = open(path, errors="replace").read()
                    except FileNotFoundError:
                        text = ""
                    if q.get("tail"):
                        text = "\n".join(text.splitlines()[-int(q["tail"]):]) + "\n"
                    return self._send(200, text, "text/plain")
                if parts[:2] == ["api", "node"]:
                    a = mgr.allocator
                    return self._send(200, {"gpus": a.inv.count if a else 0, "hbm_gb": a.inv.hbm_gb if a else 0,
                                            "free": a.free if a else [], "allocations": a.snapshot() if a else {},
                                            "running_pods": mgr.kubelet.running_pods() if mgr.kubelet else []})
                if parts[:2] == ["api", "summary"]:
                    return self._send(200, {"items": job_summary(mgr)})
                if parts == ["dashboard"]:
                    return self._send(200, dashboard_html(job_summary(mgr)), "text/html; charset=utf-8")
                if parts == ["healthz"]:
                    return self._send(200, "ok", "text/plain")
                return self._err(404, f"no route {u.path}")
            except NotFound as e:
                return self._err(404, str(e))
            except KeyError as e:
                return self._err(400, str(e))

        def do_POST(self):
            u = urlparse(self.path)
            n = int(self.headers.get("Content-Length", "0"))
            body = json.loads(self.rfile.read(n) or b"{}")
            if u.path == "/api/apply":
                try:
                    return self._send(201, mgr.apply(body))
                except AlreadyExists as e:
                    return self._err(409, str(e))
                except (ValueError, KeyError) as e:
                    return self._err(400, str(e))
            return self._err(404, f"no route {u.path}")

        def do_DELETE(self):
            parts = [p for p in urlparse(self.path).path.split("/") if p]
            if parts[:2] == ["api", "objects"] and len(parts) == 5:
                try:
                    mgr.store.delete(resolve_kind(parts[2]), parts[3], parts[4])
                    return self._send(200, {"deleted": parts[4]})
                except NotFound as e:
                    return self._err(404, str(e))
                except KeyError as e:
                    return self._err(400, str(e))
            return self._err(404, "no route")

    return Handler


class APIServer:
    def __init__(self, mgr, port: int, addr: str = "127.0.0.1"):
        self.httpd = ThreadingHTTPServer((addr, port), make_handler(mgr))
        self.httpd.daemon_threads = True
        self.port = self.httpd.server_address[1]
        self.thread: Optional[threading.Thread] = None

    def start(self):
        self.thread = threading.Thread(target=self.httpd.serve_forever, name="kdl-api", daemon=True)
        self.thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()
