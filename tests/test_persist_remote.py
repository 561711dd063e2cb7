"""MySQL and Aliyun SLS backends (the reference's two remote backends) against
local fakes: the MySQL SQL runs through the DB-API adapter on sqlite3; SLS
requests go to an in-process HTTP server that checks the request signature and
decodes the protobuf LogGroup."""
import http.server
import json
import threading
import urllib.parse

import pytest

from kubedl_amd.persist import new_event_backend, new_object_backend, remote
from kubedl_amd.persist.backends import Query


def _job(uid="u1", rv="1", cond="Running"):
    return {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
            "metadata": {"name": "j", "namespace": "ns", "uid": uid, "resourceVersion": rv,
                         "creationTimestamp": "2026-01-01T00:00:00Z"},
            "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1, "template": {"spec": {"containers": [
                {"name": "pytorch", "image": "img"}]}}}}},
            "status": {"conditions": [{"type": cond, "status": "True"}]}}


def test_mysql_backend_env_and_sql(tmp_path, monkeypatch):
    monkeypatch.setenv("MYSQL_HOST", "db.example")
    monkeypatch.setenv("MYSQL_PORT", "3307")
    cfg = remote.mysql_config_from_env()
    assert (cfg["host"], cfg["port"], cfg["database"], cfg["logmode"]) == ("db.example", 3307, "kubedl", "no")
    be = remote.MySQLObjectBackend(connect=remote.sqlite_connect_for_tests(str(tmp_path / "m.db")))
    be.initialize()
    be.save_job(_job(rv="2"), "r1")
    be.save_job(_job(rv="1", cond="Failed"), "r1")  # older resourceVersion: ignored
    assert be.get_job("ns", "j", "u1")["status"] == "Running"
    be.stop_job("ns", "j", "u1")
    rows = be.list_jobs(Query(namespace="ns"))
    assert rows[0]["status"] == "Stopped" and rows[0]["is_in_etcd"] == 0
    be.close()


def test_mysql_without_driver_fails_loudly():
    be = new_object_backend("mysql", "/tmp")
    with pytest.raises(RuntimeError, match="pymysql"):
        be.initialize()


def test_sls_backend_requires_env(monkeypatch):
    for k in ("SLS_ENDPOINT", "SLS_KEY_ID", "SLS_KEY_SECRET", "SLS_PROJECT", "SLS_LOG_STORE"):
        monkeypatch.delenv(k, raising=False)
    with pytest.raises(RuntimeError, match="empty sls endpoint"):
        new_event_backend("aliyun-sls", "/tmp").initialize()


class _FakeSLS(http.server.BaseHTTPRequestHandler):
    store = []
    fail = []

    def log_message(self, *a):
        pass

    def _check_sig(self, body=b""):
        u = urllib.parse.urlsplit(self.path)
        params = dict(urllib.parse.parse_qsl(u.query, keep_blank_values=True))
        resource = u.path + ("?" + "&".join(f"{k}={params[k]}" for k in sorted(params)) if params else "")
        hdrs = {k.lower(): v for k, v in self.headers.items() if k.lower().startswith("x-log-")}
        sig = remote.sls_signature("secret", self.command, self.headers.get("Content-MD5", ""),
                                   self.headers.get("Content-Type", ""), self.headers["Date"], hdrs, resource)
        assert self.headers["Authorization"] == f"LOG kid:{sig}"
        return u.path, params

    def _reply(self, code, obj):
        data = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def do_POST(self):
        body = self.rfile.read(int(self.headers["Content-Length"]))
        self._check_sig(body)
        if self.fail:
            code, err = self.fail.pop(0)
            return self._reply(code, {"errorCode": err, "errorMessage": "injected"})
        g = remote.decode_log_group(body)
        self.store.extend(dict(log["contents"], __source=g["source"]) for log in g["logs"])
        self._reply(200, {})

    def do_GET(self):
        _, p = self._check_sig()
        hits = [r for r in self.store if all(t.strip() in (r["ObjNamespace"], r["ObjName"], r["Name"])
                                             or t.strip() in r["ObjName"] for t in p["query"].split(" AND "))]
        if p["type"] == "histogram":
            return self._reply(200, [{"count": len(hits)}])
        off, n = int(p["offset"]), int(p["line"])
        self._reply(200, [{k: v for k, v in r.items() if not k.startswith("__")} for r in hits[off:off + n]])


def _event(i, uid):
    return {"metadata": {"name": f"ev{i}", "namespace": "ns"}, "type": "Normal", "reason": "R", "message": f"m{i}",
            "count": 1, "involvedObject": {"kind": "PyTorchJob", "namespace": "ns", "name": "j", "uid": uid},
            "firstTimestamp": f"2026-01-01T00:00:{i:02d}Z", "lastTimestamp": f"2026-01-01T00:00:{i:02d}Z",
            "source": {"component": "kdl", "host": "node0"}}


def test_sls_put_get_retry_and_dedup(monkeypatch):
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _FakeSLS)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        monkeypatch.setenv("SLS_ENDPOINT", f"http://127.0.0.1:{srv.server_port}")
        monkeypatch.setenv("SLS_KEY_ID", "kid")
        monkeypatch.setenv("SLS_KEY_SECRET", "secret")
        monkeypatch.setenv("SLS_PROJECT", "proj")
        monkeypatch.setenv("SLS_LOG_STORE", "events")
        sleeps = []
        be = remote.SLSEventBackend(sleep=sleeps.append)
        be.initialize()
        _FakeSLS.fail[:] = [(403, "WriteQuotaExceed"), (500, "InternalServerError")]
        be.save_event(_event(1, "uid-a"), "r1")
        assert sleeps == [remote.SLS_QUOTA_HOLD_S, remote.SLS_SERVER_HOLD_S]
        assert _FakeSLS.store[0]["__source"] == "kdl/node0" and _FakeSLS.store[0]["Region"] == "r1"
        for i in range(2, 6):
            be.save_event(_event(i, "uid-a" if i < 4 else f"uid-{i}"), "r1")
        ev = be.list_events("ns", "j")
        # one event per involved object per page, ordered by first timestamp (reference behaviour)
        assert [e["name"] for e in ev] == ["ev1", "ev4", "ev5"]
        _FakeSLS.fail[:] = [(400, "Unauthorized")]
        with pytest.raises(remote.SLSError):
            be.save_event(_event(9, "x"), "")
    finally:
        srv.shutdown()
