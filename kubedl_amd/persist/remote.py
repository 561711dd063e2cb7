"""Remote storage backends: MySQL objects and Aliyun SLS events.

The reference ships exactly these two (``pkg/storage/backends/objects/mysql``
and ``pkg/storage/backends/events/aliyun_sls``).  Both are registered under
the reference's names so ``--object-storage mysql`` / ``--event-storage
aliyun-sls`` select them; neither server is reachable from an offline node,
so their wire paths are covered by local fakes in ``tests/test_persist_remote.py``.

MySQL (``config.go:41-62``, ``mysql.go``)
    Connection from ``MYSQL_HOST`` (default ``localhost``), ``MYSQL_PORT``
    (3306), ``MYSQL_DB_NAME`` (``kubedl``), ``MYSQL_USER``,
    ``MYSQL_PASSWORD``; ``MYSQL_LOGMODE`` != ``no`` echoes every statement.
    The SQL is the SQLite backend's (same tables, same version-guarded upsert,
    same ``Stopped`` pseudo status) run through a DB-API adapter that maps
    ``?`` placeholders to ``%s``.  The driver is ``pymysql`` -- not in this
    image, so ``initialize()`` fails loudly naming it; a connection factory can
    be injected instead (tests use sqlite3 through the same adapter).

Aliyun SLS (``config.go:40-74``, ``sls_logstore.go``)
    ``SLS_ENDPOINT``, ``SLS_KEY_ID``, ``SLS_KEY_SECRET``, ``SLS_PROJECT``,
    ``SLS_LOG_STORE`` all required.  ``save_event`` PutLogs one LogGroup
    (protobuf, ``Topic=""``, ``Source=<component>/<host>``, log time = last
    timestamp) with the reference's retry policy: 10 attempts, 800 ms hold on
    ``WriteQuotaExceed``, 200 ms on server errors, any other error is final.
    ``list_events`` queries ``"<ns> AND <name>"``: histogram count first, then
    pages of 100 lines; each page is sorted by ``FirstTimestamp`` and
    de-duplicated by involved-object UID (the reference's behaviour: one event
    per object per page).  Requests are signed with the SLS ``LOG
    <key-id>:<hmac-sha1>`` scheme over plain HTTP(S) via ``urllib``.
"""
from __future__ import annotations

import base64
import datetime as _dt
import email.utils
import hashlib
import hmac
import json
import os
import sqlite3
import time
import urllib.error
import urllib.parse
import urllib.request
from typing import Callable, Dict, List, Optional, Tuple

from kubedl_amd.persist import backends as B
from kubedl_amd.persist import dmo


# ================================================================ MySQL
class _DBAPIAdapter:
    """Gives a DB-API connection the ``execute(sql, args) -> cursor`` shape the
    SQL backend uses, translating qmark placeholders to ``format`` style."""

    def __init__(self, conn, paramstyle: str, log: bool = False):
        self.conn = conn
        self.paramstyle = paramstyle
        self.log = log

    def execute(self, sql: str, args=()):
        if self.paramstyle == "format":
            sql = sql.replace("%", "%%").replace("?", "%s")
        if self.log:
            print(f"[mysql] {sql} {list(args)}", flush=True)
        cur = self.conn.cursor()
        cur.execute(sql, tuple(args))
        try:
            self.conn.commit()
        except Exception:  # noqa: BLE001 - autocommit connections
            pass
        return cur

    def close(self) -> None:
        self.conn.close()


def mysql_config_from_env() -> dict:
    """``GetMysqlDBSource`` (config.go:48-62)."""
    return {"host": os.environ.get("MYSQL_HOST") or "localhost",
            "port": int(os.environ.get("MYSQL_PORT") or "3306"),
            "database": os.environ.get("MYSQL_DB_NAME") or "kubedl",
            "user": os.environ.get("MYSQL_USER", ""),
            "password": os.environ.get("MYSQL_PASSWORD", ""),
            "logmode": os.environ.get("MYSQL_LOGMODE") or "no"}


class MySQLObjectBackend(B.SQLiteObjectBackend):
    NAME = "mysql"

    def __init__(self, connect: Optional[Callable[[dict], Tuple[object, str]]] = None):
        super().__init__(path="")
        self.cfg = mysql_config_from_env()
        self._connect = connect

    def _default_connect(self, cfg: dict):
        try:
            import pymysql  # type: ignore
        except ImportError as e:
            raise RuntimeError("object storage backend 'mysql' needs the pymysql driver, which is not "
                               "installed; use --object-storage sqlite on this node") from e
        conn = pymysql.connect(host=cfg["host"], port=cfg["port"], user=cfg["user"], password=cfg["password"],
                               database=cfg["database"], charset="utf8", autocommit=True)
        return conn, "format"

    def initialize(self) -> None:
        conn, style = (self._connect or self._default_connect)(self.cfg)
        self.db = _DBAPIAdapter(conn, style, log=self.cfg["logmode"] not in ("", "no", "false"))
        pk = ("id INTEGER PRIMARY KEY AUTOINCREMENT" if style == "qmark"
              else "id BIGINT PRIMARY KEY AUTO_INCREMENT")
        txt = "TEXT" if style == "qmark" else "VARCHAR(1024)"
        self.db.execute(f"CREATE TABLE IF NOT EXISTS job_info ({pk}, "
                        + ", ".join(f"{col} {txt}" for col in B._JOB_COLS) + ")")
        self.db.execute(f"CREATE TABLE IF NOT EXISTS replica_info ({pk}, "
                        + ", ".join(f"{col} {txt}" for col in B._POD_COLS) + ")")

    def close(self) -> None:
        if self.db is not None:
            self.db.close()
            self.db = None


def sqlite_connect_for_tests(path: str):
    """Connection factory running the MySQL backend's SQL on sqlite3 (qmark)."""
    def connect(_cfg):
        return sqlite3.connect(path, check_same_thread=False, isolation_level=None), "qmark"
    return connect


# ================================================================ SLS
class SLSError(Exception):
    def __init__(self, code: str, message: str = "", status: int = 0):
        super().__init__(f"{code}: {message}")
        self.code, self.message, self.status = code, message, status


def _pb_varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _pb_bytes(field: int, data: bytes) -> bytes:
    return _pb_varint(field << 3 | 2) + _pb_varint(len(data)) + data


def encode_log_group(logs: List[Tuple[int, List[Tuple[str, str]]]], topic: str, source: str) -> bytes:
    """SLS ``LogGroup`` protobuf: Logs=1 {Time=1 varint, Contents=2 {Key=1,
    Value=2}}, Topic=3, Source=4."""
    out = bytearray()
    for t, contents in logs:
        body = _pb_varint(1 << 3 | 0) + _pb_varint(int(t))
        for k, v in contents:
            body += _pb_bytes(2, _pb_bytes(1, k.encode()) + _pb_bytes(2, v.encode()))
        out += _pb_bytes(1, body)
    out += _pb_bytes(3, topic.encode())
    out += _pb_bytes(4, source.encode())
    return bytes(out)


def _pb_fields(buf: bytes):
    i = 0
    while i < len(buf):
        key, i = _pb_read_varint(buf, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _pb_read_varint(buf, i)
            yield f, v
        elif wt == 2:
            n, i = _pb_read_varint(buf, i)
            yield f, buf[i:i + n]
            i += n
        else:
            raise ValueError(f"unsupported wire type {wt}")


def _pb_read_varint(buf: bytes, i: int):
    shift = v = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            return v, i


def decode_log_group(buf: bytes) -> dict:
    """Inverse of :func:`encode_log_group` (used by the test fake)."""
    out = {"logs": [], "topic": "", "source": ""}
    for f, v in _pb_fields(buf):
        if f == 1:
            log = {"time": 0, "contents": {}}
            for lf, lv in _pb_fields(v):
                if lf == 1:
                    log["time"] = lv
                elif lf == 2:
                    kv = dict(_pb_fields(lv))
                    log["contents"][kv.get(1, b"").decode()] = kv.get(2, b"").decode()
            out["logs"].append(log)
        elif f == 3:
            out["topic"] = v.decode()
        elif f == 4:
            out["source"] = v.decode()
    return out


def sls_signature(secret: str, verb: str, content_md5: str, content_type: str, date: str,
                  headers: Dict[str, str], resource: str) -> str:
    canon_headers = "\n".join(f"{k}:{headers[k]}" for k in sorted(headers) if k.startswith(("x-log-", "x-acs-")))
    sts = f"{verb}\n{content_md5}\n{content_type}\n{date}\n{canon_headers}\n{resource}"
    return base64.b64encode(hmac.new(secret.encode(), sts.encode(), hashlib.sha1).digest()).decode()


class SLSClient:
    """Minimal signed SLS REST client (PutLogs, GetHistograms, GetLogs)."""

    def __init__(self, endpoint: str, key_id: str, key_secret: str, timeout: float = 10.0):
        self.endpoint = endpoint if "://" in endpoint else "http://" + endpoint
        self.key_id, self.key_secret, self.timeout = key_id, key_secret, timeout

    def _request(self, project: str, verb: str, path: str, params: Optional[dict] = None,
                 body: bytes = b"", content_type: str = ""):
        u = urllib.parse.urlsplit(self.endpoint)
        host = f"{project}.{u.netloc}" if project and not u.netloc.startswith(("127.", "localhost")) else u.netloc
        date = email.utils.formatdate(usegmt=True)
        headers = {"x-log-apiversion": "0.6.0", "x-log-signaturemethod": "hmac-sha1",
                   "x-log-bodyrawsize": str(len(body)), "x-log-project": project}
        md5 = hashlib.md5(body).hexdigest().upper() if body else ""
        resource = path
        if params:
            resource += "?" + "&".join(f"{k}={params[k]}" for k in sorted(params))
        sig = sls_signature(self.key_secret, verb, md5, content_type, date, headers, resource)
        req_headers = dict(headers, Date=date, Host=host, Authorization=f"LOG {self.key_id}:{sig}")
        if body:
            req_headers["Content-MD5"] = md5
            req_headers["Content-Type"] = content_type
        url = f"{u.scheme}://{u.netloc}{path}"
        if params:
            url += "?" + urllib.parse.urlencode(params)
        req = urllib.request.Request(url, data=body or None, method=verb, headers=req_headers)
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                return r.status, dict(r.headers), r.read()
        except urllib.error.HTTPError as e:
            raw = e.read()
            try:
                err = json.loads(raw)
            except ValueError:
                err = {"errorCode": "ServerError" if e.code >= 500 else "ClientError", "errorMessage": raw.decode()}
            raise SLSError(err.get("errorCode", ""), err.get("errorMessage", ""), e.code) from None
        except OSError as e:
            raise SLSError("ServerError", str(e)) from None

    def put_logs(self, project: str, logstore: str, group: bytes) -> None:
        self._request(project, "POST", f"/logstores/{logstore}/shards/lb", body=group,
                      content_type="application/x-protobuf")

    def get_histograms(self, project: str, logstore: str, frm: int, to: int, query: str) -> int:
        _, _, data = self._request(project, "GET", f"/logstores/{logstore}",
                                   {"type": "histogram", "from": frm, "to": to, "query": query, "topic": ""})
        return sum(int(h.get("count", 0)) for h in json.loads(data or b"[]"))

    def get_logs(self, project: str, logstore: str, frm: int, to: int, query: str,
                 lines: int, offset: int) -> List[Dict[str, str]]:
        _, _, data = self._request(project, "GET", f"/logstores/{logstore}",
                                   {"type": "log", "from": frm, "to": to, "query": query, "topic": "",
                                    "line": lines, "offset": offset, "reverse": "false"})
        return json.loads(data or b"[]")


SLS_RETRY_TIMES = 10
SLS_QUOTA_HOLD_S = 0.8
SLS_SERVER_HOLD_S = 0.2
SLS_MAX_LINES = 100


def _rfc3339_to_unix(ts: str) -> int:
    if not ts:
        return 0
    return int(_dt.datetime.fromisoformat(ts.replace("Z", "+00:00")).timestamp())


class SLSEventBackend(B.EventStorageBackend):
    NAME = "aliyun-sls"

    def __init__(self, client: Optional[SLSClient] = None, sleep=time.sleep):
        self.client = client
        self.project = self.logstore = ""
        self._sleep = sleep

    def name(self) -> str:
        return self.NAME

    def initialize(self) -> None:
        """``GetSLSClient`` (config.go:50-74): every variable is required."""
        vals = {}
        for env, what in (("SLS_ENDPOINT", "sls endpoint"), ("SLS_KEY_ID", "sls key id"),
                          ("SLS_KEY_SECRET", "sls key secret"), ("SLS_PROJECT", "sls project name"),
                          ("SLS_LOG_STORE", "sls log store")):
            vals[env] = os.environ.get(env, "")
            if not vals[env]:
                raise RuntimeError(f"empty {what}")
        if self.client is None:
            self.client = SLSClient(vals["SLS_ENDPOINT"], vals["SLS_KEY_ID"], vals["SLS_KEY_SECRET"])
        self.project, self.logstore = vals["SLS_PROJECT"], vals["SLS_LOG_STORE"]

    def close(self) -> None:
        pass

    @staticmethod
    def to_log_group(event: dict, region: str) -> bytes:
        """``toSLSLogGroup`` (sls_logstore.go:140-205)."""
        row = dmo.event_to_dmo(event, region)
        contents = [("FirstTimestamp", row.get("first_timestamp") or ""),
                    ("LastTimestamp", row.get("last_timestamp") or ""),
                    ("Count", str(row.get("count") or 1)), ("Name", row.get("name") or ""),
                    ("Kind", row.get("kind") or ""), ("ObjUID", row.get("obj_uid") or ""),
                    ("ObjNamespace", row.get("obj_namespace") or ""), ("ObjName", row.get("obj_name") or ""),
                    ("Type", row.get("type") or ""), ("Reason", row.get("reason") or ""),
                    ("Message", row.get("message") or "")]
        if region:
            contents.append(("Region", region))
        src = event.get("source") or {}
        return encode_log_group([(_rfc3339_to_unix(row.get("last_timestamp") or ""), contents)], "",
                                f"{src.get('component', '')}/{src.get('host', '')}")

    def save_event(self, event: dict, region: str) -> None:
        group = self.to_log_group(event, region)
        err: Optional[Exception] = None
        for _ in range(SLS_RETRY_TIMES):
            try:
                self.client.put_logs(self.project, self.logstore, group)
                return
            except SLSError as e:
                err = e
                if e.code == "WriteQuotaExceed":
                    self._sleep(SLS_QUOTA_HOLD_S)
                elif e.code in ("InternalServerError", "ServerBusy", "ServerError") or e.status >= 500:
                    self._sleep(SLS_SERVER_HOLD_S)
                else:
                    raise
        raise RuntimeError(f"SLS PutLogs failed after retry {SLS_RETRY_TIMES} times: {err}")

    @staticmethod
    def _unwrap(raw: Dict[str, str]) -> dict:
        return {"name": raw.get("Name", ""), "kind": raw.get("Kind", ""), "type": raw.get("Type", ""),
                "obj_namespace": raw.get("ObjNamespace", ""), "obj_name": raw.get("ObjName", ""),
                "obj_uid": raw.get("ObjUID", ""), "reason": raw.get("Reason", ""),
                "message": raw.get("Message", ""), "count": int(raw["Count"]), "region": raw.get("Region"),
                "first_timestamp": raw.get("FirstTimestamp", ""), "last_timestamp": raw.get("LastTimestamp", "")}

    def list_events(self, job_namespace: str, job_name: str, start: str = "", end: str = "") -> List[dict]:
        query = f"{job_namespace} AND {job_name}"
        frm = _rfc3339_to_unix(start) if start else 0
        to = _rfc3339_to_unix(end) if end else int(time.time()) + 1
        remaining = self.client.get_histograms(self.project, self.logstore, frm, to, query)
        out: List[dict] = []
        offset = 0
        while remaining > 0:
            n = min(SLS_MAX_LINES, remaining)
            logs = self.client.get_logs(self.project, self.logstore, frm, to, query, n, offset)
            logs.sort(key=lambda r: r.get("FirstTimestamp", ""))
            seen = set()
            for raw in logs:
                e = self._unwrap(raw)
                if e["obj_uid"] not in seen:
                    seen.add(e["obj_uid"])
                    out.append(e)
            remaining -= SLS_MAX_LINES
            offset += SLS_MAX_LINES
        return out


B.register_object_backend("mysql", lambda home: MySQLObjectBackend())
B.register_event_backend("aliyun-sls", lambda home: SLSEventBackend())
