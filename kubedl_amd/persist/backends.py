"""Storage backends (``pkg/storage/backends``): interfaces, registry, and the
local implementations.

``ObjectStorageBackend`` (``interface.go:31-60``): initialize / close / name /
save_pod / list_pods / stop_pod / save_job / get_job / list_jobs / stop_job /
delete_job.  ``EventStorageBackend``: save_event / list_events.

Local backends (the reference ships MySQL (gorm) and Aliyun SLS, neither
reachable from a single offline node):

* ``sqlite`` object backend -- the same three tables and columns as the MySQL
  backend (``mysql.go``), the same version-guarded upsert (a row is only
  overwritten by a newer ``resourceVersion``) and the same ``Stopped`` pseudo
  status / ``is_in_etcd=0`` marking for objects that left the store;
* ``jsonl`` event backend -- append-only ``events.jsonl`` (SLS-like log store),
  deduplicated on read by ``obj_uid + reason + message`` keeping the latest;
* ``sqlite`` event backend -- ``event_info`` table in the same database.

Quirks of the reference NOT reproduced: ``StopPod``'s swapped
arguments, queries on non-existent columns, and the event ``count`` column
mapped onto ``reason``.
"""
from __future__ import annotations

import json
import os
import sqlite3
import threading
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

from kubedl_amd.persist import dmo

STOPPED = "Stopped"


@dataclass
class Query:
    """``backends.Query`` (query.go:25-41)."""
    job_id: str = ""
    name: str = ""
    namespace: str = ""
    region: str = ""
    status: str = ""
    start_time: str = ""
    end_time: str = ""
    is_del: Optional[int] = None
    page_num: int = 0
    page_size: int = 0


class ObjectStorageBackend:
    def initialize(self) -> None: ...
    def close(self) -> None: ...
    def name(self) -> str: ...
    def save_pod(self, pod: dict, default_container: str, region: str) -> None: ...
    def list_pods(self, job_id: str, region: str = "") -> List[dict]: ...
    def stop_pod(self, namespace: str, name: str, pod_id: str) -> None: ...
    def save_job(self, job: dict, region: str) -> None: ...
    def get_job(self, namespace: str, name: str, job_id: str, region: str = "") -> Optional[dict]: ...
    def list_jobs(self, q: Query) -> List[dict]: ...
    def stop_job(self, namespace: str, name: str, job_id: str, region: str = "") -> None: ...
    def delete_job(self, namespace: str, name: str, job_id: str, region: str = "") -> None: ...


class EventStorageBackend:
    def initialize(self) -> None: ...
    def close(self) -> None: ...
    def name(self) -> str: ...
    def save_event(self, event: dict, region: str) -> None: ...
    def list_events(self, job_namespace: str, job_name: str, start: str = "", end: str = "") -> List[dict]: ...


_JOB_COLS = ["name", "namespace", "job_id", "version", "status", "kind", "resources", "deploy_region",
             "tenant", "owner", "deleted", "is_in_etcd", "gmt_created", "gmt_modified", "gmt_finished"]
_POD_COLS = ["name", "namespace", "pod_id", "version", "status", "image", "job_id", "replica_type",
             "resources", "host_ip", "pod_ip", "deploy_region", "deleted", "is_in_etcd", "remark",
             "gmt_created", "gmt_modified", "gmt_started", "gmt_finished"]
_EVENT_COLS = ["name", "kind", "type", "obj_namespace", "obj_name", "obj_uid", "reason", "message", "count",
               "region", "first_timestamp", "last_timestamp"]


def _now() -> str:
    from kubedl_amd.api import common as c
    return c.now()


class SQLiteObjectBackend(ObjectStorageBackend):
    NAME = "sqlite"

    def __init__(self, path: str):
        self.path = path
        self.db: Optional[sqlite3.Connection] = None
        self._lock = threading.Lock()

    def name(self) -> str:
        return self.NAME

    def initialize(self) -> None:
        os.makedirs(os.path.dirname(os.path.abspath(self.path)) or ".", exist_ok=True)
        self.db = sqlite3.connect(self.path, check_same_thread=False, isolation_level=None)
        self.db.execute("PRAGMA journal_mode=WAL")
        self.db.execute("CREATE TABLE IF NOT EXISTS job_info (id INTEGER PRIMARY KEY AUTOINCREMENT, "
                        + ", ".join(f"{col} TEXT" for col in _JOB_COLS) + ")")
        self.db.execute("CREATE TABLE IF NOT EXISTS replica_info (id INTEGER PRIMARY KEY AUTOINCREMENT, "
                        + ", ".join(f"{col} TEXT" for col in _POD_COLS) + ")")
        self.db.execute("CREATE INDEX IF NOT EXISTS job_uid ON job_info(job_id)")
        self.db.execute("CREATE INDEX IF NOT EXISTS pod_uid ON replica_info(pod_id)")

    def close(self) -> None:
        if self.db is not None:
            self.db.close()
            self.db = None

    # ------------------------------------------------------------ helpers
    @staticmethod
    def _newer(new_v: str, old_v: str) -> bool:
        try:
            return int(new_v or 0) >= int(old_v or 0)
        except ValueError:
            return True

    def _upsert(self, table: str, cols: List[str], key_col: str, row: dict) -> None:
        with self._lock:
            cur = self.db.execute(f"SELECT id, version FROM {table} WHERE {key_col}=? AND namespace=? AND name=?",
                                  (row[key_col], row["namespace"], row["name"])).fetchone()
            row = dict(row)
            row["gmt_modified"] = _now()
            vals = [None if row.get(col) is None else str(row.get(col)) for col in cols]
            if cur is None:
                self.db.execute(f"INSERT INTO {table} ({', '.join(cols)}) VALUES ({', '.join('?' * len(cols))})",
                                vals)
            elif self._newer(row.get("version", ""), cur[1]):
                self.db.execute(f"UPDATE {table} SET {', '.join(f'{col}=?' for col in cols)} WHERE id=?",
                                vals + [cur[0]])

    def _rows(self, table: str, cols: List[str], where: str, args) -> List[dict]:
        with self._lock:
            cur = self.db.execute(f"SELECT {', '.join(cols)} FROM {table} {where}", args)
            out = []
            for r in cur.fetchall():
                d = dict(zip(cols, r))
                for k in ("deleted", "is_in_etcd", "count"):
                    if d.get(k) is not None:
                        d[k] = int(d[k])
                out.append(d)
            return out

    # ------------------------------------------------------------ pods
    def save_pod(self, pod: dict, default_container: str, region: str) -> None:
        self._upsert("replica_info", _POD_COLS, "pod_id", dmo.pod_to_dmo(pod, default_container, region))

    def list_pods(self, job_id: str, region: str = "") -> List[dict]:
        where, args = "WHERE job_id=?", [job_id]
        if region:
            where += " AND deploy_region=?"
            args.append(region)
        return self._rows("replica_info", _POD_COLS, where + " ORDER BY replica_type, name", args)

    def stop_pod(self, namespace: str, name: str, pod_id: str) -> None:
        with self._lock:
            row = self.db.execute("SELECT id, status FROM replica_info WHERE pod_id=? AND namespace=? AND name=?",
                                  (pod_id, namespace, name)).fetchone()
            if row is None:
                return
            status = row[1] if row[1] in ("Succeeded", "Failed") else STOPPED
            self.db.execute("UPDATE replica_info SET status=?, is_in_etcd='0', gmt_modified=?, "
                            "gmt_finished=COALESCE(gmt_finished, ?) WHERE id=?", (status, _now(), _now(), row[0]))

    # ------------------------------------------------------------ jobs
    def save_job(self, job: dict, region: str) -> None:
        self._upsert("job_info", _JOB_COLS, "job_id", dmo.job_to_dmo(job, region))

    def get_job(self, namespace: str, name: str, job_id: str, region: str = "") -> Optional[dict]:
        rows = self._rows("job_info", _JOB_COLS, "WHERE namespace=? AND name=? AND job_id=?",
                          (namespace, name, job_id))
        return rows[0] if rows else None

    def list_jobs(self, q: Query) -> List[dict]:
        conds, args = [], []
        for col, val in (("job_id", q.job_id), ("namespace", q.namespace), ("deploy_region", q.region),
                         ("status", q.status)):
            if val:
                conds.append(f"{col}=?")
                args.append(val)
        if q.name:
            conds.append("name LIKE ?")
            args.append(f"%{q.name}%")
        if q.start_time:
            conds.append("gmt_created >= ?")
            args.append(q.start_time)
        if q.end_time:
            conds.append("gmt_created <= ?")
            args.append(q.end_time)
        if q.is_del is not None:
            conds.append("deleted=?")
            args.append(str(q.is_del))
        where = ("WHERE " + " AND ".join(conds)) if conds else ""
        where += " ORDER BY gmt_created DESC"
        if q.page_size:
            where += f" LIMIT {int(q.page_size)} OFFSET {int(max(q.page_num - 1, 0) * q.page_size)}"
        return self._rows("job_info", _JOB_COLS, where, args)

    def stop_job(self, namespace: str, name: str, job_id: str, region: str = "") -> None:
        with self._lock:
            row = self.db.execute("SELECT id, status FROM job_info WHERE job_id=? AND namespace=? AND name=?",
                                  (job_id, namespace, name)).fetchone()
            if row is None:
                return
            status = row[1] if row[1] in ("Succeeded", "Failed") else STOPPED
            self.db.execute("UPDATE job_info SET status=?, is_in_etcd='0', gmt_modified=?, "
                            "gmt_finished=COALESCE(gmt_finished, ?) WHERE id=?", (status, _now(), _now(), row[0]))

    def delete_job(self, namespace: str, name: str, job_id: str, region: str = "") -> None:
        with self._lock:
            self.db.execute("UPDATE job_info SET deleted='1', is_in_etcd='0', gmt_modified=? "
                            "WHERE job_id=? AND namespace=? AND name=?", (_now(), job_id, namespace, name))


class SQLiteEventBackend(EventStorageBackend):
    NAME = "sqlite"

    def __init__(self, path: str):
        self.path = path
        self.db: Optional[sqlite3.Connection] = None
        self._lock = threading.Lock()

    def name(self) -> str:
        return self.NAME

    def initialize(self) -> None:
        os.makedirs(os.path.dirname(os.path.abspath(self.path)) or ".", exist_ok=True)
        self.db = sqlite3.connect(self.path, check_same_thread=False, isolation_level=None)
        self.db.execute("CREATE TABLE IF NOT EXISTS event_info ("
                        + ", ".join(f"{col} TEXT" for col in _EVENT_COLS) + ", PRIMARY KEY(name))")

    def close(self) -> None:
        if self.db is not None:
            self.db.close()
            self.db = None

    def save_event(self, event: dict, region: str) -> None:
        row = dmo.event_to_dmo(event, region)
        with self._lock:
            self.db.execute(f"INSERT OR REPLACE INTO event_info ({', '.join(_EVENT_COLS)}) VALUES "
                            f"({', '.join('?' * len(_EVENT_COLS))})",
                            [None if row.get(col) is None else str(row[col]) for col in _EVENT_COLS])

    def list_events(self, job_namespace: str, job_name: str, start: str = "", end: str = "") -> List[dict]:
        conds, args = ["obj_namespace=?", "(obj_name=? OR obj_name LIKE ?)"], [job_namespace, job_name,
                                                                             job_name + "-%"]
        if start:
            conds.append("first_timestamp >= ?")
            args.append(start)
        if end:
            conds.append("first_timestamp <= ?")
            args.append(end)
        with self._lock:
            rows = self.db.execute(f"SELECT {', '.join(_EVENT_COLS)} FROM event_info WHERE {' AND '.join(conds)} "
                                   "ORDER BY first_timestamp", args).fetchall()
        out = [dict(zip(_EVENT_COLS, r)) for r in rows]
        for d in out:
            d["count"] = int(d["count"] or 1)
        return out


class JSONLEventBackend(EventStorageBackend):
    """Append-only event log (the SLS logstore stand-in)."""
    NAME = "jsonl"

    def __init__(self, path: str):
        self.path = path
        self._lock = threading.Lock()

    def name(self) -> str:
        return self.NAME

    def initialize(self) -> None:
        os.makedirs(os.path.dirname(os.path.abspath(self.path)) or ".", exist_ok=True)
        open(self.path, "a").close()

    def close(self) -> None:
        pass

    def save_event(self, event: dict, region: str) -> None:
        row = dmo.event_to_dmo(event, region)
        with self._lock, open(self.path, "a") as f:
            f.write(json.dumps(row) + "\n")

    def list_events(self, job_namespace: str, job_name: str, start: str = "", end: str = "") -> List[dict]:
        latest: Dict[tuple, dict] = {}
        with self._lock, open(self.path) as f:
            for line in f:
                try:
                    r = json.loads(line)
                except ValueError:
                    continue
                if r.get("obj_namespace") != job_namespace:
                    continue
                if r.get("obj_name") != job_name and not str(r.get("obj_name", "")).startswith(job_name + "-"):
                    continue
                if start and (r.get("first_timestamp") or "") < start:
                    continue
                if end and (r.get("first_timestamp") or "") > end:
                    continue
                latest[(r.get("obj_uid"), r.get("reason"), r.get("message"))] = r
        return sorted(latest.values(), key=lambda r: r.get("first_timestamp") or "")


# ---------------------------------------------------------------- registry
_lock = threading.Lock()
_object_ctors: Dict[str, Callable[[str], ObjectStorageBackend]] = {}
_event_ctors: Dict[str, Callable[[str], EventStorageBackend]] = {}


def register_object_backend(name: str, ctor) -> None:
    with _lock:
        _object_ctors[name] = ctor


def register_event_backend(name: str, ctor) -> None:
    with _lock:
        _event_ctors[name] = ctor


def new_object_backend(name: str, home: str) -> ObjectStorageBackend:
    with _lock:
        ctor = _object_ctors.get(name)
    if ctor is None:
        raise KeyError(f"unknown object storage backend {name!r}; known: {sorted(_object_ctors)}")
    return ctor(home)


def new_event_backend(name: str, home: str) -> EventStorageBackend:
    with _lock:
        ctor = _event_ctors.get(name)
    if ctor is None:
        raise KeyError(f"unknown event storage backend {name!r}; known: {sorted(_event_ctors)}")
    return ctor(home)


register_object_backend("sqlite", lambda home: SQLiteObjectBackend(os.path.join(home, "persist.db")))
register_event_backend("sqlite", lambda home: SQLiteEventBackend(os.path.join(home, "persist.db")))
register_event_backend("jsonl", lambda home: JSONLEventBackend(os.path.join(home, "events.jsonl")))
