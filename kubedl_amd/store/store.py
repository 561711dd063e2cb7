"""Local object store + watch bus: the API-server stand-in for one MI355X node.

KubeDL talks to a Kubernetes API server for every object it reads or writes
(boundary (a)).  On a single node we replace it with an
in-process store that keeps the same object model:

* objects are JSON-shaped dicts keyed by ``(kind, namespace, name)`` with
  ``metadata.uid``, ``resourceVersion`` (monotonic, optimistic concurrency on
  update), ``generation`` (bumped on spec change), ``creationTimestamp``,
  ``deletionTimestamp``, labels, annotations and ``ownerReferences``;
* ``delete`` cascades to dependents through ``ownerReferences`` the way the
  k8s garbage collector does for pods/services owned by a job
  (reference relies on k8s GC: SURVEY.md §3.4);
* ``watch`` delivers ``ADDED`` / ``MODIFIED`` / ``DELETED`` events to
  subscribers (controllers' informers) synchronously after the write is
  committed and the lock released, so handlers may write back;
* an optional sqlite file makes the store durable (the "etcd"): every
  committed write is journaled and reloaded on restart;
* a service port table maps ``<namespace>/<service>:<containerPort>`` to a
  unique 127.0.0.1 port so two jobs that both ask for port 23456 can run side
  by side (headless-Service DNS replacement).
"""
from __future__ import annotations

import copy
import itertools
import json
import os
import socket
import sqlite3
import threading
import time
import uuid
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple

from kubedl_amd.api import common as c

ADDED, MODIFIED, DELETED = "ADDED", "MODIFIED", "DELETED"

Key = Tuple[str, str, str]


class NotFound(KeyError):
    pass


class AlreadyExists(ValueError):
    pass


class Conflict(RuntimeError):
    pass


def obj_key(obj: Dict[str, Any]) -> Key:
    md = obj.get("metadata") or {}
    return obj["kind"], md.get("namespace", "default") or "default", md["name"]


def match_labels(obj: Dict[str, Any], selector: Optional[Dict[str, str]]) -> bool:
    if not selector:
        return True
    labels = (obj.get("metadata") or {}).get("labels") or {}
    return all(labels.get(k) == v for k, v in selector.items())


class Store:
    def __init__(self, db_path: Optional[str] = None, port_range: Tuple[int, int] = (20000, 45000)):
        self._lock = threading.RLock()
        self._objs: Dict[Key, Dict[str, Any]] = {}
        self._rv = itertools.count(1)
        self._watchers: List[Tuple[Optional[str], Callable[[str, Dict[str, Any]], None]]] = []
        self._ports: Dict[str, int] = {}
        self._port_range = port_range
        # start the scan at a per-store offset: two control planes on one host
        # (parallel test workers, two `kdl` homes) would otherwise hand out the
        # same first port between its free-check and the rank's bind
        self._next_port = port_range[0] + (os.getpid() * 7919 + time.monotonic_ns()) % (port_range[1] - port_range[0])
        self._db: Optional[sqlite3.Connection] = None
        if db_path:
            self._open_db(db_path)

    # ------------------------------------------------------------ durability
    def _open_db(self, path: str) -> None:
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        self._db = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
        self._db.execute("PRAGMA journal_mode=WAL")
        self._db.execute("CREATE TABLE IF NOT EXISTS objects (kind TEXT, namespace TEXT, name TEXT, "
                         "rv INTEGER, body TEXT, PRIMARY KEY(kind, namespace, name))")
        self._db.execute("CREATE TABLE IF NOT EXISTS ports (key TEXT PRIMARY KEY, port INTEGER)")
        max_rv = 0
        for kind, ns, name, rv, body in self._db.execute("SELECT kind, namespace, name, rv, body FROM objects"):
            self._objs[(kind, ns, name)] = json.loads(body)
            max_rv = max(max_rv, int(rv))
        for key, port in self._db.execute("SELECT key, port FROM ports"):
            self._ports[key] = int(port)
        self._rv = itertools.count(max_rv + 1)

    def _journal_put(self, obj: Dict[str, Any]) -> None:
        if self._db is None:
            return
        k = obj_key(obj)
        self._db.execute("INSERT OR REPLACE INTO objects VALUES (?,?,?,?,?)",
                         (k[0], k[1], k[2], int(obj["metadata"]["resourceVersion"]), json.dumps(obj)))

    def _journal_del(self, k: Key) -> None:
        if self._db is None:
            return
        self._db.execute("DELETE FROM objects WHERE kind=? AND namespace=? AND name=?", k)

    def close(self) -> None:
        if self._db is not None:
            self._db.close()
            self._db = None

    # ------------------------------------------------------------ watch bus
    def watch(self, handler: Callable[[str, Dict[str, Any]], None], kind: Optional[str] = None):
        """Subscribe ``handler(event_type, obj_copy)``; returns an unsubscribe fn."""
        entry = (kind, handler)
        with self._lock:
            self._watchers.append(entry)

        def cancel():
            with self._lock:
                if entry in self._watchers:
                    self._watchers.remove(entry)
        return cancel

    def _emit(self, events: Iterable[Tuple[str, Dict[str, Any]]]) -> None:
        with self._lock:
            watchers = list(self._watchers)
        for etype, obj in events:
            for kind, h in watchers:
                if kind is None or kind == obj.get("kind"):
                    try:
                        h(etype, copy.deepcopy(obj))
                    except Exception as e:  # a broken handler must not break writers
                        import logging
                        logging.getLogger("kubedl_amd.store").exception("watch handler failed: %s", e)

    # ------------------------------------------------------------ CRUD
    def create(self, obj: Dict[str, Any]) -> Dict[str, Any]:
        obj = copy.deepcopy(obj)
        md = obj.setdefault("metadata", {})
        if not md.get("name"):
            gen = md.get("generateName")
            if not gen:
                raise ValueError("metadata.name is required")
            md["name"] = gen + uuid.uuid4().hex[:5]
        md.setdefault("namespace", "default")
        if not md["namespace"]:
            md["namespace"] = "default"
        k = obj_key(obj)
        with self._lock:
            if k in self._objs:
                raise AlreadyExists(f"{k[0]} {k[1]}/{k[2]} already exists")
            md["uid"] = md.get("uid") or str(uuid.uuid4())
            md["resourceVersion"] = str(next(self._rv))
            md["generation"] = 1
            md.setdefault("creationTimestamp", c.now())
            self._objs[k] = obj
            self._journal_put(obj)
            out = copy.deepcopy(obj)
        self._emit([(ADDED, out)])
        return out

    def get(self, kind: str, namespace: str, name: str) -> Dict[str, Any]:
        with self._lock:
            o = self._objs.get((kind, namespace or "default", name))
            if o is None:
                raise NotFound(f"{kind} {namespace}/{name} not found")
            return copy.deepcopy(o)

    def try_get(self, kind: str, namespace: str, name: str) -> Optional[Dict[str, Any]]:
        try:
            return self.get(kind, namespace, name)
        except NotFound:
            return None

    def list(self, kind: str, namespace: Optional[str] = None,
             labels: Optional[Dict[str, str]] = None) -> List[Dict[str, Any]]:
        with self._lock:
            out = [copy.deepcopy(o) for (k, ns, _), o in self._objs.items()
                   if k == kind and (namespace is None or ns == namespace) and match_labels(o, labels)]
        out.sort(key=lambda o: (o["metadata"]["namespace"], o["metadata"]["name"]))
        return out

    def kinds(self) -> List[str]:
        with self._lock:
            return sorted({k for k, _, _ in self._objs})

    def _update(self, obj: Dict[str, Any], status_only: bool, check_rv: bool) -> Dict[str, Any]:
        k = obj_key(obj)
        with self._lock:
            cur = self._objs.get(k)
            if cur is None:
                raise NotFound(f"{k[0]} {k[1]}/{k[2]} not found")
            rv = (obj.get("metadata") or {}).get("resourceVersion")
            if check_rv and rv is not None and rv != cur["metadata"]["resourceVersion"]:
                raise Conflict(f"{k[0]} {k[1]}/{k[2]}: resourceVersion {rv} != "
                               f"{cur['metadata']['resourceVersion']}")
            new = copy.deepcopy(cur)
            if status_only:
                new["status"] = copy.deepcopy(obj.get("status"))
            else:
                for f in obj:
                    if f in ("metadata", "status"):
                        continue
                    new[f] = copy.deepcopy(obj[f])
                for f in ("labels", "annotations", "ownerReferences", "finalizers"):
                    if f in obj.get("metadata", {}):
                        new["metadata"][f] = copy.deepcopy(obj["metadata"][f])
                if "status" in obj and k[0] in ("Pod", "Service", "Event", "PodGroup"):
                    new["status"] = copy.deepcopy(obj["status"])
                if json.dumps(new.get("spec"), sort_keys=True) != json.dumps(cur.get("spec"), sort_keys=True):
                    new["metadata"]["generation"] = int(cur["metadata"].get("generation", 1)) + 1
            if new == cur:
                return copy.deepcopy(cur)
            new["metadata"]["resourceVersion"] = str(next(self._rv))
            self._objs[k] = new
            self._journal_put(new)
            out = copy.deepcopy(new)
        self._emit([(MODIFIED, out)])
        return out

    def update(self, obj: Dict[str, Any], check_rv: bool = False) -> Dict[str, Any]:
        return self._update(obj, status_only=False, check_rv=check_rv)

    def update_status(self, obj: Dict[str, Any], check_rv: bool = False) -> Dict[str, Any]:
        return self._update(obj, status_only=True, check_rv=check_rv)

    def patch(self, kind: str, namespace: str, name: str,
              fn: Callable[[Dict[str, Any]], None]) -> Dict[str, Any]:
        """Read-modify-write under the store lock (no lost updates)."""
        with self._lock:
            cur = self.get(kind, namespace, name)
            fn(cur)
            cur.setdefault("metadata", {})["resourceVersion"] = None
            return self._update(cur, status_only=False, check_rv=False)

    def delete(self, kind: str, namespace: str, name: str, cascade: bool = True) -> Dict[str, Any]:
        events = []
        with self._lock:
            k = (kind, namespace or "default", name)
            o = self._objs.pop(k, None)
            if o is None:
                raise NotFound(f"{kind} {namespace}/{name} not found")
            self._journal_del(k)
            o["metadata"]["deletionTimestamp"] = c.now()
            events.append((DELETED, copy.deepcopy(o)))
            if cascade:
                events.extend(self._collect_dependents(o["metadata"]["uid"]))
            if kind == "Service":
                self._release_ports(namespace or "default", name)
        self._emit(events)
        return events[0][1]

    def _collect_dependents(self, uid: str) -> List[Tuple[str, Dict[str, Any]]]:
        out = []
        dependents = [k for k, o in self._objs.items()
                      if any(r.get("uid") == uid for r in (o["metadata"].get("ownerReferences") or []))]
        for k in dependents:
            o = self._objs.pop(k, None)
            if o is None:
                continue
            self._journal_del(k)
            o["metadata"]["deletionTimestamp"] = c.now()
            out.append((DELETED, copy.deepcopy(o)))
            if k[0] == "Service":
                self._release_ports(k[1], k[2])
            out.extend(self._collect_dependents(o["metadata"]["uid"]))
        return out

    # ------------------------------------------------------------ service ports
    def host_port(self, namespace: str, service: str, container_port: int) -> int:
        """Stable 127.0.0.1 port standing in for ``<service>.<ns>.svc:<containerPort>``."""
        key = f"{namespace}/{service}:{int(container_port)}"
        with self._lock:
            p = self._ports.get(key)
            if p is not None:
                return p
            used = set(self._ports.values())
            lo, hi = self._port_range
            for _ in range(hi - lo):
                cand = self._next_port
                self._next_port = lo + (self._next_port + 1 - lo) % (hi - lo)
                if cand in used or not _port_free(cand):
                    continue
                self._ports[key] = cand
                if self._db is not None:
                    self._db.execute("INSERT OR REPLACE INTO ports VALUES (?,?)", (key, cand))
                return cand
            raise RuntimeError("no free local port for service")

    def _release_ports(self, namespace: str, service: str) -> None:
        pref = f"{namespace}/{service}:"
        for key in [k for k in self._ports if k.startswith(pref)]:
            self._ports.pop(key, None)
            if self._db is not None:
                self._db.execute("DELETE FROM ports WHERE key=?", (key,))

    def port_table(self) -> Dict[str, int]:
        with self._lock:
            return dict(self._ports)


def _port_free(port: int) -> bool:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind(("127.0.0.1", port))
        return True
    except OSError:
        return False
    finally:
        s.close()
