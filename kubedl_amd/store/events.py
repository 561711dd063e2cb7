"""Event recorder (``record.EventRecorder`` equivalent).

Every create/delete/transition the reference announces with
``Recorder.Event(f)`` (e.g. ``pkg/job_controller/pod.go:291,367,421-430``,
``service.go:310-327`` and the per-kind status files) becomes a ``core/v1``
``Event`` object in the store.  Identical events (same involved object, type,
reason and message) are aggregated by bumping ``count`` and
``lastTimestamp``, like the client-go correlator does.
"""
from __future__ import annotations

import threading
import uuid
from typing import Any, Dict, List

from kubedl_amd.api import common as c
from kubedl_amd.store.store import NotFound, Store

NORMAL = "Normal"
WARNING = "Warning"


class EventRecorder:
    def __init__(self, store: Store, component: str = "kubedl"):
        self.store = store
        self.component = component
        self._lock = threading.Lock()
        self._index: Dict[tuple, str] = {}

    def event(self, obj: Dict[str, Any], etype: str, reason: str, message: str) -> None:
        md = obj.get("metadata") or {}
        ns = md.get("namespace", "default")
        key = (md.get("uid"), etype, reason, message)
        ts = c.now()
        with self._lock:
            name = self._index.get(key)
            if name is not None:
                try:
                    def bump(ev):
                        ev["count"] = int(ev.get("count", 1)) + 1
                        ev["lastTimestamp"] = ts
                    self.store.patch("Event", ns, name, bump)
                    return
                except NotFound:
                    self._index.pop(key, None)
            name = f"{md.get('name')}.{uuid.uuid4().hex[:16]}"
            ev = {
                "apiVersion": "v1", "kind": "Event",
                "metadata": {"name": name, "namespace": ns},
                "involvedObject": {"kind": obj.get("kind"), "namespace": ns, "name": md.get("name"),
                                   "uid": md.get("uid"), "apiVersion": obj.get("apiVersion"),
                                   "resourceVersion": md.get("resourceVersion")},
                "reason": reason, "message": message, "type": etype, "count": 1,
                "firstTimestamp": ts, "lastTimestamp": ts,
                "source": {"component": self.component},
            }
            self.store.create(ev)
            self._index[key] = name

    def eventf(self, obj, etype, reason, fmt, *args) -> None:
        self.event(obj, etype, reason, fmt % args if args else fmt)

    def events_for(self, obj: Dict[str, Any]) -> List[Dict[str, Any]]:
        md = obj.get("metadata") or {}
        evs = [e for e in self.store.list("Event", md.get("namespace"))
               if (e.get("involvedObject") or {}).get("uid") == md.get("uid")]
        evs.sort(key=lambda e: e.get("firstTimestamp", ""))
        return evs
