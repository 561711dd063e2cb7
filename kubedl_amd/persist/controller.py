"""Persist controllers (``controllers/persist``): mirror jobs, pods and events
into the configured storage backends.

* jobs of every kind: saved on every change; when the job leaves the store
  it is stopped (``StopJob``) and marked deleted (``DeleteJob``) -- keyed by
  ``<uid>/<name>`` so a re-created job never overwrites the old row
  (``job_persist_controller.go:46-123``); [fix] the reference deletes with the
  empty name/namespace of the not-found object (``tfjob_persist_controller.go:68``),
  we use the last known identity;
* pods owned by a KubeDL job (owner kind is one of the four kinds and the pod
  carries ``group-name``): saved, and stopped when deleted
  (``pod_persist_controller.go:50-140``, ``persist/util/filter.go:26-41``);
* events whose involved object is a KubeDL job or a KubeDL pod (a pod that no
  longer exists counts as managed) (``events_event_handler.go:25-108``).

Writes happen on a dedicated worker thread fed by the store watch, so a slow
backend never stalls reconciles.
"""
from __future__ import annotations

import logging
import queue
import threading
from typing import Optional

from kubedl_amd.api import common as c
from kubedl_amd.api import kinds as K
from kubedl_amd.persist.backends import new_event_backend, new_object_backend
from kubedl_amd.store import DELETED, Store

log = logging.getLogger("kubedl_amd.persist")


def is_kubedl_managed_pod(pod: dict) -> bool:
    md = pod.get("metadata") or {}
    if c.GROUP_NAME_LABEL not in (md.get("labels") or {}):
        return False
    return any(r.get("kind") in K.BY_KIND for r in md.get("ownerReferences") or [])


class PersistController:
    def __init__(self, store: Store, home: str, object_storage: str = "", event_storage: str = "",
                 region: str = ""):
        self.store = store
        self.region = region
        self.objects = new_object_backend(object_storage, home) if object_storage else None
        self.events = new_event_backend(event_storage, home) if event_storage else None
        self._q: "queue.Queue" = queue.Queue()
        self._thread: Optional[threading.Thread] = None
        self._cancel = None
        self._known_pods = {}

    def start(self) -> None:
        if self.objects:
            self.objects.initialize()
        if self.events:
            self.events.initialize()
        self._cancel = self.store.watch(lambda et, o: self._q.put((et, o)))
        self._thread = threading.Thread(target=self._run, name="kdl-persist", daemon=True)
        self._thread.start()
        # initial sync of what the store already holds
        for kind in K.BY_KIND:
            for j in self.store.list(kind):
                self._q.put(("ADDED", j))

    def stop(self) -> None:
        if self._cancel:
            self._cancel()
        self._q.put(None)
        if self._thread:
            self._thread.join(timeout=10)
        if self.objects:
            self.objects.close()
        if self.events:
            self.events.close()

    def flush(self, timeout: float = 10.0) -> None:
        done = threading.Event()
        self._q.put(("__flush__", done))
        done.wait(timeout)

    def _run(self) -> None:
        while True:
            item = self._q.get()
            if item is None:
                return
            etype, obj = item
            if etype == "__flush__":
                obj.set()
                continue
            try:
                self._handle(etype, obj)
            except Exception:
                log.exception("persist %s %s failed", etype, obj.get("kind"))

    def _handle(self, etype: str, obj: dict) -> None:
        kind = obj.get("kind")
        md = obj.get("metadata") or {}
        if kind in K.BY_KIND and self.objects:
            if etype == DELETED:
                self.objects.stop_job(md["namespace"], md["name"], md.get("uid", ""), self.region)
                self.objects.delete_job(md["namespace"], md["name"], md.get("uid", ""), self.region)
            else:
                self.objects.save_job(obj, self.region)
        elif kind == "Pod" and self.objects and is_kubedl_managed_pod(obj):
            self._known_pods[md.get("uid")] = True
            if etype == DELETED:
                self.objects.stop_pod(md["namespace"], md["name"], md.get("uid", ""))
            else:
                owner = next(r for r in md.get("ownerReferences") or [] if r.get("kind") in K.BY_KIND)
                self.objects.save_pod(obj, K.BY_KIND[owner["kind"]].default_container, self.region)
        elif kind == "Event" and self.events and etype != DELETED:
            io = obj.get("involvedObject") or {}
            if io.get("kind") in K.BY_KIND:
                self.events.save_event(obj, self.region)
            elif io.get("kind") == "Pod":
                pod = self.store.try_get("Pod", io.get("namespace", "default"), io.get("name", ""))
                if pod is None or is_kubedl_managed_pod(pod):
                    self.events.save_event(obj, self.region)
