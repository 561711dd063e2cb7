"""ControllerExpectations (k8s ``controller.ControllerExpectations``).

The reconcile loop must not act on a stale view of pods/services it just
created or deleted.  Before each create (delete) it raises the expected
count for ``<ns>/<job>/<rtype>/pods|services``; the watch handlers lower it
when the creation (deletion) is observed.  ``satisfied`` gates reconcile
(``pkg/job_controller/expectations.go:11-27``).  Expectations older than a
TTL are considered satisfied so a lost event can never wedge a job.
"""
from __future__ import annotations

import threading
import time
from typing import Dict, List


class Expectations:
    TTL = 300.0

    def __init__(self, ttl: float | None = None):
        self._lock = threading.Lock()
        self._exp: Dict[str, List[float]] = {}  # key -> [add, del, timestamp]
        self.ttl = self.TTL if ttl is None else ttl

    def expect_creations(self, key: str, n: int) -> None:
        self._raise(key, n, 0)

    def expect_deletions(self, key: str, n: int) -> None:
        self._raise(key, 0, n)

    def _raise(self, key: str, add: int, dele: int) -> None:
        with self._lock:
            e = self._exp.get(key)
            if e is None:
                self._exp[key] = [add, dele, time.monotonic()]
            else:
                e[0] += add
                e[1] += dele
                e[2] = time.monotonic()

    def creation_observed(self, key: str) -> None:
        with self._lock:
            e = self._exp.get(key)
            if e is not None and e[0] > 0:
                e[0] -= 1

    def deletion_observed(self, key: str) -> None:
        with self._lock:
            e = self._exp.get(key)
            if e is not None and e[1] > 0:
                e[1] -= 1

    def satisfied_key(self, key: str) -> bool:
        with self._lock:
            e = self._exp.get(key)
            if e is None:
                return True
            if e[0] <= 0 and e[1] <= 0:
                return True
            return time.monotonic() - e[2] > self.ttl

    def satisfied(self, keys) -> bool:
        """SatisfyExpectations: every pods/services key of the job is fulfilled."""
        return all(self.satisfied_key(k) for k in keys)

    def delete(self, key: str) -> None:
        with self._lock:
            self._exp.pop(key, None)

    def delete_prefix(self, prefix: str) -> None:
        with self._lock:
            for k in [k for k in self._exp if k.startswith(prefix)]:
                self._exp.pop(k, None)

    def get(self, key: str):
        with self._lock:
            e = self._exp.get(key)
            return None if e is None else (e[0], e[1])
