"""Rate-limited, de-duplicating work queue (client-go ``workqueue`` semantics).

* ``add(key)``: a key is queued at most once; a key being processed is marked
  dirty and re-queued when ``done`` is called (one worker per key at a time --
  the reference's reconcile concurrency model, SURVEY.md §5 "Race detection").
* ``add_after(key, delay)``: delayed enqueue (TTL requeue, ``RequeueAfter``).
* ``add_rate_limited(key)`` / ``forget(key)`` / ``num_requeues(key)``: per-item
  exponential backoff; ``num_requeues`` is what ``ReconcileJobs`` reads as
  ``previousRetry`` (``pkg/job_controller/job.go:119``) and what the
  ``BackoffStatesQueue`` exists for (``job_controller.go:28-46``).
"""
from __future__ import annotations

import heapq
import itertools
import threading
import time
from typing import Dict, Hashable, List, Optional, Set, Tuple


class RateLimitingQueue:
    def __init__(self, base_delay: float = 0.005, max_delay: float = 1000.0):
        self._cv = threading.Condition()
        self._queue: List[Hashable] = []
        self._dirty: Set[Hashable] = set()
        self._processing: Set[Hashable] = set()
        self._waiting: List[Tuple[float, int, Hashable]] = []
        self._seq = itertools.count()
        self._failures: Dict[Hashable, int] = {}
        self._base = base_delay
        self._max = max_delay
        self._shutdown = False

    # ---------------------------------------------------------------- basic
    def add(self, key: Hashable) -> None:
        with self._cv:
            if self._shutdown or key in self._dirty:
                return
            self._dirty.add(key)
            if key in self._processing:
                return
            self._queue.append(key)
            self._cv.notify()

    def __len__(self) -> int:
        with self._cv:
            return len(self._queue)

    def get(self, timeout: Optional[float] = None) -> Tuple[Optional[Hashable], bool]:
        """Block for the next key.  Returns ``(key, shutdown)``."""
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cv:
            while True:
                self._promote_waiting_locked()
                if self._queue:
                    key = self._queue.pop(0)
                    self._processing.add(key)
                    self._dirty.discard(key)
                    return key, False
                if self._shutdown:
                    return None, True
                wait = None
                if self._waiting:
                    wait = max(0.0, self._waiting[0][0] - time.monotonic())
                if deadline is not None:
                    rem = deadline - time.monotonic()
                    if rem <= 0:
                        return None, False
                    wait = rem if wait is None else min(wait, rem)
                self._cv.wait(wait)

    def done(self, key: Hashable) -> None:
        with self._cv:
            self._processing.discard(key)
            if key in self._dirty:
                self._queue.append(key)
                self._cv.notify()

    def shutdown(self) -> None:
        with self._cv:
            self._shutdown = True
            self._cv.notify_all()

    @property
    def shutting_down(self) -> bool:
        return self._shutdown

    # ---------------------------------------------------------------- delayed
    def add_after(self, key: Hashable, delay: float) -> None:
        if delay <= 0:
            self.add(key)
            return
        with self._cv:
            if self._shutdown:
                return
            heapq.heappush(self._waiting, (time.monotonic() + delay, next(self._seq), key))
            self._cv.notify()

    def _promote_waiting_locked(self) -> None:
        now = time.monotonic()
        while self._waiting and self._waiting[0][0] <= now:
            _, _, key = heapq.heappop(self._waiting)
            if key in self._dirty:
                continue
            self._dirty.add(key)
            if key not in self._processing:
                self._queue.append(key)

    # ---------------------------------------------------------------- rate limit
    def when(self, key: Hashable) -> float:
        with self._cv:
            n = self._failures.get(key, 0)
            self._failures[key] = n + 1
        return min(self._base * (2 ** n), self._max)

    def add_rate_limited(self, key: Hashable) -> None:
        self.add_after(key, self.when(key))

    def forget(self, key: Hashable) -> None:
        with self._cv:
            self._failures.pop(key, None)

    def num_requeues(self, key: Hashable) -> int:
        with self._cv:
            return self._failures.get(key, 0)

    def idle(self) -> bool:
        with self._cv:
            return not self._queue and not self._processing and not self._waiting
