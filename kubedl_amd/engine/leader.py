"""Leader election for the controller manager on one node.

Reference: ``main.go:56-57,73`` turns controller-runtime's leader election ON by
default ("ensure there is only one active controller manager").  There it is a
ConfigMap/Lease lock in the API server; here the managers that could race are
processes sharing one ``--home`` (one store, one node runtime, one GPU pool), so
the lock is an exclusive ``flock`` on ``<home>/leader.lock``:

* the first manager takes it and runs the controllers, scheduler and kubelet;
* a second manager on the same home blocks as a standby (it does not open the
  store or spawn ranks -- two kubelets would double-spawn onto the same GPUs);
* the kernel releases the lock when the leader exits (cleanly or killed), and
  the standby takes over, loading the durable store and re-reconciling.

``flock`` locks belong to the open file description, so two managers inside ONE
process (tests) exclude each other as well as two processes do.
"""
from __future__ import annotations

import fcntl
import json
import logging
import os
import socket
import time
from typing import Optional

log = logging.getLogger("kubedl_amd.leader")

LOCK_NAME = "leader.lock"


class LeaderLock:
    def __init__(self, home: str, identity: Optional[str] = None):
        self.path = os.path.join(home, LOCK_NAME)
        self.identity = identity or f"{socket.gethostname()}_{os.getpid()}"
        self._fd: Optional[int] = None

    @property
    def held(self) -> bool:
        return self._fd is not None

    def holder(self) -> dict:
        """The current leader's record (best effort; {} when none was written)."""
        try:
            with open(self.path) as f:
                return json.loads(f.read() or "{}")
        except (OSError, ValueError):
            return {}

    def try_acquire(self) -> bool:
        if self._fd is not None:
            return True
        os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
        fd = os.open(self.path, os.O_RDWR | os.O_CREAT, 0o644)
        try:
            fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
        except OSError:
            os.close(fd)
            return False
        rec = json.dumps({"holderIdentity": self.identity, "acquireTime": time.time()}).encode()
        os.ftruncate(fd, 0)
        os.pwrite(fd, rec, 0)
        self._fd = fd
        return True

    def acquire(self, timeout: Optional[float] = None, poll: float = 0.2, stop=None) -> bool:
        """Block until leader (True), ``timeout`` passes or ``stop()`` is true (False)."""
        deadline = None if timeout is None else time.time() + timeout
        logged = False
        while not self.try_acquire():
            if not logged:
                log.info("attempting to acquire leader lease %s (held by %s)", self.path,
                         self.holder().get("holderIdentity", "?"))
                logged = True
            if (deadline is not None and time.time() >= deadline) or (stop is not None and stop()):
                return False
            time.sleep(poll)
        log.info("successfully acquired lease %s as %s", self.path, self.identity)
        return True

    def release(self) -> None:
        if self._fd is None:
            return
        try:
            fcntl.flock(self._fd, fcntl.LOCK_UN)
        finally:
            os.close(self._fd)
            self._fd = None
