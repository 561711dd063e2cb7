"""SIGINT/SIGTERM handling (``pkg/util/signals/signal.go:27-43``).

``setup_signal_handler()`` returns a ``threading.Event`` set on the first
SIGINT or SIGTERM; a second signal exits the process with status 1.  It can be
installed once per process (the reference panics on a second call).
"""
from __future__ import annotations

import os
import signal
import threading

_installed = False


def setup_signal_handler() -> threading.Event:
    global _installed
    if _installed:
        raise RuntimeError("setup_signal_handler called twice")
    _installed = True
    stop = threading.Event()

    def _handler(signum, frame):
        if stop.is_set():
            os._exit(1)  # second signal: exit directly
        stop.set()

    for s in (signal.SIGINT, signal.SIGTERM):
        signal.signal(s, _handler)
    return stop
