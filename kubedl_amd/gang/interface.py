"""``GangScheduler`` interface and registry.

Reference: ``pkg/gang_schedule/interface.go:30-52`` (CreateGang, BindPodToGang,
GetGang, DeleteGang, Name) and ``registry/registry.go:27-73`` (a global
name -> scheduler map guarded by a mutex; ``RegisterGangSchedulers``
instantiates every registered constructor).
"""
from __future__ import annotations

import threading
from typing import Callable, Dict, List, Optional


class GangScheduler:
    """A gang scheduler makes the pods of one job schedulable all-or-nothing."""

    def create_gang(self, job: dict, replicas: Dict[str, dict]) -> dict:
        raise NotImplementedError

    def bind_pod_to_gang(self, pod_template: dict, entity: dict) -> None:
        raise NotImplementedError

    def get_gang(self, namespace: str, name: str) -> Optional[dict]:
        raise NotImplementedError

    def delete_gang(self, namespace: str, name: str) -> None:
        raise NotImplementedError

    def name(self) -> str:
        raise NotImplementedError


_lock = threading.Lock()
_constructors: Dict[str, Callable[..., GangScheduler]] = {}
_instances: Dict[str, GangScheduler] = {}


def register(name: str, ctor: Callable[..., GangScheduler]) -> None:
    with _lock:
        _constructors[name] = ctor


def register_gang_schedulers(store, **kw) -> None:
    with _lock:
        for n, ctor in _constructors.items():
            _instances[n] = ctor(store, **kw)


def get(name: str) -> Optional[GangScheduler]:
    with _lock:
        return _instances.get(name)


def names() -> List[str]:
    with _lock:
        return sorted(_constructors)
