"""Structured loggers bound to a job / replica type / pod / workqueue key.

Reference: ``pkg/util/logger.go:26-80`` (logrus ``WithFields``).  Here a
``logging.LoggerAdapter`` carries the fields; the default formatter appends
them as ``key=value`` pairs, and ``logging.LogRecord.kdl_fields`` keeps them
for structured handlers.  Jobs and pods are the object dicts of
``kubedl_amd.store`` (``metadata.namespace/name/uid/ownerReferences``).
"""
from __future__ import annotations

import logging
from typing import Any, Dict, Optional

_BASE = logging.getLogger("kubedl")


class FieldsAdapter(logging.LoggerAdapter):
    """Appends ``k=v`` fields to every message (logrus text-format style)."""

    def process(self, msg, kwargs):
        fields: Dict[str, Any] = dict(self.extra or {})
        extra = kwargs.setdefault("extra", {})
        extra["kdl_fields"] = fields
        tail = " ".join(f"{k}={v}" for k, v in fields.items())
        return (f"{msg} {tail}" if tail else msg), kwargs

    def with_fields(self, **fields) -> "FieldsAdapter":
        merged = dict(self.extra or {})
        merged.update(fields)
        return FieldsAdapter(self.logger, merged)


def _meta(obj: dict) -> dict:
    return obj.get("metadata") or {}


def _dotted(ns: str, name: str) -> str:
    # the reference logs "namespace.name" (matches the controller's key logging)
    return f"{ns}.{name}"


def logger_for_job(job: dict, logger: Optional[logging.Logger] = None) -> FieldsAdapter:
    md = _meta(job)
    return FieldsAdapter(logger or _BASE, {"job": _dotted(md.get("namespace", ""), md.get("name", "")),
                                           "uid": md.get("uid", "")})


def logger_for_replica(job: dict, rtype: str, logger: Optional[logging.Logger] = None) -> FieldsAdapter:
    return logger_for_job(job, logger).with_fields(**{"replica-type": rtype})


def logger_for_pod(pod: dict, kind: str, logger: Optional[logging.Logger] = None) -> FieldsAdapter:
    """``job`` is set only when the pod's controller owner is of ``kind``."""
    md = _meta(pod)
    job = ""
    for ref in md.get("ownerReferences") or []:
        if ref.get("controller"):
            if ref.get("kind") == kind:
                job = _dotted(md.get("namespace", ""), ref.get("name", ""))
            break
    return FieldsAdapter(logger or _BASE, {"job": job, "pod": _dotted(md.get("namespace", ""), md.get("name", "")),
                                           "uid": md.get("uid", "")})


def logger_for_key(key: str, logger: Optional[logging.Logger] = None) -> FieldsAdapter:
    """Workqueue key ``namespace/name`` -> ``job=namespace.name``."""
    return FieldsAdapter(logger or _BASE, {"job": key.replace("/", ".")})


def logger_for_unstructured(obj: dict, kind: str, logger: Optional[logging.Logger] = None) -> FieldsAdapter:
    md = _meta(obj)
    job = _dotted(md.get("namespace", ""), md.get("name", "")) if obj.get("kind") == kind else ""
    return FieldsAdapter(logger or _BASE, {"job": job, "uid": md.get("uid", "")})
