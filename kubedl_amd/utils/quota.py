"""Container resource arithmetic (``pkg/util/quota/resources.go:8-35``).

Quantities use the Kubernetes string forms (``"500m"``, ``"2Gi"``, ``"1"``) and
are parsed exactly (``persist/dmo.parse_quantity``, a ``Fraction``).
"""
from __future__ import annotations

from typing import Dict, Iterable

from kubedl_amd.persist.dmo import format_quantity, parse_quantity, _is_binary


def _add(a: Dict[str, str], b: Dict[str, str]) -> Dict[str, str]:
    out = dict(a)
    for k, v in (b or {}).items():
        out[k] = format_quantity(parse_quantity(out[k]) + parse_quantity(v), _is_binary(k)) if k in out else v
    return out


def _max(a: Dict[str, str], b: Dict[str, str]) -> Dict[str, str]:
    out = dict(a)
    for k, v in (b or {}).items():
        if k not in out or parse_quantity(v) > parse_quantity(out[k]):
            out[k] = v
    return out


def sum_up_containers_resources(containers: Iterable[dict]) -> dict:
    """Per-resource sum of requests and of limits over the containers."""
    req: Dict[str, str] = {}
    lim: Dict[str, str] = {}
    for ct in containers or []:
        r = ct.get("resources") or {}
        req = _add(req, r.get("requests") or {})
        lim = _add(lim, r.get("limits") or {})
    return {"requests": req, "limits": lim}


def maximum_containers_resources(containers: Iterable[dict]) -> dict:
    """Per-resource maximum of requests and of limits over the containers."""
    req: Dict[str, str] = {}
    lim: Dict[str, str] = {}
    for ct in containers or []:
        r = ct.get("resources") or {}
        req = _max(req, r.get("requests") or {})
        lim = _max(lim, r.get("limits") or {})
    return {"requests": req, "limits": lim}
