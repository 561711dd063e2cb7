"""The ``kubedl.io/tenancy`` annotation: ``{"tenant", "user", "idc", "region"}``.

Reference: ``pkg/util/tenancy/tenancy.go:25-43``.  ``get_tenancy`` returns None
when the annotation is absent and raises ``ValueError`` on malformed JSON (the
reference returns the json error).
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass
from typing import Optional

from kubedl_amd.api import common as c


@dataclass
class Tenancy:
    tenant: str = ""
    user: str = ""
    idc: str = ""
    region: str = ""

    def to_json(self) -> str:
        d = asdict(self)
        for k in ("idc", "region"):  # omitempty
            if not d[k]:
                d.pop(k)
        return json.dumps(d, sort_keys=True)


def get_tenancy(obj: dict) -> Optional[Tenancy]:
    raw = ((obj.get("metadata") or {}).get("annotations") or {}).get(c.ANNOTATION_TENANCY_INFO)
    if raw is None:
        return None
    try:
        d = json.loads(raw)
    except json.JSONDecodeError as e:
        raise ValueError(f"malformed {c.ANNOTATION_TENANCY_INFO} annotation: {e}") from e
    return Tenancy(tenant=d.get("tenant", ""), user=d.get("user", ""), idc=d.get("idc", ""),
                   region=d.get("region", ""))


def set_tenancy(obj: dict, t: Tenancy) -> None:
    md = obj.setdefault("metadata", {})
    md.setdefault("annotations", {})[c.ANNOTATION_TENANCY_INFO] = t.to_json()
