"""JSON/YAML codec for job manifests (``kubectl apply -f`` input format).

Objects stay JSON-shaped dicts, so field names (``tfReplicaSpecs``,
``cleanPodPolicy``, ``replicaStatuses`` ...) and ``omitempty`` behaviour are
whatever the manifest/status carries -- nothing is renamed on the way in or
out.  YAML is read with ``yaml.safe_load_all`` only.
"""
from __future__ import annotations

import io
import json
from typing import Any, Dict, Iterable, List

import yaml


def loads(text: str) -> List[Dict[str, Any]]:
    """Parse one or more manifests (YAML multi-doc or JSON / JSON list / v1 List)."""
    text = text.strip()
    docs: List[Any]
    if text.startswith("{") or text.startswith("["):
        try:
            obj = json.loads(text)
            docs = obj if isinstance(obj, list) else [obj]
        except json.JSONDecodeError:
            docs = list(yaml.safe_load_all(io.StringIO(text)))
    else:
        docs = list(yaml.safe_load_all(io.StringIO(text)))
    out: List[Dict[str, Any]] = []
    for d in docs:
        if not d:
            continue
        if isinstance(d, dict) and d.get("kind") == "List" and isinstance(d.get("items"), list):
            out.extend(x for x in d["items"] if x)
        elif isinstance(d, dict):
            out.append(d)
        else:
            raise ValueError(f"manifest document is not an object: {type(d).__name__}")
    return out


def load_file(path: str) -> List[Dict[str, Any]]:
    with open(path) as f:
        return loads(f.read())


def dumps_json(obj: Any, indent: int | None = 2) -> str:
    return json.dumps(obj, indent=indent, sort_keys=False)


def dumps_yaml(obj: Any) -> str:
    return yaml.safe_dump(obj, sort_keys=False, default_flow_style=False)


def dumps(objs: Iterable[Dict[str, Any]], fmt: str = "yaml") -> str:
    objs = list(objs)
    if fmt == "json":
        if len(objs) == 1:
            return dumps_json(objs[0])
        return dumps_json({"apiVersion": "v1", "kind": "List", "items": objs})
    return "---\n".join(dumps_yaml(o) for o in objs)
