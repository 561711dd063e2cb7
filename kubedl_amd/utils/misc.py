"""``pkg/util/util.go`` + ``pointer.go`` equivalents."""
from __future__ import annotations

import json
import os
import secrets

ENV_KUBEFLOW_NAMESPACE = "KUBEFLOW_NAMESPACE"
_LETTERS = "0123456789abcdefghijklmnopqrstuvwxyz"


def pformat(value) -> str:
    """Strings as-is, everything else as indented JSON (``repr`` if not JSON-able)."""
    if isinstance(value, str):
        return value
    try:
        return json.dumps(value, indent=2, sort_keys=True)
    except (TypeError, ValueError):
        return repr(value)


def rand_string(n: int) -> str:
    """n characters of [0-9a-z] (pod-name suffixes, test fixtures)."""
    return "".join(secrets.choice(_LETTERS) for _ in range(n))


def kubeflow_namespace(default: str = "kubedl") -> str:
    return os.environ.get(ENV_KUBEFLOW_NAMESPACE) or default
