"""CustomResourceDefinition manifests for the four job kinds.

The reference generates ``config/crd/bases/*.yaml`` with controller-gen from
its Go types (``Makefile:40-47``).  Here they are generated from
``kubedl_amd.api.kinds`` so the schema the local runtime validates against and
the one published for a Kubernetes install never drift:

* ``apiextensions.k8s.io/v1`` CRD, namespaced, ``status`` subresource;
* printer columns State / Age / Finished-TTL / Max-Lifetime exactly as the
  kubebuilder markers (``api/tensorflow/v1/types.go:28-31``);
* spec schema: the replica-spec map restricted to the kind's replica types,
  ``replicas``/``restartPolicy``/``template`` per replica, the inlined
  ``RunPolicy`` fields, plus ``minFinishWorkNum``/``minFinishWorkRate`` for
  XDLJob; the pod template is ``x-kubernetes-preserve-unknown-fields``;
* status schema: ``conditions`` and ``replicaStatuses`` required
  (``kubeflow.org_pytorchjobs.yaml:149-151``).

``python -m kubedl_amd.api.crd [outdir]`` writes one YAML file per kind
(``config/crd/bases`` by default, as ``make manifests`` does).
"""
from __future__ import annotations

import os
import sys
from typing import Dict

import yaml

from kubedl_amd.api import kinds as K

RESTART_POLICIES = ["Always", "OnFailure", "Never", "ExitCode"]
CLEAN_POD_POLICIES = ["", "All", "Running", "None"]
CONDITION_TYPES = ["Created", "Running", "Restarting", "Succeeded", "Failed"]


def _replica_spec_schema() -> dict:
    return {"type": "object", "properties": {
        "replicas": {"type": "integer", "format": "int32"},
        "restartPolicy": {"type": "string", "enum": RESTART_POLICIES},
        "template": {"type": "object", "x-kubernetes-preserve-unknown-fields": True}}}


def _run_policy_props() -> Dict[str, dict]:
    return {"cleanPodPolicy": {"type": "string", "enum": CLEAN_POD_POLICIES},
            "ttlSecondsAfterFinished": {"type": "integer", "format": "int32"},
            "activeDeadlineSeconds": {"type": "integer", "format": "int64"},
            "backoffLimit": {"type": "integer", "format": "int32"},
            "schedulingPolicy": {"type": "object", "properties": {
                "minAvailable": {"type": "integer", "format": "int32"}}}}


def _status_schema() -> dict:
    cond = {"type": "object", "required": ["type", "status"], "properties": {
        "type": {"type": "string", "enum": CONDITION_TYPES}, "status": {"type": "string"},
        "reason": {"type": "string"}, "message": {"type": "string"},
        "lastUpdateTime": {"type": "string", "format": "date-time"},
        "lastTransitionTime": {"type": "string", "format": "date-time"}}}
    rs = {"type": "object", "properties": {k: {"type": "integer", "format": "int32"}
                                           for k in ("active", "succeeded", "failed")}}
    return {"type": "object", "required": ["conditions", "replicaStatuses"], "properties": {
        "conditions": {"type": "array", "items": cond},
        "replicaStatuses": {"type": "object", "additionalProperties": rs},
        "startTime": {"type": "string", "format": "date-time"},
        "completionTime": {"type": "string", "format": "date-time"},
        "lastReconcileTime": {"type": "string", "format": "date-time"}}}


def crd_for(info: K.KindInfo) -> dict:
    spec_props = dict(_run_policy_props())
    spec_props[info.spec_field] = {"type": "object",
                                   "properties": {rt: _replica_spec_schema() for rt in info.replica_types}}
    if info.kind == "XDLJob":
        spec_props["minFinishWorkNum"] = {"type": "integer", "format": "int32"}
        spec_props["minFinishWorkRate"] = {"type": "integer", "format": "int32"}
    columns = [{"name": "State", "type": "string", "JSONPath": ".status.conditions[-1:].type"},
               {"name": "Age", "type": "date", "JSONPath": ".metadata.creationTimestamp"},
               {"name": "Finished-TTL", "type": "integer", "JSONPath": ".spec.ttlSecondsAfterFinished"},
               {"name": "Max-Lifetime", "type": "integer", "JSONPath": ".spec.activeDeadlineSeconds"}]
    return {"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
            "metadata": {"name": info.crd_name},
            "spec": {"group": info.group, "scope": "Namespaced",
                     "names": {"kind": info.kind, "listKind": info.kind + "List", "plural": info.plural,
                               "singular": info.singular},
                     "versions": [{"name": info.version, "served": True, "storage": True,
                                   "subresources": {"status": {}},
                                   "additionalPrinterColumns": [
                                       {"name": col["name"], "type": col["type"], "jsonPath": col["JSONPath"]}
                                       for col in columns],
                                   "schema": {"openAPIV3Schema": {"type": "object", "properties": {
                                       "apiVersion": {"type": "string"}, "kind": {"type": "string"},
                                       "metadata": {"type": "object"},
                                       "spec": {"type": "object", "properties": spec_props},
                                       "status": _status_schema()}}}}]}}


def write_all(outdir: str) -> list:
    os.makedirs(outdir, exist_ok=True)
    paths = []
    for info in K.ALL_KINDS:
        p = os.path.join(outdir, f"{info.group}_{info.plural}.yaml")
        with open(p, "w") as f:
            f.write("\n---\n")
            yaml.safe_dump(crd_for(info), f, sort_keys=False)
        paths.append(p)
    return paths


if __name__ == "__main__":
    for p in write_all(sys.argv[1] if len(sys.argv) > 1 else "config/crd/bases"):
        print(p)
