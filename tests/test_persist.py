"""Persistence: DMO converters (``pkg/storage/dmo/converters/*_test.go``
behaviours), sqlite/jsonl backends and the persist controller end to end."""
import json
import os
import sys
import time

import pytest

from kubedl_amd.persist import dmo
from kubedl_amd.persist.backends import (JSONLEventBackend, Query, SQLiteEventBackend,
                                         SQLiteObjectBackend)


def _job(status_types=(), tenancy=None, completion=None):
    md = {"name": "j1", "namespace": "ns", "uid": "uid-1", "resourceVersion": "7",
          "creationTimestamp": "2026-01-01T00:00:00.000000Z"}
    if tenancy:
        md["annotations"] = {"kubedl.io/tenancy": json.dumps(tenancy)}
    st = {"conditions": [{"type": t, "status": "True"} for t in status_types]}
    if completion:
        st["completionTime"] = completion
    tmpl = {"spec": {"initContainers": [{"name": "init", "resources": {"limits": {"cpu": "4", "memory": "1Gi"}}}],
                     "containers": [
                         {"name": "tensorflow", "image": "img:1",
                          "resources": {"limits": {"cpu": "1", "memory": "512Mi", "amd.com/gpu": "1"},
                                        "requests": {"cpu": "500m"}}},
                         {"name": "side", "resources": {"limits": {"cpu": "2", "memory": "1Gi"}}}]}}
    return {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": md,
            "spec": {"tfReplicaSpecs": {"Worker": {"replicas": 2, "template": tmpl}}}, "status": st}


def test_quantities():
    assert dmo.parse_quantity("500m") * 2 == 1
    assert dmo.parse_quantity("1Gi") == 2 ** 30
    assert dmo.format_quantity(dmo.parse_quantity("1536Mi"), binary=True) == "1536Mi"
    assert dmo.format_quantity(dmo.parse_quantity("1500m")) == "1500m"
    assert dmo.format_quantity(dmo.parse_quantity("2")) == "2"


def test_compute_pod_resources_max_of_init_and_sum():
    res = dmo.compute_pod_resources(_job()["spec"]["tfReplicaSpecs"]["Worker"]["template"]["spec"])
    # limits: sum(containers) = cpu 3, memory 1.5Gi, gpu 1; init max = cpu 4, memory 1Gi -> max
    assert res["limits"] == {"amd.com/gpu": "1", "cpu": "4", "memory": "1536Mi"}
    assert res["requests"] == {"cpu": "500m"}


def test_job_to_dmo():
    row = dmo.job_to_dmo(_job(), region="r1")
    assert row["status"] == "Created" and row["job_id"] == "uid-1" and row["kind"] == "TFJob"
    assert row["deploy_region"] == "r1" and row["tenant"] == "" and row["owner"] == ""
    assert row["deleted"] == 0 and row["is_in_etcd"] == 1 and row["gmt_finished"] is None
    res = json.loads(row["resources"])
    assert res["Worker"]["replicas"] == 2 and res["Worker"]["resources"]["limits"]["cpu"] == "4"
    row = dmo.job_to_dmo(_job(("Created", "Running", "Failed"), {"tenant": "t", "user": "u", "region": "rg"},
                              completion="2026-01-02T00:00:00.000000Z"))
    assert row["status"] == "Failed" and row["tenant"] == "t" and row["owner"] == "u"
    assert row["deploy_region"] == "rg" and row["gmt_finished"] == "2026-01-02T00:00:00.000000Z"


def _pod(phase, term=None, owner_kind="TFJob"):
    st = {"phase": phase, "podIP": "127.0.0.1", "hostIP": "127.0.0.1",
          "containerStatuses": [{"name": "side", "state": {"running": {"startedAt": "S0"}}},
                                {"name": "tensorflow", "state": term or {"running": {"startedAt": "S1"}}}]}
    return {"kind": "Pod", "metadata": {"name": "j1-worker-0", "namespace": "ns", "uid": "p1", "resourceVersion": "3",
                                        "creationTimestamp": "C0",
                                        "labels": {"group-name": "kubeflow.org", "replica-type": "worker"},
                                        "ownerReferences": [{"kind": owner_kind, "uid": "uid-1", "controller": True}]},
            "spec": {"containers": [{"name": "side", "image": "side:1"}, {"name": "tensorflow", "image": "tf:1"}]},
            "status": st}


def test_pod_to_dmo():
    row = dmo.pod_to_dmo(_pod("Running"), "tensorflow")
    assert row["image"] == "tf:1" and row["status"] == "Running" and row["gmt_started"] == "S1"
    assert row["job_id"] == "uid-1" and row["replica_type"] == "worker" and row["pod_ip"] == "127.0.0.1"
    row = dmo.pod_to_dmo(_pod("Failed", {"terminated": {"exitCode": 137, "reason": "OOMKilled", "startedAt": "S",
                                                        "finishedAt": "F", "message": "m"}}), "tensorflow")
    assert row["remark"] == "Reason: OOMKilled\nExitCode: 137\nMessage: m"
    assert row["gmt_started"] == "S" and row["gmt_finished"] == "F"
    # any controller reference is the dependent owner (k8sutil.ResolveDependentOwner);
    # the persist controller only feeds pods owned by a job kind
    assert dmo.pod_to_dmo(_pod("Running", owner_kind="ReplicaSet"), "tensorflow")["job_id"] == "uid-1"
    p = _pod("Running")
    p["metadata"]["ownerReferences"] = []
    with pytest.raises(dmo.ConvertError):
        dmo.pod_to_dmo(p, "tensorflow")


def test_sqlite_object_backend(tmp_path):
    b = SQLiteObjectBackend(str(tmp_path / "p.db"))
    b.initialize()
    b.save_job(_job(("Created",)), "")
    b.save_job(_job(("Created", "Running")), "")
    old = _job(("Created",))
    old["metadata"]["resourceVersion"] = "3"  # older version must not overwrite
    b.save_job(old, "")
    row = b.get_job("ns", "j1", "uid-1")
    assert row["status"] == "Running"
    assert len(b.list_jobs(Query(namespace="ns"))) == 1
    assert b.list_jobs(Query(status="Failed")) == []
    b.save_pod(_pod("Running"), "tensorflow", "")
    assert [p["name"] for p in b.list_pods("uid-1")] == ["j1-worker-0"]
    b.stop_pod("ns", "j1-worker-0", "p1")
    p = b.list_pods("uid-1")[0]
    assert p["status"] == "Stopped" and p["is_in_etcd"] == 0
    b.stop_job("ns", "j1", "uid-1")
    b.delete_job("ns", "j1", "uid-1")
    row = b.get_job("ns", "j1", "uid-1")
    assert row["status"] == "Stopped" and row["deleted"] == 1 and row["is_in_etcd"] == 0
    b.close()


@pytest.mark.parametrize("cls", [JSONLEventBackend, SQLiteEventBackend])
def test_event_backends(tmp_path, cls):
    b = cls(str(tmp_path / ("e.jsonl" if cls is JSONLEventBackend else "e.db")))
    b.initialize()
    ev = {"metadata": {"name": "e1"}, "involvedObject": {"kind": "TFJob", "namespace": "ns", "name": "j1", "uid": "u"},
          "reason": "SuccessfulCreatePod", "message": "Created pod: j1-worker-0", "type": "Normal", "count": 1,
          "firstTimestamp": "2026-01-01T00:00:01Z", "lastTimestamp": "2026-01-01T00:00:01Z"}
    b.save_event(ev, "r")
    ev2 = dict(ev, count=3, lastTimestamp="2026-01-01T00:00:09Z")
    b.save_event(ev2, "r")
    other = dict(ev, metadata={"name": "e2"}, involvedObject={"kind": "TFJob", "namespace": "ns", "name": "zz", "uid": "x"})
    b.save_event(other, "r")
    out = b.list_events("ns", "j1")
    assert len(out) == 1 and out[0]["count"] == 3 and out[0]["obj_uid"] == "u" and out[0]["region"] == "r"
    b.close()


def test_persist_controller_end_to_end(tmp_path):
    from kubedl_amd.engine.manager import Manager, ManagerOptions
    m = Manager(ManagerOptions(home=str(tmp_path), gpus=0, object_storage="sqlite", event_storage="jsonl")).start()
    try:
        job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {
            "name": "pj", "namespace": "default", "annotations": {"kubedl.io/tenancy": '{"tenant":"t1","user":"alice"}'}},
            "spec": {"pytorchReplicaSpecs": {"Master": {"template": {"spec": {"containers": [
                {"name": "pytorch", "image": "x", "command": [sys.executable, "-c", "pass"]}]}}}}}}
        uid = m.apply(job)["metadata"]["uid"]
        m.wait_for_condition("PyTorchJob", "default", "pj", ["Succeeded"], timeout=30)
        time.sleep(0.2)
        m.persist.flush()
        row = m.persist.objects.get_job("default", "pj", uid)
        assert row["status"] == "Succeeded" and row["tenant"] == "t1" and row["owner"] == "alice"
        pods = m.persist.objects.list_pods(uid)
        assert len(pods) == 1 and pods[0]["status"] == "Succeeded"
        evs = m.persist.events.list_events("default", "pj")
        assert any(e["reason"] == "JobSucceeded" for e in evs)
        m.delete("PyTorchJob", "default", "pj")
        time.sleep(0.2)
        m.persist.flush()
        row = m.persist.objects.get_job("default", "pj", uid)
        assert row["deleted"] == 1 and row["is_in_etcd"] == 0
    finally:
        m.stop()
