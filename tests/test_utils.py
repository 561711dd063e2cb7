"""kubedl_amd.utils: the reference's pkg/util helpers (loggers, k8sutil, quota,
tenancy, misc, signals).  CPU only."""
import json
import logging
import signal

import pytest

from kubedl_amd.api import common as c
from kubedl_amd.utils import k8sutil, misc, quota, tenancy
from kubedl_amd.utils import log as klog


def _pod(name, phase="Running", deleting=False, rtype="worker", owner_kind="PyTorchJob"):
    md = {"name": name, "namespace": "ns", "uid": "u-" + name, "labels": {c.REPLICA_TYPE_LABEL: rtype},
          "ownerReferences": [{"kind": owner_kind, "name": "job1", "uid": "j-1", "controller": True}]}
    if deleting:
        md["deletionTimestamp"] = c.now()
    return {"metadata": md, "status": {"phase": phase}}


def test_k8sutil_filters_and_totals():
    pods = [_pod("a"), _pod("b", "Succeeded"), _pod("c", "Failed"), _pod("d", deleting=True), _pod("e", "Pending")]
    assert [p["metadata"]["name"] for p in k8sutil.filter_active_pods(pods)] == ["a", "e"]
    assert [k8sutil.is_pod_active(p) for p in pods] == [True, False, False, False, True]
    assert k8sutil.filter_pod_count(pods, "Running") == 2
    specs = {"Master": {"replicas": 1}, "Worker": {"replicas": 3}}
    assert k8sutil.get_total_replicas(specs) == 4
    st = {"Master": {"active": 1}, "Worker": {"active": 2, "failed": 1}}
    assert k8sutil.get_total_active_replicas(st) == 3
    assert k8sutil.get_total_failed_replicas(st) == 1
    assert k8sutil.resolve_dependent_owner(pods[0]) == ("j-1", "job1")
    assert k8sutil.resolve_dependent_owner({"metadata": {}}) == ("", "")
    assert k8sutil.get_replica_type(pods[0]) == "worker"
    assert len(k8sutil.pods_by_replica_type(pods + [_pod("m", rtype="master")], "Master")) == 1


def test_loggers_carry_reference_fields(caplog):
    job = {"kind": "TFJob", "metadata": {"namespace": "kubedl", "name": "mnist", "uid": "123"}}
    with caplog.at_level(logging.INFO, logger="kubedl"):
        klog.logger_for_job(job).info("reconcile")
        klog.logger_for_replica(job, "ps").info("replica")
        klog.logger_for_pod(_pod("p0", owner_kind="TFJob"), "TFJob").info("pod")
        klog.logger_for_pod(_pod("p1", owner_kind="TFJob"), "PyTorchJob").info("other kind")
        klog.logger_for_key("kubedl/mnist").info("key")
        klog.logger_for_unstructured(job, "TFJob").info("unstructured")
    recs = caplog.records
    assert recs[0].kdl_fields == {"job": "kubedl.mnist", "uid": "123"}
    assert recs[1].kdl_fields["replica-type"] == "ps"
    assert recs[2].kdl_fields == {"job": "ns.job1", "pod": "ns.p0", "uid": "u-p0"}
    assert recs[3].kdl_fields["job"] == ""
    assert recs[4].kdl_fields == {"job": "kubedl.mnist"}
    assert recs[5].kdl_fields["job"] == "kubedl.mnist"
    assert "job=kubedl.mnist" in recs[0].getMessage()


def test_quota_sum_and_max():
    cts = [{"resources": {"requests": {"cpu": "500m", "memory": "1Gi"}, "limits": {"cpu": "1"}}},
           {"resources": {"requests": {"cpu": "1500m", "memory": "512Mi", "amd.com/gpu": "1"},
                          "limits": {"cpu": "2", "memory": "2Gi"}}},
           {}]
    s = quota.sum_up_containers_resources(cts)
    assert s["requests"] == {"cpu": "2", "memory": "1536Mi", "amd.com/gpu": "1"}
    assert s["limits"] == {"cpu": "3", "memory": "2Gi"}
    m = quota.maximum_containers_resources(cts)
    assert m["requests"] == {"cpu": "1500m", "memory": "1Gi", "amd.com/gpu": "1"}
    assert m["limits"] == {"cpu": "2", "memory": "2Gi"}


def test_tenancy_roundtrip_and_errors():
    obj = {"metadata": {}}
    assert tenancy.get_tenancy(obj) is None
    tenancy.set_tenancy(obj, tenancy.Tenancy(tenant="t1", user="alice", region="cn-hz"))
    raw = json.loads(obj["metadata"]["annotations"][c.ANNOTATION_TENANCY_INFO])
    assert raw == {"tenant": "t1", "user": "alice", "region": "cn-hz"}  # idc omitted (omitempty)
    t = tenancy.get_tenancy(obj)
    assert (t.tenant, t.user, t.idc, t.region) == ("t1", "alice", "", "cn-hz")
    obj["metadata"]["annotations"][c.ANNOTATION_TENANCY_INFO] = "{not json"
    with pytest.raises(ValueError):
        tenancy.get_tenancy(obj)


def test_misc_helpers(monkeypatch):
    assert misc.pformat("x") == "x"
    assert json.loads(misc.pformat({"a": [1, 2]})) == {"a": [1, 2]}
    assert misc.pformat({1, 2}).startswith("{")  # not JSON-able -> repr
    s = misc.rand_string(12)
    assert len(s) == 12 and set(s) <= set("0123456789abcdefghijklmnopqrstuvwxyz")
    monkeypatch.setenv(misc.ENV_KUBEFLOW_NAMESPACE, "team-a")
    assert misc.kubeflow_namespace() == "team-a"


def test_signal_handler_sets_event(monkeypatch):
    from kubedl_amd.utils import signals
    monkeypatch.setattr(signals, "_installed", False)
    old = {s: signal.getsignal(s) for s in (signal.SIGINT, signal.SIGTERM)}
    try:
        stop = signals.setup_signal_handler()
        assert not stop.is_set()
        signal.getsignal(signal.SIGTERM)(signal.SIGTERM, None)
        assert stop.is_set()
        with pytest.raises(RuntimeError):
            signals.setup_signal_handler()
    finally:
        for s, h in old.items():
            signal.signal(s, h)
