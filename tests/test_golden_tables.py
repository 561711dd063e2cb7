"""The reference's table-driven unit tests, one pytest case per table row.

Each table below restates the inputs and expected outputs of a reference Go
test (cited per table) as data and runs them against this framework's
equivalent function; comparison is whole-object equality wherever the
reference uses ``reflect.DeepEqual``.

* ``api/tensorflow/v1/defaults_test.go:78-271``  -> ``kinds._default_tfjob``
* ``api/xdl/v1alpha1/defaults_test.go:91-511``    -> ``kinds._default_xdljob``
* ``pkg/storage/dmo/converters/pod_test.go``      -> ``dmo.pod_to_dmo``
* ``pkg/storage/dmo/converters/job_test.go``      -> ``dmo.job_to_dmo``
* ``pkg/storage/dmo/converters/event_test.go``    -> ``dmo.event_to_dmo``
* ``pkg/job_controller/job_test.go:15-237``       -> ``JobController`` limits/cleanup
* ``pkg/job_controller/service_ref_manager_test.go:33-200`` -> ``ControllerRefManager.claim``
* ``controllers/xgboost/pod_test.go:69-137``      -> ``XGBoostController.set_cluster_spec``

Deliberate differences from the Go structs: times are RFC3339 strings (the
store's representation); absent Go pointers are ``None``; event rows also carry
``obj_namespace/obj_name/obj_uid`` (documented fix in ``persist/dmo.py``), so the
event table compares the reference's columns only.
"""
import copy
import datetime

import pytest

from kubedl_amd.api import common as c
from kubedl_amd.api import kinds as K
from kubedl_amd.engine.control import ControllerRefManager, ServiceControl
from kubedl_amd.engine.job_controller import gen_owner_reference
from kubedl_amd.engine.testing import new_job_controller, new_test_job
from kubedl_amd.persist import dmo
from kubedl_amd.store import EventRecorder, Store

TEST_IMAGE = "test-image:latest"


def _ports(port_name, port, default_name, default_port):
    """``expectedTFJob`` / ``expectedXDLJob``: the given port (if named) then
    the default port unless the given one already is the default."""
    ports = []
    if port_name:
        ports.append({"name": port_name, "containerPort": port})
    if port_name != default_name:
        ports.append({"name": default_name, "containerPort": default_port})
    return ports


def _replica(container, restart=None, replicas=None, ports=None):
    ctr = {"name": container, "image": TEST_IMAGE}
    if ports is not None:
        ctr["ports"] = ports
    rs = {"template": {"spec": {"containers": [ctr]}}}
    if restart is not None:
        rs["restartPolicy"] = restart
    if replicas is not None:
        rs["replicas"] = replicas
    return rs


# =================================================================== TFJob defaults
TF_DEFAULT = [{"name": "tfjob-port", "containerPort": 2222}]
TF_CUSTOM = [{"name": "customPort", "containerPort": 1234}]

TF_CASES = {
    # name: (spec extras, worker replica spec, expected (cleanPodPolicy, restart, portName, port))
    "set replicas": ({}, _replica("tensorflow", "Always", None, TF_DEFAULT),
                     ("Running", "Always", "tfjob-port", 2222)),
    "set replicas with default restartpolicy": ({}, _replica("tensorflow", None, None, TF_DEFAULT),
                                                ("Running", "ExitCode", "tfjob-port", 2222)),
    "set replicas with default port": ({}, _replica("tensorflow", "Always", 1, None),
                                       ("Running", "Always", "", 0)),
    "set replicas adding default port": ({}, _replica("tensorflow", "Always", 1, TF_CUSTOM),
                                         ("Running", "Always", "customPort", 1234)),
    "set custom cleanpod policy": ({"cleanPodPolicy": "All"}, _replica("tensorflow", "Always", 1, TF_CUSTOM),
                                   ("All", "Always", "customPort", 1234)),
}


@pytest.mark.parametrize("name", list(TF_CASES))
def test_tf_set_defaults_table(name):
    extra, worker, (cpp, restart, pname, port) = TF_CASES[name]
    job = {"kind": "TFJob", "spec": dict(copy.deepcopy(extra), tfReplicaSpecs={"Worker": copy.deepcopy(worker)})}
    K.TFJOB.defaulter(job)
    want = {"cleanPodPolicy": cpp, "tfReplicaSpecs": {
        "Worker": _replica("tensorflow", restart, 1, _ports(pname, port, "tfjob-port", 2222))}}
    assert job["spec"] == want


def test_tf_set_type_names():
    job = {"kind": "TFJob", "spec": {"tfReplicaSpecs": {"WORKER": _replica("tensorflow", "Always", None, TF_DEFAULT)}}}
    K.TFJOB.defaulter(job)
    assert "WORKER" not in job["spec"]["tfReplicaSpecs"] and "Worker" in job["spec"]["tfReplicaSpecs"]


# =================================================================== XDLJob defaults
XDL_DEFAULT = [{"name": "xdljob-port", "containerPort": 2222}]
XDL_CUSTOM = [{"name": "customPort", "containerPort": 1234}]
R, N = "Running", "Never"

XDL_CASES = {
    # name: (spec extras, worker spec, (cleanPodPolicy, restart, portName, port, minNum, minRate, backoff))
    "set replicas": ({}, _replica("xdl", "Always", None, XDL_DEFAULT),
                     (R, "Always", "xdljob-port", 2222, None, 90, 20)),
    "set replicas with default restart policy": ({}, _replica("xdl", None, None, XDL_DEFAULT),
                                                 (R, N, "xdljob-port", 2222, None, 90, 20)),
    "set replicas with default port": ({}, _replica("xdl", "Always", 1, None),
                                       (R, "Always", "", 0, None, 90, 20)),
    "set replicas adding default port": ({}, _replica("xdl", "Always", 1, XDL_CUSTOM),
                                         (R, "Always", "customPort", 1234, None, 90, 20)),
    "set custom clean pod policy": ({"cleanPodPolicy": "All"}, _replica("xdl", "Always", 1, XDL_CUSTOM),
                                    ("All", "Always", "customPort", 1234, None, 90, 20)),
    "set default min finish attributes": ({}, _replica("xdl", None, None, XDL_DEFAULT),
                                          (R, N, "xdljob-port", 2222, None, 90, 20)),
    "set add min finish work num": ({"minFinishWorkNum": 10}, _replica("xdl", None, None, XDL_DEFAULT),
                                    (R, N, "xdljob-port", 2222, 10, None, 20)),
    "set add min finish work percentage": ({"minFinishWorkRate": 100}, _replica("xdl", None, None, XDL_DEFAULT),
                                           (R, N, "xdljob-port", 2222, None, 100, 20)),
    "set add backoff limit": ({"backoffLimit": 100}, _replica("xdl", None, None, XDL_DEFAULT),
                              (R, N, "xdljob-port", 2222, None, 90, 100)),
    "set add bakcoff limit per type": ({}, _replica("xdl", None, None, XDL_DEFAULT),
                                       (R, N, "xdljob-port", 2222, None, 90, 20)),
}


@pytest.mark.parametrize("name", list(XDL_CASES))
def test_xdl_set_defaults_table(name):
    extra, worker, (cpp, restart, pname, port, min_num, min_rate, backoff) = XDL_CASES[name]
    job = {"kind": "XDLJob", "spec": dict(copy.deepcopy(extra), xdlReplicaSpecs={"Worker": copy.deepcopy(worker)})}
    K.XDLJOB.defaulter(job)
    want = {"cleanPodPolicy": cpp, "backoffLimit": backoff, "xdlReplicaSpecs": {
        "Worker": _replica("xdl", restart, 1, _ports(pname, port, "xdljob-port", 2222))}}
    if min_num is not None:
        want["minFinishWorkNum"] = min_num
    if min_rate is not None:
        want["minFinishWorkRate"] = min_rate
    assert job["spec"] == want


def test_xdl_set_type_names():
    job = {"kind": "XDLJob", "spec": {"backoffLimit": 20, "minFinishWorkNum": 1, "minFinishWorkRate": 90,
                                      "xdlReplicaSpecs": {"WORKER": _replica("xdl", "Always", None, XDL_DEFAULT)}}}
    K.XDLJOB.defaulter(job)
    assert "WORKER" not in job["spec"]["xdlReplicaSpecs"] and "Worker" in job["spec"]["xdlReplicaSpecs"]


# =================================================================== DMO pod converter
NS, REGION, MAIN = "kubedl-test", "test-region", "tensorflow"
IMG = "kubedl/tf-mnist-with-summaries:1.0"
POD_UID, JOB_UID = "6f06d2fd-22c6-11e9-96bb-0242ac1d5327", "7f06d2fd-22c6-11e9-96bb-0242ac1d5327"
T_CREATE, T_START, T_FINISH = "2019-02-10T12:27:00Z", "2019-02-10T12:28:00Z", "2019-02-11T12:28:00Z"
TENANCY = {c.ANNOTATION_TENANCY_INFO: '{"tenant":"foo","user":"bar","idc":"test-idc","region":"test-region"}'}


def _pod(annotations=None, owner=True, labels=True, phase=None, statuses=None, containers=None, full=True):
    md = {}
    if full:
        md.update(name="tfjob-0-test", namespace=NS, uid=POD_UID, resourceVersion="3", creationTimestamp=T_CREATE)
    if labels and full:
        md["labels"] = {c.REPLICA_TYPE_LABEL: "ps"}
    if annotations:
        md["annotations"] = dict(annotations)
    if owner:
        md["ownerReferences"] = [{"controller": True, "uid": JOB_UID}]
    pod = {"metadata": md, "spec": {"containers": containers or [{"name": MAIN, "image": IMG}]}, "status": {}}
    if phase:
        pod["status"].update(phase=phase, podIP="127.0.0.1", hostIP="192.168.1.1")
    if statuses is not None:
        pod["status"]["containerStatuses"] = statuses
    return pod


def _term(name=MAIN, **extra):
    return {"name": name, "state": {"terminated": dict(startedAt=T_START, finishedAt=T_FINISH, **extra)}}


def _row(region=REGION, status="Unknown", ips=False, started=None, finished=None, remark=None, resources="{}"):
    return {"name": "tfjob-0-test", "namespace": NS, "pod_id": POD_UID, "version": "3", "gmt_created": T_CREATE,
            "deploy_region": region, "job_id": JOB_UID, "replica_type": "ps", "resources": resources,
            "deleted": 0, "is_in_etcd": 1, "pod_ip": "127.0.0.1" if ips else None,
            "host_ip": "192.168.1.1" if ips else None, "image": IMG, "status": status,
            "gmt_started": started, "gmt_finished": finished, "remark": remark}


_REQ1 = {"resources": {"requests": {"cpu": "1", "memory": "1Gi"}}}
POD_CASES = {
    "owner reference error": (_pod(TENANCY, owner=False, full=False), REGION, None),
    "replica type error": (_pod(TENANCY, labels=False, full=False), REGION, None),
    "replica type in tf style": (_pod(), REGION, _row()),
    "success status Unknown": (_pod(TENANCY), REGION, _row()),
    "success status Pending": (_pod(TENANCY, phase="Pending", statuses=[{"name": "", "state": {}}]), REGION,
                               _row(status="Pending", ips=True)),
    "success status Running": (_pod(TENANCY, phase="Running",
                                    statuses=[{"name": "", "state": {"running": {"startedAt": T_START}}}]),
                               REGION, _row(status="Running", ips=True, started=T_START)),
    "success status Succeeded": (_pod(TENANCY, phase="Succeeded", statuses=[_term()]), REGION,
                                 _row(status="Succeeded", ips=True, started=T_START, finished=T_FINISH)),
    "success status Failed": (_pod(TENANCY, phase="Failed",
                                   statuses=[_term(exitCode=137, reason="Reason07", message="Message07")]),
                              REGION, _row(status="Failed", ips=True, started=T_START, finished=T_FINISH,
                                           remark="Reason: Reason07\nExitCode: 137\nMessage: Message07")),
    "success without region": (_pod(phase="Succeeded", statuses=[_term()]), "",
                               _row(region=None, status="Succeeded", ips=True, started=T_START, finished=T_FINISH)),
    "single container resource": (_pod(phase="Succeeded", statuses=[_term()],
                                       containers=[dict(name=MAIN, image=IMG, **_REQ1)]), "",
                                  _row(region=None, status="Succeeded", ips=True, started=T_START,
                                       finished=T_FINISH, resources='{"requests":{"cpu":"1","memory":"1Gi"}}')),
    "multiple container resources combination": (
        _pod(phase="Succeeded", statuses=[_term(), _term("sidecar")],
             containers=[dict(name=MAIN, image=IMG, **_REQ1), dict(name="sidecar", image=IMG, **_REQ1)]), "",
        _row(region=None, status="Succeeded", ips=True, started=T_START, finished=T_FINISH,
             resources='{"requests":{"cpu":"2","memory":"2Gi"}}')),
}


@pytest.mark.parametrize("name", list(POD_CASES))
def test_convert_pod_to_dmo_table(name):
    pod, region, want = POD_CASES[name]
    if want is None:
        with pytest.raises(dmo.ConvertError):
            dmo.pod_to_dmo(pod, MAIN, region)
        return
    assert dmo.pod_to_dmo(pod, MAIN, region) == want


def test_convert_pod_terminated_without_times_gets_now():
    """converters/pod.go:137-142: a finished pod with no terminated state gets
    started = creation and finished = now."""
    row = dmo.pod_to_dmo(_pod(phase="Succeeded", statuses=[{"name": MAIN, "state": {}}]), MAIN, "")
    assert row["gmt_started"] == T_CREATE and row["gmt_finished"] is not None


# =================================================================== DMO job converter
JOB_META = {"namespace": NS, "uid": POD_UID, "resourceVersion": "3", "creationTimestamp": "2019-02-10T12:27:00Z"}
DONE = {"completionTime": "2019-02-11T12:27:00Z", "conditions": [{"type": "Succeeded"}]}


def _ctr(name=None):
    ct = {"image": IMG, "resources": {"requests": {"cpu": "1", "memory": "1Gi"}}}
    if name:
        ct["name"] = name
    return ct


def _typed_job(kind, name, rtype, containers, status, replicas=None, annotations=None):
    rs = {"template": {"spec": {"containers": containers}}}
    if replicas is not None:
        rs["replicas"] = replicas
    md = dict(JOB_META, name=name)
    if annotations:
        md["annotations"] = annotations
    return {"kind": kind, "metadata": md, "spec": {K.BY_KIND[kind].spec_field: {rtype: rs}}, "status": status}


def _job_row(name, kind, status, region=None, tenant="", owner="", finished=None, resources=""):
    return {"name": name, "namespace": NS, "job_id": POD_UID, "version": "3", "kind": kind,
            "resources": resources, "gmt_created": "2019-02-10T12:27:00Z", "deploy_region": region,
            "tenant": tenant, "owner": owner, "deleted": 0, "is_in_etcd": 1, "gmt_finished": finished,
            "status": status}


_RES = '{"%s":{"resources":{"requests":{"cpu":"%s","memory":"%sGi"}},"replicas":%d}}'
JOB_CASES = {
    "tfjob with created status": (
        _typed_job("TFJob", "tfjob-test", "Worker", [_ctr()], {"startTime": "2019-02-11T12:27:00Z"}), REGION,
        _job_row("tfjob-test", "TFJob", "Created", region=REGION, resources=_RES % ("Worker", 1, 1, 0))),
    "tfjob with region": (
        _typed_job("TFJob", "tfjob-test", "Worker", [_ctr(MAIN), _ctr("sidecar")], DONE, 1, TENANCY), "",
        _job_row("tfjob-test", "TFJob", "Succeeded", region=REGION, tenant="foo", owner="bar",
                 finished="2019-02-11T12:27:00Z", resources=_RES % ("Worker", 2, 2, 1))),
    "xdljob with status succeed": (
        _typed_job("XDLJob", "xdljob-test", "Master", [_ctr(MAIN)], DONE, 1), "",
        _job_row("xdljob-test", "XDLJob", "Succeeded", finished="2019-02-11T12:27:00Z",
                 resources=_RES % ("Master", 1, 1, 1))),
    "pytorchjob with succeed status": (
        _typed_job("PyTorchJob", "pytorchjob-test", "Worker", [_ctr(MAIN)], DONE, 1), "",
        _job_row("pytorchjob-test", "PyTorchJob", "Succeeded", finished="2019-02-11T12:27:00Z",
                 resources=_RES % ("Worker", 1, 1, 1))),
    "xgboostjob with region": (
        _typed_job("XGBoostJob", "xgboostjob-test", "Worker", [_ctr(MAIN)], DONE, 1), "",
        _job_row("xgboostjob-test", "XGBoostJob", "Succeeded", finished="2019-02-11T12:27:00Z",
                 resources=_RES % ("Worker", 1, 1, 1))),
}


@pytest.mark.parametrize("name", list(JOB_CASES))
def test_convert_job_to_dmo_table(name):
    job, region, want = JOB_CASES[name]
    assert dmo.job_to_dmo(job, region) == want


# =================================================================== DMO event converter
def _event(typ, count=None):
    ev = {"metadata": {"name": "test-event", "namespace": NS},
          "involvedObject": {"name": "test-tfjob", "namespace": NS, "kind": "TFJob"},
          "reason": "reason for test event", "message": "message for test event",
          "firstTimestamp": T_CREATE, "lastTimestamp": T_CREATE, "type": typ}
    if count is not None:
        ev["count"] = count
    return ev


EVENT_CASES = {
    "normal event without region": (_event("Normal"), "", None, 0),
    "normal event with region": (_event("Normal"), REGION, REGION, 0),
    "warning event with region": (_event("Warning"), REGION, REGION, 0),
    "normal event with counts": (_event("Normal", 10), REGION, REGION, 10),
}


@pytest.mark.parametrize("name", list(EVENT_CASES))
def test_convert_event_to_dmo_table(name):
    ev, region, want_region, want_count = EVENT_CASES[name]
    row = dmo.event_to_dmo(ev, region)
    ref_cols = {k: row[k] for k in ("name", "kind", "type", "reason", "message", "region", "count",
                                    "first_timestamp", "last_timestamp")}
    assert ref_cols == {"name": "test-event", "kind": "TFJob", "type": ev["type"],
                        "reason": "reason for test event", "message": "message for test event",
                        "region": want_region, "count": want_count,
                        "first_timestamp": T_CREATE, "last_timestamp": T_CREATE}


# =================================================================== job_controller/job_test.go
def _phase_pod(name, phase):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
            "spec": {}, "status": {"phase": phase}}


@pytest.mark.parametrize("policy,del_running,del_succeeded", [
    ("Running", True, False),
    ("All", True, True),
    ("None", False, False),
])
def test_delete_pods_and_services_table(policy, del_running, del_succeeded):
    jc, pods, svcs = new_job_controller()
    for n in ("runningPod", "succeededPod"):
        jc.store.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": n, "namespace": "default"},
                         "spec": {}})
    all_pods = [_phase_pod("runningPod", "Running"), _phase_pod("succeededPod", "Succeeded")]
    jc.delete_pods_and_services({"cleanPodPolicy": policy}, new_test_job(), all_pods)
    assert ("runningPod" in pods.deleted) == del_running
    assert ("runningPod" in svcs.deleted) == del_running
    assert ("succeededPod" in pods.deleted) == del_succeeded
    assert ("succeededPod" in svcs.deleted) == del_succeeded


@pytest.mark.parametrize("backoff_limit,should_pass", [(0, False)])
def test_past_backoff_limit_table(backoff_limit, should_pass):
    jc, _, _ = new_job_controller()
    all_pods = [_phase_pod("runningPod", "Running"), _phase_pod("succeededPod", "Succeeded")]
    assert jc.past_backoff_limit("fake-job", {"backoffLimit": backoff_limit}, {}, all_pods) is should_pass


@pytest.mark.parametrize("deadline,should_pass", [(0, True), (2, False)])
def test_past_active_deadline_table(deadline, should_pass):
    jc, _, _ = new_job_controller()
    assert jc.past_active_deadline({"activeDeadlineSeconds": deadline}, {"startTime": c.now()}) is should_pass


@pytest.mark.parametrize("completion", ["one day ago", "now"])
def test_cleanup_job_ttl_zero_deletes_job(completion):
    """TestCleanupJobIfTTL / TestCleanupJob: ttl 0 after completion -> the job is deleted."""
    jc, _, _ = new_job_controller()
    job = jc.store.create(new_test_job())
    t = datetime.datetime.now(datetime.timezone.utc)
    if completion == "one day ago":
        t -= datetime.timedelta(days=1)
    else:
        t -= datetime.timedelta(seconds=1)  # RFC3339 keeps whole seconds
    status = {"completionTime": t.strftime("%Y-%m-%dT%H:%M:%SZ")}
    jc.cleanup_job({"ttlSecondsAfterFinished": 0}, status, job)
    assert jc.store.list(job["kind"]) == []


# =================================================================== service_ref_manager_test.go
def _ref_manager_case(name):
    store = Store()
    job = new_test_job(name="test-job")
    sel = {"group-name": "test.kubedl.io", "test-job-name": "test-job"}
    mine = gen_owner_reference(job)

    def svc(sname, owner_job=job, labels=None, deleting=False, owned=True):
        md = {"name": sname, "namespace": "default", "labels": dict(labels or sel),
              "ownerReferences": [gen_owner_reference(owner_job)] if owned else []}
        if deleting:
            md["deletionTimestamp"] = c.now()
        return store.create({"apiVersion": "v1", "kind": "Service", "metadata": md, "spec": {}})

    other = dict(sel, **{"group-name": "testing"})
    if name == "Claim services with correct label":
        objs, want = [svc("service1"), svc("service2", labels=other)], ["service1"]
    elif name == "Controller marked for deletion can not claim services":
        job["metadata"]["deletionTimestamp"] = c.now()
        objs, want = [svc("service1", owned=False), svc("service2", owned=False)], []
    elif name == "Controller marked for deletion can not claim new services":
        job["metadata"]["deletionTimestamp"] = c.now()
        objs, want = [svc("service1"), svc("service2", owned=False)], ["service1"]
    elif name == "Controller can not claim services owned by another controller":
        job2 = new_test_job(name="test-job")
        job2["metadata"]["uid"] = "AAAAA"
        objs, want = [svc("service1"), svc("service2", owner_job=job2)], ["service1"]
    elif name == "Controller releases claimed services when selector doesn't match":
        objs, want = [svc("service1"), svc("service2", labels=other)], ["service1"]
    else:  # "Controller does not claim orphaned services marked for deletion"
        objs, want = [svc("service1", deleting=True), svc("service2", labels=other, deleting=True)], ["service1"]
    mgr = ControllerRefManager(ServiceControl(store, EventRecorder(store)), job, sel, mine)
    return store, job, mgr, objs, want


REF_CASES = ["Claim services with correct label",
             "Controller marked for deletion can not claim services",
             "Controller marked for deletion can not claim new services",
             "Controller can not claim services owned by another controller",
             "Controller releases claimed services when selector doesn't match",
             "Controller does not claim orphaned services marked for deletion"]


@pytest.mark.parametrize("name", REF_CASES)
def test_claim_services_table(name):
    store, job, mgr, objs, want = _ref_manager_case(name)
    claimed = mgr.claim(objs)
    assert [o["metadata"]["name"] for o in claimed] == want
    if name == "Controller releases claimed services when selector doesn't match":
        refs = store.get("Service", "default", "service2")["metadata"]["ownerReferences"]
        assert all(r["uid"] != job["metadata"]["uid"] for r in refs)  # released
    if "marked for deletion" in name:  # nothing adopted
        for o in objs:
            if not o["metadata"]["ownerReferences"]:
                assert not store.get("Service", "default", o["metadata"]["name"])["metadata"]["ownerReferences"]


# =================================================================== controllers/xgboost/pod_test.go
def _xgb_job(workers):
    tmpl = {"spec": {"containers": [{"name": "xgboostjob", "image": "test-image-for-kubeflow-xgboost-operator:latest",
                                     "args": ["Fake", "Fake"],
                                     "ports": [{"name": "xgboostjob-port", "containerPort": 9999}]}]}}
    specs = {"Master": {"replicas": 1, "template": copy.deepcopy(tmpl)}}
    if workers > 0:
        specs["Worker"] = {"replicas": workers, "template": copy.deepcopy(tmpl)}
    return {"kind": "XGBoostJob", "metadata": {"name": "test-xgboostjob", "namespace": "default"},
            "spec": {"xgbReplicaSpecs": specs}}


XGB_CASES = [
    (0, "Master", "0", {"WORLD_SIZE": "1", "MASTER_PORT": "9999", "RANK": "0", "MASTER_ADDR": "test-xgboostjob-master-0"}),
    (1, "Master", "1", {"WORLD_SIZE": "2", "MASTER_PORT": "9999", "RANK": "1", "MASTER_ADDR": "test-xgboostjob-master-0"}),
    (2, "Master", "0", {"WORLD_SIZE": "3", "MASTER_PORT": "9999", "RANK": "0", "MASTER_ADDR": "test-xgboostjob-master-0"}),
    (2, "Worker", "1", {"WORLD_SIZE": "3", "MASTER_PORT": "9999", "RANK": "1", "MASTER_ADDR": "test-xgboostjob-master-0"}),
    (2, "Worker", "1", {"WORLD_SIZE": "3", "MASTER_PORT": "9999", "RANK": "1", "MASTER_ADDR": "test-xgboostjob-master-0"}),
]


@pytest.mark.parametrize("workers,rtype,index,want", XGB_CASES)
def test_xgboost_cluster_spec_table(workers, rtype, index, want):
    from kubedl_amd.controllers.xgboost import XGBoostJobReconciler as XGB
    job = _xgb_job(workers)
    tmpl = copy.deepcopy(job["spec"]["xgbReplicaSpecs"][rtype]["template"])
    XGB.set_cluster_spec(XGB.__new__(XGB), job, tmpl, rtype.lower(), index)
    env = {e["name"]: e["value"] for e in tmpl["spec"]["containers"][0]["env"]}
    assert {k: env[k] for k in want} == want


# =================================================================== job_controller/pod_test.go, status_test.go, util_test.go
@pytest.mark.parametrize("replica_policy,pod_policy", [
    ("ExitCode", "Never"), ("Never", "Never"), ("Always", "Always"), ("OnFailure", "OnFailure")])
def test_set_restart_policy_table(replica_policy, pod_policy):
    """TestSetRestartPolicy: ExitCode is implemented by the controller, so the pod gets Never."""
    jc, pods, _ = new_job_controller()
    job = new_test_job(workers=2, restart_policy=replica_policy)
    specs = job["spec"]["testReplicaSpecs"]
    jc.create_new_pod(job, "worker", "0", specs["Worker"], False, specs)
    assert pods.templates[-1]["spec"]["restartPolicy"] == pod_policy


def test_update_job_replica_statuses():
    """TestUpdateJobReplicaStatuses: 2 failed, 3 succeeded, 1 running -> counts per phase."""
    jc, _, _ = new_job_controller()
    job = new_test_job(workers=6, master=False)
    spec = job["spec"]["testReplicaSpecs"]["Worker"]
    phases = ["Failed"] * 2 + ["Succeeded"] * 3 + ["Running"]
    pods = [{"metadata": {"name": f"test-job-worker-{i}", "namespace": "default",
                          "labels": {c.REPLICA_TYPE_LABEL: "worker", c.REPLICA_INDEX_LABEL: str(i)}},
             "status": {"phase": ph}} for i, ph in enumerate(phases)]
    status = {"conditions": [], "replicaStatuses": {}}
    jc.reconcile_pods(job, status, pods, "Worker", spec, {"Worker": spec}, [False])
    assert status["replicaStatuses"]["Worker"] == {"failed": 2, "succeeded": 3, "active": 1}


def test_gen_general_name():
    """TestGenGeneralName: '/' in the job key becomes '-'."""
    assert c.gen_general_name("1/2/3/4/5", "worker", "1") == "1-2-3-4-5-worker-1"


# =================================================================== metrics/status_counter_test.go
@pytest.mark.parametrize("conds,running,pending", [(["Created"], 0, 1), (["Created", "Running"], 1, 0)])
def test_job_status_counter(conds, running, pending):
    """JobStatusCounter: pending = only the Created condition; running = last condition Running."""
    from kubedl_amd.metrics.job_metrics import MetricsRegistry
    reg = MetricsRegistry()
    reg.job_metrics("TFJob")
    status = {"conditions": [], "replicaStatuses": {}}
    for t in conds:
        c.update_job_conditions(status, t, "", "")
    reg.lister = lambda kind: [{"kind": "TFJob", "status": status}] if kind == "TFJob" else []
    got = {m.name: m.samples[0].value for m in reg.registry.collect() if m.name in ("kubedl_jobs_running",
                                                                                        "kubedl_jobs_pending")}
    assert got == {"kubedl_jobs_running": running, "kubedl_jobs_pending": pending}


# =================================================================== service_control_test.go, pod_control_test.go
@pytest.mark.parametrize("with_ref", [False, True], ids=["plain", "controllerRef"])
@pytest.mark.parametrize("kind", ["Service", "Pod"])
def test_object_control_create(kind, with_ref):
    """ServiceControl/PodControl create: the stored object keeps labels, name,
    namespace and spec (ports / containers); with a controller reference it is owned."""
    from kubedl_amd.engine.control import PodControl
    store = Store()
    job = new_test_job(name="test-job")
    labels = {"group-name": "test.kubedl.io", "test-job-name": "test-job"}
    md = {"name": f"{kind.lower()}-name", "namespace": "default", "labels": dict(labels), "ownerReferences": []}
    if with_ref:
        md["ownerReferences"] = [gen_owner_reference(job)]
    spec = ({"ports": [{"name": "test-port", "protocol": "TCP", "port": 8888, "targetPort": 8888}]}
            if kind == "Service" else {"containers": [{"name": "c", "image": "img"}]})
    ctl = (ServiceControl if kind == "Service" else PodControl)(store, EventRecorder(store))
    ctl.create(job, {"apiVersion": "v1", "kind": kind, "metadata": md, "spec": spec})
    got = store.get(kind, "default", f"{kind.lower()}-name")
    assert got["metadata"]["labels"] == labels and got["spec"] == spec
    refs = got["metadata"].get("ownerReferences") or []
    assert (refs == [gen_owner_reference(job)]) if with_ref else refs == []
    reasons = {e["reason"] for e in store.list("Event")}
    assert ("SuccessfulCreateService" if kind == "Service" else "SuccessfulCreatePod") in reasons
