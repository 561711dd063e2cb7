"""The object store (kubedl_amd/store): the API-server stand-in the engine,
controllers and CLI share.  CRUD per kind (the reference's controller suite:
create/get/delete of each CR), resourceVersion/generation, optimistic
concurrency, cascade delete through ownerReferences, watch events, sqlite
durability and the service host-port table."""
import threading

import pytest

from kubedl_amd.store import ADDED, DELETED, MODIFIED, AlreadyExists, EventRecorder, NotFound, Store
from kubedl_amd.store.store import Conflict

KINDS = [("kubeflow.org/v1", "TFJob"), ("kubeflow.org/v1", "PyTorchJob"),
         ("xgboostjob.kubeflow.org/v1alpha1", "XGBoostJob"), ("xdl.kubedl.io/v1alpha1", "XDLJob")]


def _obj(api, kind, name, ns="default", **extra):
    o = {"apiVersion": api, "kind": kind, "metadata": {"name": name, "namespace": ns}, "spec": {"x": 1}}
    o.update(extra)
    return o


@pytest.mark.parametrize("api,kind", KINDS)
def test_crud_per_kind(api, kind):
    s = Store()
    created = s.create(_obj(api, kind, "j1"))
    md = created["metadata"]
    assert md["uid"] and md["resourceVersion"] and md["generation"] == 1 and md["creationTimestamp"]
    with pytest.raises(AlreadyExists):
        s.create(_obj(api, kind, "j1"))
    got = s.get(kind, "default", "j1")
    assert got == created
    got["spec"]["x"] = 2
    upd = s.update(got)
    assert upd["metadata"]["generation"] == 2
    assert int(upd["metadata"]["resourceVersion"]) > int(md["resourceVersion"])
    st = s.update_status({**upd, "status": {"conditions": [{"type": "Created"}]}, "spec": {"x": 99}})
    assert st["spec"]["x"] == 2 and st["status"]["conditions"][0]["type"] == "Created"  # status-only write
    assert st["metadata"]["generation"] == 2
    assert [o["metadata"]["name"] for o in s.list(kind)] == ["j1"]
    s.delete(kind, "default", "j1")
    with pytest.raises(NotFound):
        s.get(kind, "default", "j1")
    assert s.try_get(kind, "default", "j1") is None


def test_optimistic_concurrency_and_noop_update():
    s = Store()
    a = s.create(_obj("v1", "Pod", "p"))
    b = s.update({**a, "spec": {"x": 5}}, check_rv=True)
    with pytest.raises(Conflict):
        s.update({**a, "spec": {"x": 6}}, check_rv=True)  # stale resourceVersion
    same = s.update(b)
    assert same["metadata"]["resourceVersion"] == b["metadata"]["resourceVersion"]  # no-op keeps rv


def test_cascade_delete_and_watch_events():
    s = Store()
    seen = []
    cancel = s.watch(lambda et, o: seen.append((et, o["kind"], o["metadata"]["name"])))
    job = s.create(_obj("kubeflow.org/v1", "PyTorchJob", "j"))
    ref = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "name": "j", "uid": job["metadata"]["uid"],
           "controller": True}
    pod = s.create({"kind": "Pod", "metadata": {"name": "j-master-0", "namespace": "default",
                                                 "ownerReferences": [ref]}})
    s.create({"kind": "Service", "metadata": {"name": "j-master-0", "namespace": "default", "ownerReferences": [ref]}})
    # a grandchild (owned by the pod) goes too
    s.create({"kind": "Event", "metadata": {"name": "ev", "namespace": "default", "ownerReferences": [
        {"kind": "Pod", "name": "j-master-0", "uid": pod["metadata"]["uid"]}]}})
    s.create(_obj("v1", "Pod", "unrelated"))
    port = s.host_port("default", "j-master-0", 23456)
    assert s.host_port("default", "j-master-0", 23456) == port  # stable
    s.patch("PyTorchJob", "default", "j", lambda o: o["metadata"].setdefault("labels", {}).update(a="b"))
    s.delete("PyTorchJob", "default", "j")
    assert [o["metadata"]["name"] for o in s.list("Pod")] == ["unrelated"]
    assert s.list("Service") == [] and s.list("Event") == []
    assert "default/j-master-0:23456" not in s.port_table()  # service ports released
    kinds = [(et, k) for et, k, _ in seen]
    assert (MODIFIED, "PyTorchJob") in kinds
    assert kinds.count((DELETED, "Pod")) == 1 and (DELETED, "Service") in kinds and (DELETED, "Event") in kinds
    assert kinds[0] == (ADDED, "PyTorchJob")
    cancel()
    s.create(_obj("v1", "Pod", "after"))
    assert (ADDED, "Pod", "after") not in seen


def test_sqlite_durability(tmp_path):
    db = str(tmp_path / "store.db")
    s = Store(db_path=db)
    j = s.create(_obj("kubeflow.org/v1", "TFJob", "durable"))
    s.update_status({**j, "status": {"conditions": [{"type": "Running"}]}})
    port = s.host_port("default", "svc", 2222)
    s.create(_obj("v1", "Pod", "gone"))
    s.delete("Pod", "default", "gone")
    s.close()
    s2 = Store(db_path=db)
    j2 = s2.get("TFJob", "default", "durable")
    assert j2["metadata"]["uid"] == j["metadata"]["uid"]
    assert j2["status"]["conditions"][0]["type"] == "Running"
    assert s2.try_get("Pod", "default", "gone") is None
    assert s2.port_table().get("default/svc:2222") == port
    # resourceVersions keep increasing across a restart
    j3 = s2.update({**j2, "spec": {"x": 7}})
    assert int(j3["metadata"]["resourceVersion"]) > int(j2["metadata"]["resourceVersion"])


def test_concurrent_patches_lose_no_update():
    s = Store()
    s.create({"kind": "Pod", "metadata": {"name": "c", "namespace": "default"}, "spec": {"n": 0}})

    def bump():
        for _ in range(200):
            s.patch("Pod", "default", "c", lambda o: o["spec"].__setitem__("n", o["spec"]["n"] + 1))

    ts = [threading.Thread(target=bump) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert s.get("Pod", "default", "c")["spec"]["n"] == 800


def test_event_recorder_aggregates():
    s = Store()
    job = s.create(_obj("kubeflow.org/v1", "PyTorchJob", "j"))
    rec = EventRecorder(s)
    for _ in range(3):
        rec.event(job, "Normal", "SuccessfulCreatePod", "Created pod: j-master-0")
    rec.event(job, "Warning", "Other", "x")
    evs = rec.events_for(job)
    by = {e["reason"]: e for e in evs}
    assert by["SuccessfulCreatePod"]["count"] == 3 and by["Other"]["count"] == 1
    assert by["SuccessfulCreatePod"]["involvedObject"]["uid"] == job["metadata"]["uid"]
