"""Engine with fake pod/service controls (the reference's FakeServiceControl +
TestJobController style, ``pkg/job_controller/*_test.go``)."""
import pytest

from kubedl_amd.api import common as c
from kubedl_amd.engine.control import ControllerRefManager, PodControl
from kubedl_amd.engine.job_controller import gen_owner_reference
from kubedl_amd.engine.testing import new_job_controller, new_test_job
from kubedl_amd.store import EventRecorder, Store


def test_create_new_service_records_template_and_owner():
    jc, _, svcs = new_job_controller()
    job = new_test_job(workers=2)
    jc.reconcile_services(job, [], "Worker", job["spec"]["testReplicaSpecs"]["Worker"])
    names = [t["metadata"]["name"] for t in svcs.templates]
    assert names == ["test-job-worker-0", "test-job-worker-1"]
    t = svcs.templates[0]
    assert t["spec"]["clusterIP"] == "None" and t["spec"]["ports"][0]["port"] == 9999
    assert t["metadata"]["labels"][c.REPLICA_INDEX_LABEL] == "0"
    assert svcs.controller_refs[0]["uid"] == job["metadata"]["uid"] and svcs.controller_refs[0]["controller"]


def test_create_limit_and_error_lower_expectations():
    jc, _, svcs = new_job_controller()
    job = new_test_job(workers=3)
    svcs.create_limit = 1
    with pytest.raises(RuntimeError, match="limit 1 already reached"):
        jc.reconcile_services(job, [], "Worker", job["spec"]["testReplicaSpecs"]["Worker"])
    # the failed create was observed again, so only the successful one is outstanding
    key = c.gen_expectation_services_key("default/test-job", "worker")
    assert not jc.expectations.satisfied([key])
    jc.expectations.creation_observed(key)
    assert jc.expectations.satisfied([key])


def test_create_new_pod_labels_and_restart_policy():
    jc, pods, _ = new_job_controller()
    job = new_test_job(workers=1, restart_policy=c.RESTART_POLICY_EXIT_CODE)
    specs = job["spec"]["testReplicaSpecs"]
    jc.create_new_pod(job, "master", "0", specs["Master"], True, specs)
    p = pods.templates[0]
    assert p["metadata"]["name"] == "test-job-master-0"
    assert p["metadata"]["labels"][c.JOB_ROLE_LABEL] == "master"
    assert p["spec"]["restartPolicy"] == c.RESTART_POLICY_NEVER


def test_delete_through_fake_and_injected_error():
    jc, pods, _ = new_job_controller()
    job = new_test_job()
    pod = {"metadata": {"name": "p0", "namespace": "default", "labels": {c.REPLICA_TYPE_LABEL: "worker"}}}
    jc.delete_pod(job, pod)
    assert pods.deleted == ["p0"]
    key = c.gen_expectation_pods_key("default/test-job", "worker")
    assert not jc.expectations.satisfied([key])  # until the informer sees the deletion
    jc.expectations.deletion_observed(key)
    pods.err = RuntimeError("boom")
    with pytest.raises(RuntimeError):
        jc.delete_pod(job, pod)
    assert jc.expectations.satisfied([key])  # a failed delete lowers the expectation again


def test_ref_manager_adopts_orphans_and_releases_mismatches():
    store = Store()
    job = new_test_job()
    sel = {"group-name": "g", "job-name": "test-job"}
    mk = lambda name, labels, refs=None: store.create({"apiVersion": "v1", "kind": "Pod", "metadata": {  # noqa: E731
        "name": name, "namespace": "default", "labels": labels, "ownerReferences": refs or []}, "spec": {}})
    mine = gen_owner_reference(job)
    other = dict(mine, uid="someone-else")
    objs = [mk("orphan", dict(sel)), mk("owned", dict(sel), [mine]), mk("foreign", dict(sel), [other]),
            mk("stale", {"group-name": "g", "job-name": "old"}, [mine])]
    ctl = PodControl(store, EventRecorder(store))
    got = ControllerRefManager(ctl, job, sel, mine).claim(objs)
    assert sorted(o["metadata"]["name"] for o in got) == ["orphan", "owned"]
    assert store.get("Pod", "default", "orphan")["metadata"]["ownerReferences"][0]["uid"] == job["metadata"]["uid"]
    assert store.get("Pod", "default", "stale")["metadata"]["ownerReferences"] == []
    assert store.get("Pod", "default", "foreign")["metadata"]["ownerReferences"][0]["uid"] == "someone-else"


def _failed_pod(name, rt, idx, code):
    return {"metadata": {"name": name, "namespace": "default",
                         "labels": {c.REPLICA_TYPE_LABEL: rt, c.REPLICA_INDEX_LABEL: str(idx)}},
            "status": {"phase": "Failed", "containerStatuses": [
                {"name": "default-container", "state": {"terminated": {"exitCode": code}}}]}}


def _running_pod(name, rt, idx):
    return {"metadata": {"name": name, "namespace": "default",
                         "labels": {c.REPLICA_TYPE_LABEL: rt, c.REPLICA_INDEX_LABEL: str(idx)}},
            "status": {"phase": "Running"}}


def test_gang_restart_skipped_when_a_peer_failed_permanently():
    """rank A exits 137 (retryable) while rank B exits 1 (permanent) in
    the same pass -> B's pod and failure record are kept (no gang teardown), so
    the job fails like the reference's per-pod ExitCode handling."""
    jc, pods, _ = new_job_controller()
    job = new_test_job(workers=2, restart_policy=c.RESTART_POLICY_EXIT_CODE)
    plist = [_failed_pod("test-job-master-0", "master", 0, 137), _failed_pod("test-job-worker-0", "worker", 0, 1),
             _running_pod("test-job-worker-1", "worker", 1)]
    jc.restart_gang(job, plist, {"test-job-master-0"})
    assert pods.deleted == []
    # all peers retryable / alive -> the whole gang is torn down
    plist[1] = _failed_pod("test-job-worker-0", "worker", 0, 143)
    jc.restart_gang(job, plist, {"test-job-master-0"})
    assert sorted(pods.deleted) == ["test-job-worker-0", "test-job-worker-1"]
