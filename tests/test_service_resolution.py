"""Peer-address resolution does not depend on store timing (VERDICT r4 missing 2).

The reference's cluster-spec endpoints are headless-Service DNS names that
resolve whenever the peer's Service exists (``controllers/tensorflow/
tensorflow.go:120-139``, ``pkg/job_controller/service.go:263-276``).  The
kubelet renders a rank's env once, at spawn, so every ``<job>-<rt>-<i>`` of the
owning job's replica specs must resolve from the job alone, to the same port
the peer's Service gets later; and a rank whose env names a service nothing
accounts for is held until it appears.
"""
import json
import os
import sys
import time

from kubedl_amd.runtime.kubelet import Kubelet, ServiceResolver
from kubedl_amd.store import Store

PY = sys.executable


def _tfjob(store):
    return store.create({
        "apiVersion": "kubeflow.org/v1", "kind": "TFJob",
        "metadata": {"name": "tf", "namespace": "default", "uid": "job-uid"},
        "spec": {"tfReplicaSpecs": {"PS": {"replicas": 1}, "Worker": {"replicas": 2}}}})


def _owner(job):
    return [{"apiVersion": job["apiVersion"], "kind": job["kind"], "name": job["metadata"]["name"],
             "uid": job["metadata"]["uid"], "controller": True}]


TF_CONFIG = json.dumps({"cluster": {"ps": ["tf-ps-0.default.svc:2222"],
                                    "worker": ["tf-worker-0.default.svc:2222", "tf-worker-1.default.svc:2222"]},
                        "task": {"type": "worker", "index": 0}, "environment": "cloud"})


def test_resolver_uses_job_replica_specs_without_services():
    store = Store()
    job = _tfjob(store)
    pod = {"metadata": {"name": "tf-worker-0", "namespace": "default", "ownerReferences": _owner(job)}}
    r = ServiceResolver(store, domain="")
    assert r.job_names("default", pod) == {"tf-ps-0", "tf-worker-0", "tf-worker-1"}
    out = r.resolve("default", "tf-worker-0", {"TF_CONFIG": TF_CONFIG}, pod)
    cfg = json.loads(out["TF_CONFIG"])
    addrs = [a for v in cfg["cluster"].values() for a in v]
    assert all(a.startswith("127.0.0.1:") for a in addrs), addrs
    assert r.unresolved("default", out) == []
    # the port a rank was handed before the Service existed is the Service's port
    assert cfg["cluster"]["worker"][1] == f"127.0.0.1:{store.host_port('default', 'tf-worker-1', 2222)}"
    # a replica index past the spec is not invented
    out = r.resolve("default", "tf-worker-0", {"X": "tf-worker-2.default.svc:2222"}, pod)
    assert r.unresolved("default", out) == ["tf-worker-2.default.svc"]


def _rank_pod(name, env, owner=None):
    script = "import os,json; open(os.environ['OUT'],'w').write(json.dumps(dict(os.environ)))"
    md = {"name": name, "namespace": "default"}
    if owner:
        md["ownerReferences"] = owner
    return {"apiVersion": "v1", "kind": "Pod", "metadata": md,
            "spec": {"nodeName": "localhost", "restartPolicy": "Never",
                     "containers": [{"name": "main", "image": "kubedl-amd/sleep", "command": [PY, "-c", script],
                                     "env": [{"name": k, "value": v} for k, v in env.items()]}]}}


def _wait_file(path, timeout=30.0):
    t_end = time.time() + timeout
    while time.time() < t_end:
        if os.path.exists(path) and os.path.getsize(path):
            try:
                return json.load(open(path))
            except ValueError:
                pass
        time.sleep(0.05)
    raise AssertionError(f"{path} never written")


def test_worker_spawned_before_any_peer_gets_full_tf_config(tmp_path):
    """Worker 0 is the only object besides the job: no PS / worker-1 Pod or Service
    exists when it starts, and its TF_CONFIG is still fully rewritten."""
    store = Store()
    job = _tfjob(store)
    k = Kubelet(store, str(tmp_path / "node"), zygote=False)
    k.start()
    try:
        out = str(tmp_path / "w0.json")
        store.create(_rank_pod("tf-worker-0", {"TF_CONFIG": TF_CONFIG, "OUT": out}, _owner(job)))
        env = _wait_file(out)
        cfg = json.loads(env["TF_CONFIG"])
        addrs = [a for v in cfg["cluster"].values() for a in v]
        assert all(a.startswith("127.0.0.1:") for a in addrs), addrs
        # the peers' Services, created afterwards, map to the same ports
        for name, addr in (("tf-ps-0", cfg["cluster"]["ps"][0]), ("tf-worker-1", cfg["cluster"]["worker"][1])):
            assert addr == f"127.0.0.1:{store.host_port('default', name, 2222)}"
    finally:
        k.stop()


def test_rank_naming_unknown_service_is_held_until_it_exists(tmp_path):
    store = Store()
    k = Kubelet(store, str(tmp_path / "node"), zygote=False)
    k.start()
    try:
        out = str(tmp_path / "ghost.json")
        store.create(_rank_pod("client", {"PEER": "ghost.default.svc:1234", "OUT": out}))
        time.sleep(0.6)
        assert not os.path.exists(out), "rank started with an unresolvable peer name"
        store.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "ghost", "namespace": "default"},
                      "spec": {"clusterIP": "None", "ports": [{"port": 1234}]}})
        env = _wait_file(out)
        assert env["PEER"] == f"127.0.0.1:{store.host_port('default', 'ghost', 1234)}"
        log = open(k.log_path("default", "client")).read()
        assert "holding main: unresolved ['ghost.default.svc']" in log
    finally:
        k.stop()
