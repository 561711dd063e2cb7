"""Pre-warmed zygote launches: ranks forked from a torch-preloaded process are
re-parented to the kubelet (subreaper), reaped with the right exit code, see
their own env/cwd/log, and launch faster than a cold interpreter."""
import os
import sys
import time

from kubedl_amd.engine.manager import Manager, ManagerOptions


def _job(name, script_mod, args):
    return {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": name, "namespace": "default"},
            "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1, "restartPolicy": "Never", "template": {"spec": {
                "containers": [{"name": "pytorch", "image": "x",
                                "command": [sys.executable, "-u", "-m", script_mod] + args}]}}}}}}


def test_zygote_launch(tmp_path, monkeypatch):
    monkeypatch.setenv("KDL_ZYGOTE", "1")
    m = Manager(ManagerOptions(home=str(tmp_path), gpus=0)).start()
    try:
        assert m.kubelet.zygote is not None
        assert m.kubelet.zygote.ready.wait(120), "zygote never became ready"
        m.apply(_job("z1", "kubedl_amd.workers.pytorch_dist", ["--cpu", "--numel", "16"]))
        job = m.wait_for_condition("PyTorchJob", "default", "z1", ["Succeeded", "Failed"], timeout=60)
        assert [c["type"] for c in job["status"]["conditions"] if c["status"] == "True"][-1] == "Succeeded"
        log = open(m.kubelet.log_path("default", "z1-master-0")).read()
        assert "pre-warmed zygote" in log and "rank 0/1" in log
        # failing module -> exit code propagates through the double fork
        m.apply(_job("z2", "kubedl_amd.workers.no_such_worker", []))
        job = m.wait_for_condition("PyTorchJob", "default", "z2", ["Succeeded", "Failed"], timeout=60)
        pod = m.store.get("Pod", "default", "z2-master-0")
        code = pod["status"]["containerStatuses"][0]["state"]["terminated"]["exitCode"]
        assert code != 0
        assert m.metrics.observed["first"]
    finally:
        m.stop()


def test_node_warm_child_reports_json():
    """runtime/node_warm.py runs in a child process and reports one JSON line
    (on a CPU host: no GPU, nothing warmed, no error)."""
    import os
    from kubedl_amd.runtime.zygote import warm_node
    res = warm_node(dict(os.environ), timeout=120)
    assert "warm_s" in res and "wall_s" in res, res
    assert res["warm"] is False and res.get("reason") == "no GPU", res


def test_node_warm_gpu_comes_from_the_inventory(tmp_path):
    """the node warm-up runs on a GPU of the node's inventory (its
    last one: the allocator hands GPUs out from 0), not on whatever is physical
    GPU 0, and a node without GPUs has no warm-up at all."""
    from kubedl_amd.runtime.kubelet import Kubelet
    from kubedl_amd.store import Store
    assert Kubelet(Store(), str(tmp_path / "a"), zygote=False, gpus=0).warm_gpu is None
    assert Kubelet(Store(), str(tmp_path / "b"), zygote=False, gpus=8).warm_gpu == 7
    assert Kubelet(Store(), str(tmp_path / "c"), zygote=False, gpus=1).warm_gpu == 0


def test_no_rank_of_an_8_rank_job_waits_on_the_node_warm_up(tmp_path, monkeypatch):
    """the node warm-up never gates pod starts.  An 8-rank
    gang (8 fake GPUs, one of them the warm-up's) is submitted while a 6 s
    warm-up holds its lock: every pod is Ready well before the warm-up ends
    (launch delays unaffected), each rank waits on the lock after its Ready,
    before its first collective, and the job succeeds."""
    import json
    from kubedl_amd.api import common as c
    from kubedl_amd.runtime import zygote as zmod
    warm_s = 6.0
    done = {}

    def fake_warm(env, timeout=180.0, gpu=None, procs=None):
        time.sleep(warm_s)
        done["t"] = time.time()
        return {"warm": True, "gpu": gpu, "wall_s": warm_s}

    monkeypatch.setattr(zmod, "warm_node", fake_warm)
    monkeypatch.setenv("KDL_ZYGOTE", "1")
    monkeypatch.setenv("KDL_NODE_WARM", "force")
    m = Manager(ManagerOptions(home=str(tmp_path), gpus=8, gang_scheduler_name="kdl-gang")).start()
    try:
        t_start = time.time()
        assert m.kubelet.zygote.warm_gpu == 7 and m.kubelet.zygote._warm_fd is not None
        tmpl = {"spec": {"containers": [{"name": "pytorch", "image": "x", "resources": {"limits": {"amd.com/gpu": 1}},
                                         "command": [sys.executable, "-u", "-m", "kubedl_amd.workers.pytorch_dist",
                                                     "--cpu", "--numel", "16"]}]}}
        job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
               "metadata": {"name": "w8", "namespace": "default"},
               "spec": {"cleanPodPolicy": "None", "pytorchReplicaSpecs": {
                   "Master": {"replicas": 1, "restartPolicy": "Never", "template": tmpl},
                   "Worker": {"replicas": 7, "restartPolicy": "Never", "template": tmpl}}}}
        m.apply(job)
        fin = m.wait_for_condition("PyTorchJob", "default", "w8", ["Succeeded", "Failed"], timeout=240)
        assert c.last_condition_type(fin["status"]) == "Succeeded", fin["status"]
        assert "t" in done
        pods = m.store.list("Pod", "default")
        assert len(pods) == 8
        gpus = {(p["metadata"].get("annotations") or {}).get("kubedl.io/gpus") for p in pods}
        assert "7" in gpus  # one rank sits on the warm-up's GPU
        for p in pods:
            log = open(m.kubelet.log_path("default", p["metadata"]["name"])).read()
            assert "for the node warm-up before the first communicator" in log, log[-800:]
        # job creation -> first / every pod Ready: never the warm-up's 6 s
        first, every = m.metrics.observed["first"], m.metrics.observed["all"]
        assert first and max(first.values()) < warm_s - 1.0, first
        assert every and max(every.values()) < warm_s - 1.0, every
    finally:
        m.stop()
