"""HBM-sliced GPU sharing: the allocator packs ``kubedl.io/hbm-gb`` slices onto
shared GPUs within 288 GB, keeps exclusive and shared use apart, and the
scheduler/kubelet carry the slice to the rank as ``KDL_HBM_LIMIT_GB``."""
import time

import pytest

from kubedl_amd.api import common as c
from kubedl_amd.engine.manager import Manager, ManagerOptions
from kubedl_amd.gang.allocator import GPUAllocator, GPUInventory


def test_slices_pack_best_fit_and_release():
    a = GPUAllocator(GPUInventory(4))
    # four 64 GB slices share one GPU (256 <= 288), the fifth does not fit there
    for i in range(4):
        al = a.allocate(f"j{i}", {"p": 0}, {"p": 64})
        assert al.pods["p"] == [0] and al.slices == {"p": 64}
    al = a.allocate("j4", {"p": 0}, {"p": 64})
    assert al.pods["p"] == [1]
    assert a.hbm_free()[0] == pytest.approx(288 - 256) and a.hbm_free()[1] == pytest.approx(224)
    # a 32 GB slice fills GPU 0's remaining room (best fit: the fullest that still fits)
    assert a.allocate("j5", {"p": 0}, {"p": 32}).pods["p"] == [0]
    assert a.used() == 2 and a.free == [2, 3]
    assert a.hbm_used() == pytest.approx(64 * 5 + 32)
    # releasing every slice of GPU 1 frees the GPU
    assert a.release("j4") == [1]
    assert a.free == [1, 2, 3]


def test_exclusive_and_shared_never_mix():
    a = GPUAllocator(GPUInventory(2))
    assert a.allocate("s", {"p": 0}, {"p": 10}).pods["p"] == [0]
    # two whole GPUs are not available any more (GPU 0 carries a slice)
    assert a.allocate("x", {"a": 1, "b": 1}) is None
    x = a.allocate("x", {"a": 1})
    assert x.pods["a"] == [1] and x.gpus == [1]
    # no room for a slice on an exclusively owned GPU, and GPU 0 has only 278 GB left
    assert a.allocate("big", {"p": 0}, {"p": 280}) is None
    assert a.allocate("fits", {"p": 0}, {"p": 278}).pods["p"] == [0]


def test_gang_with_slices_is_all_or_nothing():
    a = GPUAllocator(GPUInventory(1))
    # a three-member gang of 100 GB slices cannot fit one 288 GB GPU: nothing is placed
    assert a.allocate("g", {"m": 0, "w0": 0, "w1": 0}, {"m": 100, "w0": 100, "w1": 100}) is None
    assert a.hbm_free()[0] == pytest.approx(288) and a.used() == 0
    al = a.allocate("g", {"m": 0, "w0": 0}, {"m": 100, "w0": 100})
    assert al.pods == {"m": [0], "w0": [0]}
    with pytest.raises(ValueError):
        a.allocate("bad", {"p": 0}, {"p": -1})
    assert a.allocate("huge", {"p": 0}, {"p": 300}) is None


def test_scheduler_binds_slice_and_kubelet_exports_limit(tmp_path, monkeypatch):
    """Two single-pod jobs with 100 GB slices land on the same GPU; each rank sees
    KDL_HBM_LIMIT_GB=100 and HIP_VISIBLE_DEVICES of that GPU."""
    monkeypatch.setenv("KDL_ZYGOTE", "0")
    m = Manager(ManagerOptions(home=str(tmp_path), gpus=2)).start()
    try:
        out = tmp_path / "env"
        out.mkdir()
        for name in ("s1", "s2"):
            job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                   "metadata": {"name": name, "namespace": "default"},
                   "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1, "restartPolicy": "Never", "template": {
                       "spec": {"containers": [{
                           "name": "pytorch", "image": "kubedl-amd/sleep",
                           "command": ["bash", "-c",
                                       f"echo $HIP_VISIBLE_DEVICES $KDL_HBM_LIMIT_GB > {out}/{name}; sleep 2"],
                           "resources": {"limits": {c.HBM_RESOURCE: 100}}}]}}}}}}
            m.apply(job)
        for name in ("s1", "s2"):
            st = m.wait_for_condition("PyTorchJob", "default", name, ["Succeeded", "Failed"], timeout=60)
            assert c.last_condition_type(st["status"]) == "Succeeded"
        got = {name: (out / name).read_text().split() for name in ("s1", "s2")}
        assert got["s1"] == got["s2"] == ["0", "100"], got
        deadline = time.time() + 10
        while m.allocator.used() and time.time() < deadline:
            time.sleep(0.1)
        assert m.allocator.used() == 0
    finally:
        m.stop()


def test_hbm_quantity_parsing():
    assert c.parse_hbm_gb("32") == 32 and c.parse_hbm_gb(16.5) == 16.5
    assert c.parse_hbm_gb("32G") == pytest.approx(32) and c.parse_hbm_gb("32Gi") == pytest.approx(34.359738368)
    assert c.parse_hbm_gb("512Mi") == pytest.approx(0.536870912)
    with pytest.raises(ValueError):
        c.parse_hbm_gb("lots")
    with pytest.raises(ValueError):
        c.parse_hbm_gb("-4")


def _job(name, containers):
    return {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": name, "namespace": "default"},
            "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1, "restartPolicy": "Never", "template": {
                "spec": {"containers": containers}}}}}}


def test_per_container_hbm_and_malformed_request_isolated(tmp_path, monkeypatch):
    """(1) each container of a two-container slice pod caps its allocator
    at its OWN request, not the pod's summed slice; (2) a pod with a malformed
    kubedl.io/hbm-gb is marked Unschedulable without stopping the scheduler pass
    for the other pods on the node."""
    monkeypatch.setenv("KDL_ZYGOTE", "0")
    m = Manager(ManagerOptions(home=str(tmp_path / "home"), gpus=2)).start()
    try:
        out = tmp_path / "env"
        out.mkdir()
        bad = {"name": "pytorch", "image": "kubedl-amd/sleep", "command": ["true"],
               "resources": {"limits": {c.HBM_RESOURCE: "lots"}}}
        m.apply(_job("bad", [bad]))
        ctrs = [{"name": n, "image": "kubedl-amd/sleep",
                 "command": ["bash", "-c", f"echo $KDL_HBM_LIMIT_GB > {out}/{n}"],
                 "resources": {"limits": {c.HBM_RESOURCE: gb}}} for n, gb in (("pytorch", "100G"), ("side", 50))]
        m.apply(_job("two", ctrs))
        st = m.wait_for_condition("PyTorchJob", "default", "two", ["Succeeded", "Failed"], timeout=60)
        assert c.last_condition_type(st["status"]) == "Succeeded", st["status"]
        assert (out / "pytorch").read_text().split() == ["100"]
        assert (out / "side").read_text().split() == ["50"]
        deadline = time.time() + 10
        msg = ""
        while time.time() < deadline:
            pod = m.store.try_get("Pod", "default", "bad-master-0")
            conds = ((pod or {}).get("status") or {}).get("conditions") or []
            msg = " ".join(x.get("message", "") for x in conds)
            if "invalid resource request" in msg:
                break
            time.sleep(0.1)
        assert "invalid resource request" in msg, msg
    finally:
        m.stop()


def test_gang_ranks_see_the_gang_gpu_set(tmp_path, monkeypatch):
    """Gang members see the gang's GPUs with their own first (cuda:0 is the
    rank's GPU, as in a pod; peers visible for the xGMI transports),
    LOCAL_RANK = 0, LOCAL_WORLD_SIZE = gang size; two concurrent 4-rank gangs
    get disjoint sets."""
    from kubedl_amd.runtime.gpu_env import rank_gpu_env
    assert rank_gpu_env(["5"], ["7", "5", "6", "4"]) == {"HIP_VISIBLE_DEVICES": "5,4,6,7", "LOCAL_RANK": "0",
                                                         "LOCAL_WORLD_SIZE": "4", "KDL_GANG_GPU_INDEX": "1"}
    assert rank_gpu_env(["3"]) == {"HIP_VISIBLE_DEVICES": "3", "LOCAL_RANK": "0", "LOCAL_WORLD_SIZE": "1"}
    monkeypatch.setenv("KDL_ZYGOTE", "0")
    m = Manager(ManagerOptions(home=str(tmp_path / "home"), gpus=8, gang_scheduler_name="kdl-gang")).start()
    try:
        out = tmp_path / "env"
        out.mkdir()
        for name in ("ga", "gb"):
            ctr = {"name": "pytorch", "image": "x", "resources": {"limits": {"amd.com/gpu": 1}},
                   "command": ["bash", "-c", f"echo $HIP_VISIBLE_DEVICES $LOCAL_RANK $LOCAL_WORLD_SIZE $RANK "
                                             f"> {out}/{name}-$RANK; sleep 1"]}
            spec = lambda n: {"replicas": n, "restartPolicy": "Never",  # noqa: E731
                              "template": {"spec": {"containers": [dict(ctr)]}}}
            m.apply({"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                     "metadata": {"name": name, "namespace": "default"},
                     "spec": {"pytorchReplicaSpecs": {"Master": spec(1), "Worker": spec(3)}}})
        for name in ("ga", "gb"):
            st = m.wait_for_condition("PyTorchJob", "default", name, ["Succeeded", "Failed"], timeout=60)
            assert c.last_condition_type(st["status"]) == "Succeeded", st["status"]
        sets = {}
        for name in ("ga", "gb"):
            rows = [(out / f"{name}-{r}").read_text().split() for r in range(4)]
            vis = {",".join(sorted(row[0].split(","), key=int)) for row in rows}
            assert len(vis) == 1, rows  # every rank of a job sees the same set
            gl = vis.pop().split(",")
            assert len(gl) == 4 and all(row[2] == "4" and row[1] == "0" for row in rows)
            # each rank's own device (cuda:0 = first visible) is distinct
            assert sorted(row[0].split(",")[0] for row in rows) == sorted(gl)
            sets[name] = set(gl)
        assert not (sets["ga"] & sets["gb"])  # disjoint gangs
        # each gang inside one NUMA half of the node (allocator best fit)
        halves = [set(map(str, g)) for g in m.allocator.inv.numa_groups]
        assert all(any(sets[n] <= h for h in halves) for n in sets), (sets, halves)
    finally:
        m.stop()
