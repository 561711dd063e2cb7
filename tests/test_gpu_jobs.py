"""Multi-rank jobs through the whole control plane on a real MI355X.

A two-rank PyTorchJob whose ranks ask for HBM slices (``kubedl.io/hbm-gb``)
instead of whole GPUs: the scheduler packs both onto GPU 0, the kubelet gives
each rank ``HIP_VISIBLE_DEVICES=0``, ``LOCAL_RANK=0``, its own remapped
``MASTER_PORT`` rendezvous and ``KDL_HBM_LIMIT_GB``; the ranks run the fused
ResNet engine on the GPU with a gloo process group (RCCL refuses two ranks on
one device) and the job reaches Succeeded with both launch delays observed.
On an 8-GPU node the same job with ``amd.com/gpu: 1`` per rank is what
``bench.py --gpus N`` submits.
"""
import time

import pytest
import torch

from kubedl_amd.api import common as c
from kubedl_amd.engine.manager import Manager, ManagerOptions

pytestmark = pytest.mark.gpu


def _rank_spec(name):
    return {"replicas": 1, "restartPolicy": "Never", "template": {"spec": {"containers": [{
        "name": "pytorch", "image": "kubedl-amd/resnet50",
        "args": ["--tiny", "--batch", "8", "--image", "64", "--steps", "3", "--warmup", "1"],
        "env": [{"name": "KDL_DIST_BACKEND", "value": "gloo"}],
        "resources": {"limits": {c.HBM_RESOURCE: 48}}}]}}}


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_two_rank_job_shares_one_gpu_by_hbm_slices(tmp_path):
    m = Manager(ManagerOptions(home=str(tmp_path), gpus=1)).start()
    try:
        job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
               "metadata": {"name": "slices", "namespace": "default"},
               "spec": {"pytorchReplicaSpecs": {"Master": _rank_spec("m"), "Worker": _rank_spec("w")}}}
        m.apply(job)
        done = m.wait_for_condition("PyTorchJob", "default", "slices", ["Succeeded", "Failed"], timeout=300)
        logs = {p: open(m.kubelet.log_path("default", p)).read()[-2000:]
                for p in ("slices-master-0", "slices-worker-0")}
        assert c.last_condition_type(done["status"]) == "Succeeded", (done["status"], logs)
        for p in ("slices-master-0", "slices-worker-0"):
            ann = m.store.get("Pod", "default", p)["metadata"].get("annotations") or {}
            assert ann.get("kubedl.io/gpus") == "0" and ann.get("kubedl.io/hbm-gb") == "48", ann
        uid = done["metadata"]["uid"]
        assert m.metrics.observed["first"].get(uid) is not None
        deadline = time.time() + 30
        while m.allocator.used() and time.time() < deadline:
            time.sleep(0.2)
        assert m.allocator.used() == 0
    finally:
        m.stop()
