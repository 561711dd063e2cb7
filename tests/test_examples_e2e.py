"""The reference's own example jobs (``/root/reference/example/*/*.yaml``),
unchanged, submitted through the control plane (``Manager.apply`` of every
document, as ``kdl run -f``) and driven to Succeeded by the local runtime.

Each example's image maps to the bundled worker for its framework
(kubedl_amd/runtime/images.py): the PyTorch send/recv demo, the TF_CONFIG
stub (TF is not in the image), the distributed hist-GBDT (XGBoost's rabit ->
torch.distributed), and the sparse-embedding CTR job with PS + Scheduler +
Workers (XDL's ``bash -c "exec python mnist.py ... $(TASK_NAME) ..."``
command exercises the kubelet's $(VAR) expansion and shell-wrapper look-through;
its ZooKeeper Service/Deployment documents are stored but need no server).
On this CPU host every rank runs on CPU/gloo; the files are read from the
reference checkout and the test skips if it is absent.
"""
import os

import pytest

from kubedl_amd.api import codec
from kubedl_amd.api import common as c
from kubedl_amd.api import kinds as K
from kubedl_amd.engine.manager import Manager, ManagerOptions

EXAMPLES = "/root/reference/example"
CASES = [
    ("pytorch/pytorch_job_mnist_mpi.yaml", "PyTorchJob", 3),
    ("tf/tf_job_mnist.yaml", "TFJob", 1),
    ("xgboost/xgboostjob_v1alpha1_iris_train.yaml", "XGBoostJob", 3),
    ("xdl/xdl_job_mnist.yaml", "XDLJob", 4),
]


@pytest.mark.parametrize("path,kind,pods", CASES, ids=[c_[1] for c_ in CASES])
def test_reference_example_runs_to_succeeded(path, kind, pods, tmp_path, monkeypatch):
    f = os.path.join(EXAMPLES, path)
    if not os.path.exists(f):
        pytest.skip("reference checkout not present")
    monkeypatch.setenv("KDL_ZYGOTE", "0")
    m = Manager(ManagerOptions(home=str(tmp_path), gpus=0)).start()
    try:
        jobs = [m.apply(obj) for obj in codec.load_file(f)]
        jobs = [j for j in jobs if j["kind"] in K.BY_KIND]
        assert [j["kind"] for j in jobs] == [kind]
        md = jobs[0]["metadata"]
        done = m.wait_for_condition(kind, md["namespace"], md["name"], ["Succeeded", "Failed"], timeout=240)
        st = done["status"]
        assert c.last_condition_type(st) == "Succeeded", st
        assert st.get("completionTime") and st.get("startTime")
        created = [p for p in m.store.list("Pod", md["namespace"])
                   if p["metadata"]["name"].startswith(md["name"] + "-")]
        # every replica of the spec got a pod (cleanPodPolicy None/Running may have removed finished ones)
        seen = {e["message"].split()[-1] for e in m.store.list("Event") if e["reason"] == "SuccessfulCreatePod"}
        assert len(seen) >= pods or len(created) >= pods, (seen, [p["metadata"]["name"] for p in created])
        assert m.metrics.observed["first"].get(md["uid"]) is not None  # launch delay observed
    finally:
        m.stop()
