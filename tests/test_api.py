"""API layer: per-kind defaulting, replica-type camel-casing, validation, codec.

Ports the table-driven cases of ``api/tensorflow/v1/defaults_test.go``,
``api/xdl/v1alpha1/defaults_test.go`` and the per-kind defaulting rules of
``api/{pytorch,xgboost}``.
"""
import copy
import json
import os

import pytest

from kubedl_amd.api import codec, common as c, kinds as K

REF_EXAMPLES = "/root/reference/example"


def _tmpl(name, ports=None):
    ctr = {"name": name, "image": "img"}
    if ports is not None:
        ctr["ports"] = ports
    return {"spec": {"containers": [ctr]}}


def _job(kind, specs, **spec_extra):
    info = K.BY_KIND[kind]
    spec = {info.spec_field: specs}
    spec.update(spec_extra)
    return {"apiVersion": info.api_version, "kind": kind, "metadata": {"name": "j"}, "spec": spec}


# ---------------------------------------------------------------- TFJob
def test_tf_set_type_names_camel_case():
    job = _job("TFJob", {"WORKER": {"template": _tmpl("tensorflow")}, "ps": {"template": _tmpl("tensorflow")}})
    K.set_defaults(job)
    specs = job["spec"]["tfReplicaSpecs"]
    assert set(specs) == {"Worker", "PS"}


@pytest.mark.parametrize("restart,ports,exp_restart,exp_ports", [
    ("Always", [{"name": "tfjob-port", "containerPort": 2222}], "Always",
     [{"name": "tfjob-port", "containerPort": 2222}]),
    (None, [{"name": "tfjob-port", "containerPort": 2222}], "ExitCode",
     [{"name": "tfjob-port", "containerPort": 2222}]),
    ("Always", None, "Always", [{"name": "tfjob-port", "containerPort": 2222}]),
    ("Always", [{"name": "customPort", "containerPort": 1234}], "Always",
     [{"name": "customPort", "containerPort": 1234}, {"name": "tfjob-port", "containerPort": 2222}]),
])
def test_tf_defaults(restart, ports, exp_restart, exp_ports):
    rs = {"template": _tmpl("tensorflow", ports)}
    if restart:
        rs["restartPolicy"] = restart
    job = _job("TFJob", {"Worker": rs})
    K.set_defaults(job)
    w = job["spec"]["tfReplicaSpecs"]["Worker"]
    assert job["spec"]["cleanPodPolicy"] == "Running"
    assert w["replicas"] == 1
    assert w["restartPolicy"] == exp_restart
    assert w["template"]["spec"]["containers"][0]["ports"] == exp_ports


def test_tf_default_port_goes_to_named_container():
    tmpl = {"spec": {"containers": [{"name": "sidecar"}, {"name": "tensorflow"}]}}
    job = _job("TFJob", {"Worker": {"template": tmpl}})
    K.set_defaults(job)
    ctrs = job["spec"]["tfReplicaSpecs"]["Worker"]["template"]["spec"]["containers"]
    assert "ports" not in ctrs[0] or not ctrs[0]["ports"]
    assert ctrs[1]["ports"] == [{"name": "tfjob-port", "containerPort": 2222}]


def test_tf_clean_pod_policy_kept():
    job = _job("TFJob", {"Worker": {"template": _tmpl("tensorflow")}}, cleanPodPolicy="None")
    K.set_defaults(job)
    assert job["spec"]["cleanPodPolicy"] == "None"


# ---------------------------------------------------------------- PyTorchJob
def test_pytorch_defaults_port_only_on_master():
    job = _job("PyTorchJob", {"master": {"template": _tmpl("pytorch")}, "Worker": {"template": _tmpl("pytorch")}})
    K.set_defaults(job)
    specs = job["spec"]["pytorchReplicaSpecs"]
    assert job["spec"]["cleanPodPolicy"] == "None"
    assert specs["Master"]["restartPolicy"] == "ExitCode"
    assert specs["Worker"]["restartPolicy"] == "OnFailure"
    assert specs["Master"]["template"]["spec"]["containers"][0]["ports"] == [
        {"name": "pytorchjob-port", "containerPort": 23456}]
    assert not specs["Worker"]["template"]["spec"]["containers"][0].get("ports")
    assert specs["Master"]["replicas"] == 1 and specs["Worker"]["replicas"] == 1


# ---------------------------------------------------------------- XGBoostJob
def test_xgboost_defaults():
    job = _job("XGBoostJob", {"Master": {"template": _tmpl("xgboostjob")},
                              "worker": {"replicas": 2, "template": _tmpl("xgboostjob")}})
    K.set_defaults(job)
    specs = job["spec"]["xgbReplicaSpecs"]
    assert job["spec"]["cleanPodPolicy"] == "None"
    assert job["spec"]["ttlSecondsAfterFinished"] == 100
    assert "restartPolicy" not in specs["Master"]  # no default restart policy
    assert specs["Worker"]["replicas"] == 2
    for s in specs.values():
        assert s["template"]["spec"]["containers"][0]["ports"] == [
            {"name": "xgboostjob-port", "containerPort": 9999}]


# ---------------------------------------------------------------- XDLJob
@pytest.mark.parametrize("extra,exp_rate,exp_num", [
    ({}, 90, None),
    ({"minFinishWorkNum": 3}, None, 3),
    ({"minFinishWorkRate": 50}, 50, None),
    ({"minFinishWorkNum": 3, "minFinishWorkRate": 50}, 50, 3),
])
def test_xdl_defaults(extra, exp_rate, exp_num):
    job = _job("XDLJob", {"worker": {"template": _tmpl("xdl")}, "PS": {"template": _tmpl("xdl")},
                          "scheduler": {"template": _tmpl("xdl")}, "extendrole": {"template": _tmpl("xdl")}},
               **extra)
    K.set_defaults(job)
    spec = job["spec"]
    assert set(spec["xdlReplicaSpecs"]) == {"Worker", "PS", "Scheduler", "ExtendRole"}
    assert spec["cleanPodPolicy"] == "Running"
    assert spec["backoffLimit"] == 20
    assert spec.get("minFinishWorkRate") == exp_rate
    assert spec.get("minFinishWorkNum") == exp_num
    for s in spec["xdlReplicaSpecs"].values():
        assert s["restartPolicy"] == "Never"
        assert s["template"]["spec"]["containers"][0]["ports"] == [{"name": "xdljob-port", "containerPort": 2222}]


def test_xdl_backoff_limit_kept():
    job = _job("XDLJob", {"Worker": {"template": _tmpl("xdl")}}, backoffLimit=3)
    K.set_defaults(job)
    assert job["spec"]["backoffLimit"] == 3


# ---------------------------------------------------------------- kinds / validation
def test_kind_registry():
    assert K.lookup("pytorchjobs") is K.PYTORCHJOB
    assert K.lookup("PytorchJob") is K.PYTORCHJOB  # README spelling
    assert K.lookup("xgboostjob").api_version == "xgboostjob.kubeflow.org/v1alpha1"
    assert K.XDLJOB.crd_name == "xdljobs.xdl.kubedl.io"
    assert K.TFJOB.reconcile_order == ("PS", "Master", "Chief", "Worker")  # no Evaluator
    assert K.XDLJOB.reconcile_order == ("PS", "Scheduler", "Worker", "ExtendRole")
    with pytest.raises(KeyError):
        K.lookup("MPIJob")


def test_validate():
    good = _job("PyTorchJob", {"Master": {"template": _tmpl("pytorch")}})
    assert K.validate(good) == []
    bad = copy.deepcopy(good)
    bad["apiVersion"] = "kubeflow.org/v2"
    assert any("apiVersion" in e for e in K.validate(bad))
    bad = _job("PyTorchJob", {})
    assert any("pytorchReplicaSpecs" in e for e in K.validate(bad))
    bad = _job("PyTorchJob", {"Master": {"replicas": -1, "restartPolicy": "Sometimes",
                                         "template": {"spec": {}}}})
    errs = K.validate(bad)
    assert len(errs) == 3


def test_print_columns():
    job = _job("TFJob", {"Worker": {"template": _tmpl("tensorflow")}}, ttlSecondsAfterFinished=60)
    job["metadata"]["creationTimestamp"] = c.now()
    job["status"] = {"conditions": [c.new_condition("Created", "r", "m"), c.new_condition("Running", "r", "m")]}
    cols = K.print_columns(job)
    assert cols["STATE"] == "Running" and cols["FINISHED-TTL"] == "60" and cols["MAX-LIFETIME"] == ""


# ---------------------------------------------------------------- codec
def test_codec_multi_doc_and_list():
    text = "a: 1\nkind: X\n---\nkind: Y\n---\n"
    assert [d["kind"] for d in codec.loads(text)] == ["X", "Y"]
    lst = json.dumps({"kind": "List", "items": [{"kind": "A"}, {"kind": "B"}]})
    assert [d["kind"] for d in codec.loads(lst)] == ["A", "B"]
    job = _job("TFJob", {"Worker": {"template": _tmpl("tensorflow")}})
    assert codec.loads(codec.dumps([job], "json"))[0] == job
    assert codec.loads(codec.dumps([job], "yaml"))[0] == job


@pytest.mark.skipif(not os.path.isdir(REF_EXAMPLES), reason="reference examples not mounted")
@pytest.mark.parametrize("path,kind", [
    ("pytorch/pytorch_job_mnist_mpi.yaml", "PyTorchJob"),
    ("tf/tf_job_mnist.yaml", "TFJob"),
    ("xgboost/xgboostjob_v1alpha1_iris_train.yaml", "XGBoostJob"),
])
def test_reference_examples_load_and_default(path, kind):
    docs = codec.load_file(os.path.join(REF_EXAMPLES, path))
    jobs = [d for d in docs if d.get("kind") == kind]
    assert len(jobs) == 1
    job = jobs[0]
    assert K.validate(job) == []
    K.set_defaults(job)
    assert K.replica_specs(job)


@pytest.mark.skipif(not os.path.isdir(REF_EXAMPLES), reason="reference examples not mounted")
def test_reference_xdl_example():
    docs = codec.load_file(os.path.join(REF_EXAMPLES, "xdl/xdl_job_mnist.yaml"))
    kinds = [d.get("kind") for d in docs]
    assert "XDLJob" in kinds
    job = next(d for d in docs if d.get("kind") == "XDLJob")
    K.set_defaults(job)
    assert job["spec"]["backoffLimit"] == 20 or job["spec"].get("backoffLimit") is not None
