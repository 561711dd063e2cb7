"""Checkpoint / resume (kubedl_amd/utils/checkpoint.py) and tracing helpers.

- bit-exact resume of the ResNet trainer (CPU, tiny model);
- atomic files, pruning, newest-complete-file selection;
- end to end through the job engine: a rank killed with a retryable exit code
  under the ExitCode policy is recreated and resumes from the last checkpoint
  instead of step 0 (the reference restarts from scratch: SURVEY.md §5).
"""
import json
import os
import sys

import torch

from kubedl_amd.parallel.dist import DistInfo
from kubedl_amd.utils.checkpoint import Checkpointer
from kubedl_amd.utils.trace import StepLog, trace_range
from kubedl_amd.workers.resnet50 import ResNetTrainer

PY = sys.executable


def _trainer():
    info = DistInfo(0, 1, 0, torch.device("cpu"), "gloo")
    return ResNetTrainer(info, batch=2, image=32, tiny=True, num_classes=10, bn_backend="torch", engine="autograd")


def test_trainer_resume_is_bit_exact(tmp_path):
    ref = _trainer()
    for _ in range(4):
        ref.step()
    a = _trainer()
    a.step()
    a.step()
    ck = Checkpointer(str(tmp_path), every=1)
    ck.save(2, a.state_dict())
    b = _trainer()  # fresh process state: random init differs from a's trajectory only via the load
    step, st = ck.load_latest()
    assert step == 2
    b.load_state_dict(st)
    b.step()
    b.step()
    assert torch.equal(b.space.param, ref.space.param)
    assert torch.equal(b.opt.mom, ref.opt.mom)
    for (n, x), (_, y) in zip(b.model.named_buffers(), ref.model.named_buffers()):
        assert torch.equal(x, y), n


def test_checkpointer_atomic_prune_and_latest(tmp_path):
    ck = Checkpointer(str(tmp_path), every=2, keep=2)
    assert not ck.due(0) and not ck.due(1) and ck.due(2) and ck.due(4)
    for s in (2, 4, 6):
        ck.save(s, {"w": torch.full((3,), float(s)), "n": s})
    files = sorted(f for f in os.listdir(tmp_path) if f.endswith(".pt"))
    assert files == ["step-00000004.pt", "step-00000006.pt"]
    assert json.load(open(tmp_path / "latest.json"))["step"] == 6
    (tmp_path / "step-00000008.pt").write_bytes(b"torn")  # a corrupt newer file is skipped
    step, st = ck.load_latest()
    assert step == 6 and st["n"] == 6 and torch.equal(st["w"], torch.full((3,), 6.0))
    # non-writer ranks never write, but read
    ck1 = Checkpointer(str(tmp_path), rank=1, every=2)
    assert ck1.save(8, {"w": torch.zeros(1)}) is None
    assert ck1.load_latest()[0] == 6
    assert Checkpointer(None).load_latest() is None


def test_trace_range_and_steplog(tmp_path):
    with trace_range("phase"):
        pass
    log = StepLog(str(tmp_path / "steps.jsonl"), rank=3)
    log.write(1, 12.5, loss=2.0)
    log.close()
    rec = json.loads((tmp_path / "steps.jsonl").read_text())
    assert rec["rank"] == 3 and rec["step"] == 1 and rec["ms"] == 12.5 and rec["loss"] == 2.0
    assert not StepLog(path="").enabled


def test_exitcode_restart_resumes_from_checkpoint(tmp_path):
    from kubedl_amd.engine.manager import Manager, ManagerOptions
    os.environ["KDL_RESTART_BACKOFF_BASE"] = "0.05"
    m = Manager(ManagerOptions(home=str(tmp_path / "home"), gpus=8, metrics_port=0)).start()
    try:
        ck, steplog = tmp_path / "ckpt", tmp_path / "steps.jsonl"
        env = [{"name": "KDL_CKPT_DIR", "value": str(ck)}, {"name": "KDL_CKPT_EVERY", "value": "1"},
               {"name": "KDL_FAULT", "value": "0:1:137"}, {"name": "KDL_STEP_LOG", "value": str(steplog)}]
        ctr = {"name": "pytorch", "image": "kubedl-amd/none", "env": env,
               "command": [PY, "-m", "kubedl_amd.workers.resnet50", "--tiny", "--cpu", "--steps", "3",
                           "--warmup", "1", "--batch", "2", "--image", "32"]}
        job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": "ck", "namespace": "default"},
               "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1, "restartPolicy": "ExitCode",
                                                           "template": {"spec": {"containers": [ctr]}}}}}}
        m.apply(job)
        done = m.wait_for_condition("PyTorchJob", "default", "ck", ["Succeeded", "Failed"], timeout=240)
        conds = [x["type"] for x in done["status"]["conditions"] if x["status"] == "True"]
        assert "Succeeded" in conds, done["status"]
        steps = [json.loads(line)["step"] for line in steplog.read_text().splitlines()]
        # first run: steps 1, 2 then exit 137 after step 2 is checkpointed; second run resumes at 3
        assert steps == [1, 2, 3, 4], steps
        assert json.load(open(ck / "latest.json"))["step"] == 4
        assert "JobRestarting" in {e["reason"] for e in m.store.list("Event")}
    finally:
        m.stop()
        os.environ.pop("KDL_RESTART_BACKOFF_BASE", None)
