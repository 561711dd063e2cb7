"""Concurrency stress (SURVEY.md §5 "race detection": the reference relies on
controller-runtime's one-key-at-a-time queues and never stress-tests them).

Many jobs submitted at once from several threads, reconciled by several
workers per kind, gang-scheduled onto 8 fake GPUs: every job reaches the
terminal state its ranks dictate, the allocator never over-commits, every GPU
is released, no reconcile raises, and the counters add up.
"""
import os
import sys
import threading
import time

from kubedl_amd.api import common as c
from kubedl_amd.engine.manager import Manager, ManagerOptions

PY = sys.executable


def _job(name, code):
    script = f"import time, sys; time.sleep(0.2); sys.exit({code})"
    ctr = lambda: {"name": "pytorch", "image": "kubedl-amd/none", "command": [PY, "-c", script],  # noqa: E731
                   "resources": {"limits": {"amd.com/gpu": 1}}}
    return {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": name, "namespace": "default"},
            "spec": {"pytorchReplicaSpecs": {
                "Master": {"replicas": 1, "restartPolicy": "Never", "template": {"spec": {"containers": [ctr()]}}},
                "Worker": {"replicas": 1, "restartPolicy": "Never", "template": {"spec": {"containers": [ctr()]}}}}}}


def test_concurrent_submits_gang_and_reconcile_workers(tmp_path):
    os.environ["KDL_RESTART_BACKOFF_BASE"] = "0.05"
    m = Manager(ManagerOptions(home=str(tmp_path), gpus=8, gang_scheduler_name="kdl-gang",
                               max_reconciles=4)).start()
    peak, stop = [0], threading.Event()

    def watch_alloc():
        while not stop.is_set():
            peak[0] = max(peak[0], m.allocator.used())
            time.sleep(0.005)

    mon = threading.Thread(target=watch_alloc, daemon=True)
    mon.start()
    try:
        names = [(f"s{i}", 1 if i % 5 == 4 else 0) for i in range(16)]
        chunks = [names[i::4] for i in range(4)]
        threads = [threading.Thread(target=lambda ch=ch: [m.apply(_job(n, code)) for n, code in ch]) for ch in chunks]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        done = {}
        for n, code in names:
            j = m.wait_for_condition("PyTorchJob", "default", n, ["Succeeded", "Failed"], timeout=120)
            done[n] = [x["type"] for x in j["status"]["conditions"] if x["status"] == "True"]
        for n, code in names:
            want = "Failed" if code else "Succeeded"
            assert want in done[n], (n, done[n])
        assert peak[0] <= 8
        deadline = time.time() + 10
        while m.allocator.used() and time.time() < deadline:
            time.sleep(0.05)
        assert m.allocator.used() == 0
        assert not [e for loop in m.loops.values() for e in loop.errors], \
            [e for loop in m.loops.values() for e in loop.errors]
        reg = m.metrics
        assert reg.created.labels("pytorchjob").get() == 16
        assert reg.success.labels("pytorchjob").get() == 13
        assert reg.failure.labels("pytorchjob").get() == 3
        assert all(c.is_succeeded(j["status"]) or c.is_failed(j["status"]) for j in m.store.list("PyTorchJob"))
    finally:
        stop.set()
        m.stop()
        os.environ.pop("KDL_RESTART_BACKOFF_BASE", None)
