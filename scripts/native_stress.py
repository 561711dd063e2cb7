"""Exercise the native host runtime (csrc/runtime: spawn / reap / kill_group /
subreaper / GPU best-fit) directly and through the control plane, with plain
``python -c`` ranks (no torch, no GPU).  Run under the sanitizer build by
``make native-asan`` / tests/test_native_asan.py:

    KDL_NATIVE_SO=build/kdl_ext/asan/_native.so LD_PRELOAD=$(gcc -print-file-name=libasan.so) \\
    ASAN_OPTIONS=detect_leaks=0 python scripts/native_stress.py

Prints ``native stress ok`` and exits 0 when every scenario behaved.
"""
import os
import signal
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("KDL_ZYGOTE", "0")
os.environ.setdefault("KDL_RESTART_BACKOFF_BASE", "0.05")

from kubedl_amd.runtime import native  # noqa: E402

PY = sys.executable


def direct(nat, tmp):
    nat.set_child_subreaper()
    env = [f"{k}={v}" for k, v in os.environ.items()]
    log = os.path.join(tmp, "direct.log")
    pids = {}
    for code in (0, 3, 137):
        pids[nat.spawn([PY, "-c", f"import os; os._exit({code})"], env, tmp, log, log)] = code
    try:  # exec failure is reported synchronously by the spawner's status pipe
        nat.spawn(["/nonexistent/binary"], env, tmp, log, log)
        raise AssertionError("spawn of a missing binary succeeded")
    except FileNotFoundError:
        pass
    sleeper = nat.spawn([PY, "-c", "import time; time.sleep(60)"], env, None, log, log)
    assert nat.alive(sleeper)
    got, t_end = {}, time.time() + 30
    while len(got) < 3 and time.time() < t_end:
        for pid, code in nat.reap([p for p in pids if p not in got]):  # (a reaped pid reports -1 after)
            got[pid] = code
        time.sleep(0.01)
    for pid, code in pids.items():
        assert got[pid] == code, (pid, got.get(pid), code)
    assert nat.kill_group(sleeper, signal.SIGTERM) == 0
    t_end = time.time() + 10
    reaped = []
    while not reaped and time.time() < t_end:
        reaped = nat.reap([sleeper])
        time.sleep(0.01)
    assert reaped and reaped[0][1] in (-15, 143, 128 + 15), reaped
    # GPU placement core: all-or-nothing best fit over the two NUMA halves
    groups = [0x0F, 0xF0]
    for free, n in ((0xFF, 4), (0b11100110, 3), (0x81, 2), (0x08, 2), (0xFF, 8), (0, 1)):
        got = nat.best_fit(free, n, groups)
        if bin(free).count("1") < n:
            assert got == -1, (free, n, got)
        else:
            assert got & ~free == 0 and bin(got).count("1") == n, (free, n, got)


def control_plane(tmp):
    from kubedl_amd.engine.manager import Manager, ManagerOptions
    m = Manager(ManagerOptions(home=os.path.join(tmp, "home"), gpus=8, gang_scheduler_name="kdl-gang")).start()

    def ctr(code, gpus=1):
        return {"name": "pytorch", "image": "none", "command": [PY, "-c", code],
                "resources": {"limits": {"amd.com/gpu": gpus}}}

    def job(name, master, worker=None, policy="ExitCode", workers=1):
        specs = {"Master": {"replicas": 1, "restartPolicy": policy, "template": {"spec": {"containers": [master]}}}}
        if worker is not None:
            specs["Worker"] = {"replicas": workers, "restartPolicy": policy,
                               "template": {"spec": {"containers": [worker]}}}
        return {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": name, "namespace": "default"},
                "spec": {"pytorchReplicaSpecs": specs}}

    try:
        marker = os.path.join(tmp, "once")
        # a worker that dies once with a retryable code: gang restart, then success
        flaky = (f"import os,sys,time; p={marker!r}\n"
                 "if not os.path.exists(p): open(p,'w').close(); os._exit(137)\n"
                 "time.sleep(0.2)")
        m.apply(job("gang", ctr("import time; time.sleep(0.5)"), ctr(flaky), workers=3))
        m.apply(job("ok", ctr("pass")))
        m.apply(job("perm", ctr("import os; os._exit(1)")))
        m.apply(job("onfail", ctr("import os; os._exit(0)"), ctr("import os; os._exit(0)"), policy="OnFailure"))
        for name, want in (("gang", "Succeeded"), ("ok", "Succeeded"), ("perm", "Failed"), ("onfail", "Succeeded")):
            j = m.wait_for_condition("PyTorchJob", "default", name, ["Succeeded", "Failed"], timeout=120)
            conds = [c["type"] for c in j["status"]["conditions"] if c["status"] == "True"]
            assert want in conds, (name, j["status"])
        assert "GangRestart" in {e["reason"] for e in m.store.list("Event")}
        # delete a running job: its ranks are killed through kill_group
        m.apply(job("long", ctr("import time; time.sleep(120)")))
        m.wait_for_condition("PyTorchJob", "default", "long", ["Running"], timeout=60)
        m.delete("PyTorchJob", "default", "long")
        t_end = time.time() + 30
        while m.kubelet.running_pods() and time.time() < t_end:
            time.sleep(0.05)
        assert not m.kubelet.running_pods(), m.kubelet.running_pods()
        assert m.allocator.used() == 0
    finally:
        m.stop()


def main():
    nat = native.load()
    assert nat is not None, "native module not built"
    print("native module:", getattr(nat, "__file__", "?"), flush=True)
    with tempfile.TemporaryDirectory(prefix="kdl-native-") as tmp:
        direct(nat, tmp)
        control_plane(tmp)
    print("native stress ok", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
