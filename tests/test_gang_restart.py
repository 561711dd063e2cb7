"""Gang-wide teardown and respawn for collective jobs (failure
detection).

The reference restarts only the failed pod of an ExitCode replica
(``pkg/job_controller/pod.go:281-307``).  Ranks of a DP job share one
communicator, so here a retryable failure of one rank deletes and recreates
the whole gang; the replacements start only after the old rank processes are
gone, and every rank resumes from the job's checkpoint.  A survivor whose
collective breaks because its peer died exits 138 (retryable), never 1.
"""
import json
import os
import sys
import time

from kubedl_amd.engine.manager import Manager, ManagerOptions
from kubedl_amd.parallel import dist as kdist

PY = sys.executable


def _rank_ctr(env, steps=3, warmup=2):
    return {"name": "pytorch", "image": "kubedl-amd/none", "env": env,
            "command": [PY, "-m", "kubedl_amd.workers.resnet50", "--tiny", "--cpu", "--steps", str(steps),
                        "--warmup", str(warmup), "--batch", "2", "--image", "32"],
            "resources": {"limits": {"cpu": "1"}}}


def test_gang_restart_two_rank_job_resumes(tmp_path):
    os.environ["KDL_RESTART_BACKOFF_BASE"] = "0.05"
    m = Manager(ManagerOptions(home=str(tmp_path / "home"), gpus=8)).start()
    try:
        ck = tmp_path / "ckpt"
        env = [{"name": "KDL_CKPT_DIR", "value": str(ck)}, {"name": "KDL_CKPT_EVERY", "value": "1"},
               {"name": "KDL_FAULT", "value": "1:2:137"}, {"name": "KDL_PG_TIMEOUT_S", "value": "300"}]
        spec = lambda: {"replicas": 1, "restartPolicy": "ExitCode",  # noqa: E731
                        "template": {"spec": {"containers": [_rank_ctr(env)]}}}
        job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
               "metadata": {"name": "gr", "namespace": "default"},
               "spec": {"pytorchReplicaSpecs": {"Master": spec(), "Worker": spec()}}}
        t0 = time.time()
        m.apply(job)
        uids0 = {}
        t_end = time.time() + 60
        while len(uids0) < 2 and time.time() < t_end:
            for p in m.store.list("Pod"):
                uids0.setdefault(p["metadata"]["name"], p["metadata"]["uid"])
            time.sleep(0.02)
        done = m.wait_for_condition("PyTorchJob", "default", "gr", ["Succeeded", "Failed"], timeout=150)
        wall = time.time() - t0
        conds = [x["type"] for x in done["status"]["conditions"] if x["status"] == "True"]
        assert "Succeeded" in conds, done["status"]
        assert wall < 120, wall  # far below the 300 s process-group timeout: nobody hung in a collective
        reasons = [e["reason"] for e in m.store.list("Event")]
        assert "GangRestart" in reasons and "JobRestarting" in reasons
        # both ranks were recreated (new pod objects), not only the one that died
        uids1 = {p["metadata"]["name"]: p["metadata"]["uid"] for p in m.store.list("Pod")}
        assert set(uids1) == {"gr-master-0", "gr-worker-0"}
        assert all(uids1[n] != uids0[n] for n in uids1), (uids0, uids1)
        # resumed from the step-3 checkpoint written before the fault, ran to 5
        assert json.load(open(ck / "latest.json"))["step"] == 5
        assert m.metrics.registry.get_sample_value("kubedl_jobs_restarted", {"kind": "pytorchjob"}) == 1
    finally:
        m.stop()
        os.environ.pop("KDL_RESTART_BACKOFF_BASE", None)


def test_comm_failure_classification():
    assert kdist.is_comm_failure(RuntimeError("[gloo/transport/tcp/pair.cc:547] Connection closed by peer [127.0.0.1]:1"))
    assert kdist.is_comm_failure(RuntimeError("NCCL error in: ProcessGroupNCCL.cpp, unhandled system error"))

    class P2PError(RuntimeError):
        pass
    assert kdist.is_comm_failure(P2PError("peer did not arrive"))
    assert not kdist.is_comm_failure(ValueError("bad shape"))
    assert not kdist.is_comm_failure(RuntimeError("CUDA out of memory"))
    # deterministic errors fail permanently instead of looping through gang restarts
    assert not kdist.is_comm_failure(RuntimeError("NCCL error in: ProcessGroupNCCL.cpp:1, invalid usage"))
    assert not kdist.is_comm_failure(RuntimeError("NCCL error: invalid argument"))
    assert not kdist.is_comm_failure(RuntimeError("Default process group has not been initialized"))
    assert not kdist.is_comm_failure(RuntimeError("user data loader timed out"))
    assert not kdist.is_comm_failure(RuntimeError("process group bucket size mismatch"))
    assert kdist.is_comm_failure(RuntimeError("[gloo/transport/tcp/unbound_buffer.cc:81] Timed out waiting 30000ms"
                                              " for recv operation to complete (gloo)"))
    assert kdist.is_comm_failure(ConnectionResetError("Connection reset by peer"))
    net = getattr(__import__("torch").distributed, "DistNetworkError", None)
    if net is not None:
        assert kdist.is_comm_failure(net("store went away"))
    # rendezvous timeout: a peer died before joining the store
    import torch.distributed as tdist
    assert kdist.is_comm_failure(tdist.DistStoreError("Timed out after 601 seconds waiting for clients. 1/2 clients"
                                                      " joined."))
    assert kdist.is_comm_failure(RuntimeError("Socket Timeout: wait timed out on the store for key rank1"))
    assert kdist.COMM_FAILURE_EXIT == 138
    from kubedl_amd.api import common as c
    assert c.is_retryable_exit_code(kdist.COMM_FAILURE_EXIT)


def test_rendezvous_timeout_exits_retryable():
    """a rank whose peer never reaches the rendezvous (rank 0's TCP
    store times out waiting for clients) exits 138 -- retryable, so the job
    restarts its gang instead of failing permanently."""
    import subprocess
    import sys
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2", RANK="0",
               KDL_PG_TIMEOUT_S="2")
    r = subprocess.run([sys.executable, "-c", "import sys\nfrom kubedl_amd.parallel import dist as kd\n"
                        "sys.exit(kd.run_rank(lambda: kd.init_from_env('cpu') and 0))"],
                       env=env, capture_output=True, text=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == kdist.COMM_FAILURE_EXIT, r.stderr[-2000:]
