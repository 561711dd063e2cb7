"""bench.py output contract (CPU dry runs; the real numbers come from the GPU box).

* job path (no WORLD_SIZE): bench.py is a kdl control plane that submits one
  N-rank PyTorchJob through store -> controller -> gang -> kubelet and prints
  rank 0's line plus the controller-path launch delays (N = 1, 2, 4);
* torchrun path: two ranks under torch.distributed.run over gloo;
* direct path: one in-process rank.
Every way, exactly one JSON line with the driver's keys, whole-job
throughput and the dp degree in the config.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _json_lines(out: str):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def _run(cmd, timeout=600, **env_over):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2", **env_over)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return _json_lines(r.stdout)


def test_bench_contract_one_rank_cpu():
    (line,) = _run([sys.executable, "bench.py", "--cpu", "--tiny", "--steps", "2", "--warmup", "1",
                    "--batch", "8", "--image", "32"], KDL_ZYGOTE="1")
    assert line["config"]["launcher"] == "kdl-pytorchjob"
    assert line["first_pod_launch_delay_s"] > 0 and line["all_pods_launch_delay_s"] >= line["first_pod_launch_delay_s"]
    assert KEYS <= set(line)
    assert line["n_gpus"] == 1 and line["steps"] == 2 and line["warmup"] == 1
    assert line["higher_is_better"] is True and line["scaling"] == "weak"
    assert line["config"]["parallelism"] == "dp1" and line["config"]["global_batch"] == 8
    assert line["value"] > 0
    assert abs(line["value"] - 8 * 1000.0 / line["ms_per_step"]) / line["value"] < 0.01
    # warm launch (ranks forked from the node's pre-imported
    # zygote) and the cold probe job (fresh interpreters) are both reported, and
    # the zygote's fork is the faster one; comm_init_s = the first collective
    assert line["launch"] == "warm (zygote)"
    assert line["cold_first_pod_launch_delay_s"] > 0 and line["cold_all_pods_launch_delay_s"] > 0
    assert line["first_pod_launch_delay_s"] < line["cold_first_pod_launch_delay_s"]
    assert line["comm_init_s"] >= 0


def test_bench_contract_two_ranks_cpu():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    lines = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                  "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--cpu",
                  "--tiny", "--steps", "2", "--warmup", "1", "--batch", "8", "--image", "32"])
    assert len(lines) == 1  # rank 0 only
    (line,) = lines
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    assert line["config"]["global_batch"] == 16 and line["config"]["allreduce"] == "rccl"
    assert abs(line["value"] - 16 * 1000.0 / line["ms_per_step"]) / line["value"] < 0.01
    # the DP bucket plan in the JSON (CPU: no device events, so
    # no exposed time; the GPU bench reports it)
    d = line["ddp"]
    assert d["active"] and d["world"] == 2 and d["transport"] == "rccl" and d["buckets"] >= 1
    assert abs(sum(d["bucket_mb"]) - d["grad_mb"]) < 0.05 * d["grad_mb"] + 0.01
    assert "exposed_ms_per_step" in d


import pytest  # noqa: E402


@pytest.mark.parametrize("n", [2, 4])
def test_bench_job_path_n_ranks_cpu(n):
    """--gpus N without an external launcher: one N-rank PyTorchJob through the
    control plane (the driver's scaling curve no longer depends on torchrun)."""
    (line,) = _run([sys.executable, "bench.py", "--gpus", str(n), "--cpu", "--tiny", "--steps", "2",
                    "--warmup", "1", "--batch", "8", "--image", "32"])
    assert KEYS <= set(line)
    assert line["n_gpus"] == n and line["config"]["parallelism"] == f"dp{n}"
    assert line["config"]["launcher"] == "kdl-pytorchjob" and line["ranks_ready"] == n
    assert line["config"]["global_batch"] == 8 * n
    assert line["first_pod_launch_delay_s"] is not None and line["all_pods_launch_delay_s"] is not None
    assert line["all_pods_launch_delay_s"] >= line["first_pod_launch_delay_s"] > 0
    assert line["job_wall_s"] >= line["all_pods_launch_delay_s"]
    # the communicator bootstrap runs beside the model build at
    # world N too, joined before the DDP broadcast (the trainer's first collective)
    st = line["startup"]
    assert st["comm_overlap"] is True and st["comm_joined_at"] is not None, st
    assert line["comm_init_s"] > 0


def test_bench_direct_path_cpu():
    (line,) = _run([sys.executable, "bench.py", "--direct", "--cpu", "--tiny", "--steps", "2", "--warmup", "1",
                    "--batch", "8", "--image", "32"])
    assert line["n_gpus"] == 1 and line["config"]["launcher"] == "direct"


def test_bench_job_path_fails_loudly_on_rank_failure():
    """A rank that dies makes the job Failed and bench.py exit non-zero."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2", KDL_FAULT="0:1:1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--cpu", "--tiny", "--steps", "2", "--warmup",
                        "2", "--batch", "8", "--image", "32", "--timeout", "120"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not _json_lines(r.stdout)
