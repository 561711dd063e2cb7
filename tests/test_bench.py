"""bench.py output contract (CPU dry runs; the real numbers come from the GPU box).

One rank, then two ranks under torch.distributed.run over gloo: rank 0 prints
exactly one JSON line with the driver's keys, whole-job throughput and the
dp degree in the config.
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


def _run(cmd, timeout=600):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return _json_lines(r.stdout)


def test_bench_contract_one_rank_cpu():
    (line,) = _run([sys.executable, "bench.py", "--cpu", "--tiny", "--steps", "2", "--warmup", "1",
                    "--batch", "8", "--image", "32"])
    assert KEYS <= set(line)
    assert line["n_gpus"] == 1 and line["steps"] == 2 and line["warmup"] == 1
    assert line["higher_is_better"] is True and line["scaling"] == "weak"
    assert line["config"]["parallelism"] == "dp1" and line["config"]["global_batch"] == 8
    assert line["value"] > 0
    assert abs(line["value"] - 8 * 1000.0 / line["ms_per_step"]) / line["value"] < 0.01


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
