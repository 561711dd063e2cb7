"""TFJob worker stand-in: the plumbing half of ``example/tf/tf_job_mnist.yaml``.

TensorFlow is not part of the MI355X stack here (no TF in the image; the
north star keeps TFJob as a CPU plumbing config).  This worker does what a
TF server does with ``TF_CONFIG`` before training:

1. parses ``TF_CONFIG`` (``{"cluster": {...}, "task": {"type", "index"},
   "environment": "cloud"}``, as rendered by the TF controller and resolved to
   ``127.0.0.1:<hostPort>`` by the runtime);
2. binds its own cluster address (so the endpoint map is real);
3. waits until every other non-evaluator task in the cluster accepts TCP
   connections (the gRPC channel warm-up a ``tf.distribute`` server does);
4. Ready, then a few steps of a tiny model on CPU (``--steps``);
   PS tasks serve until their socket is told to stop or the pod is deleted
   (the reference's PS never exits on its own either);
5. the chief (or worker 0) exits 0 -> the job Succeeds per TF status rules.

Args accepted for compatibility with the example: ``--log_dir``,
``--learning_rate``, ``--batch_size`` (ignored beyond logging).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import threading
import time

from kubedl_amd.workers import common


def _serve(sock: socket.socket, stop: threading.Event) -> None:
    sock.settimeout(0.2)
    while not stop.is_set():
        try:
            conn, _ = sock.accept()
        except socket.timeout:
            continue
        except OSError:
            return
        try:
            data = conn.recv(64)
            if data.startswith(b"STOP"):
                stop.set()
            conn.sendall(b"OK")
        except OSError:
            pass
        finally:
            conn.close()


def _wait_peer(addr: str, timeout: float) -> bool:
    host, port = addr.rsplit(":", 1)
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            with socket.create_connection((host, int(port)), timeout=1.0) as s:
                s.sendall(b"PING")
                s.recv(8)
            return True
        except OSError:
            time.sleep(0.05)
    return False


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--log_dir", default="")
    ap.add_argument("--learning_rate", type=float, default=0.01)
    ap.add_argument("--batch_size", type=int, default=150)
    ap.add_argument("--peer-timeout", type=float, default=120.0)
    args, _unknown = ap.parse_known_args(argv)
    cfg = json.loads(os.environ.get("TF_CONFIG") or "{}")
    cluster = cfg.get("cluster") or {}
    task = cfg.get("task") or {"type": "worker", "index": 0}
    ttype, tidx = task.get("type", "worker"), int(task.get("index", 0))
    stop = threading.Event()
    srv = None
    if cluster:
        me = cluster[ttype][tidx]
        host, port = me.rsplit(":", 1)
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        srv.bind((host, int(port)))
        srv.listen(64)
        threading.Thread(target=_serve, args=(srv, stop), daemon=True).start()
        peers = [a for t, addrs in cluster.items() for a in addrs if a != me]
        for a in peers:
            if not _wait_peer(a, args.peer_timeout):
                print(f"tf_stub: peer {a} unreachable", file=sys.stderr, flush=True)
                return 1
    common.signal_ready({"task": task})
    print(f"tf_stub: {ttype}:{tidx} up, cluster={ {k: len(v) for k, v in cluster.items()} }", flush=True)
    if ttype == "ps":
        while not stop.is_set():
            time.sleep(0.1)
        return 0
    import numpy as np
    rng = np.random.default_rng(tidx)
    w = np.zeros(784, np.float32)
    for s in range(args.steps):
        x = rng.standard_normal((args.batch_size, 784)).astype(np.float32)
        y = (x[:, 0] > 0).astype(np.float32)
        p = 1.0 / (1.0 + np.exp(-(x @ w)))
        w -= args.learning_rate * x.T @ (p - y) / args.batch_size
        common.report_progress(s + 1, final=s + 1 == args.steps)
    print(f"tf_stub: {ttype}:{tidx} done {args.steps} steps", flush=True)
    stop.set()
    if srv is not None:
        srv.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
