"""Pre-warmed rank-process zygote: the launch-delay lever of the local runtime.

Most of a PyTorch rank's launch delay is the interpreter start plus
``import torch`` (1.5-3 s).  The zygote is a
long-lived Python process that has already imported torch, torch.distributed
and the bundled workers but has NOT touched the GPU (no HIP initialisation,
so forking it is safe and every child still chooses its own
``HIP_VISIBLE_DEVICES``).  A launch request forks a child that

1. double-forks away so the rank is re-parented to the kubelet (which is a
   PR_SET_CHILD_SUBREAPER) and is reaped/killed exactly like a directly
   spawned rank,
2. starts a new session, redirects stdio to the pod log, applies the pod's
   environment and working directory,
3. runs ``python -m <module> <args>`` in-process via ``runpy``.

Protocol: one JSON line per request on a Unix socket ``{"argv": [...],
"env": {...}, "cwd": str, "log": str}`` -> ``{"pid": int}`` or
``{"error": str}``.  Only ``-m <module>`` invocations are eligible; anything
else goes through the native spawner.
"""
from __future__ import annotations

import json
import os
import socket
import sys
import threading
import time
from typing import List, Optional

PRELOAD = ("torch", "torch.distributed", "torch.nn.functional", "kubedl_amd.workers.common",
           "kubedl_amd.parallel.dist", "kubedl_amd.ops.optim", "kubedl_amd.models.resnet",
           "kubedl_amd.workers.resnet50", "kubedl_amd.workers.resnet_bench", "kubedl_amd.workers.pytorch_dist", "kubedl_amd.workers.xdl_ctr",
           "kubedl_amd.workers.xgboost_dist", "kubedl_amd.workers.tf_stub")


def eligible(argv: List[str]) -> Optional[int]:
    """Index of the module name if argv is ``<python> [-u] -m <module> ...``."""
    if not argv or not os.path.basename(argv[0]).startswith("python"):
        return None
    i = 1
    while i < len(argv) and argv[i] in ("-u", "-B", "-O"):
        i += 1
    if i + 1 < len(argv) and argv[i] == "-m":
        return i + 1
    return None


def _child_main(req: dict, wfd: int) -> None:
    """Runs in the first fork: fork the rank, report its pid, exit (the rank is
    then an orphan re-parented to the kubelet subreaper)."""
    inter = os.getpid()
    pid = os.fork()
    if pid > 0:
        os.write(wfd, json.dumps({"pid": pid}).encode())
        os._exit(0)
    # ---- the rank process (re-parented to the kubelet subreaper)
    code = 0
    try:
        os.close(wfd)
        os.setsid()  # own session + process group: killpg(pid) reaches the whole rank tree
        # PR_SET_PDEATHSIG only after re-parenting to the kubelet subreaper:
        # armed while the short-lived intermediate is still the parent, it
        # would fire the moment the intermediate exits.
        t_end = time.time() + 2.0
        while os.getppid() == inter and time.time() < t_end:
            time.sleep(0.001)
        try:
            import ctypes
            import signal
            libc = ctypes.CDLL("libc.so.6", use_errno=True)
            libc.prctl(1, signal.SIGKILL)  # die with the kubelet
        except Exception:
            pass
        fd = os.open(req["log"], os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        os.dup2(fd, 1)
        os.dup2(fd, 2)
        os.close(fd)
        nul = os.open(os.devnull, os.O_RDONLY)
        os.dup2(nul, 0)
        os.close(nul)
        sys.stdout = os.fdopen(1, "w", buffering=1)
        sys.stderr = os.fdopen(2, "w", buffering=1)
        os.chdir(req.get("cwd") or "/")
        os.environ.clear()
        os.environ.update(req["env"])
        if os.environ.get("OMP_NUM_THREADS"):
            import torch
            torch.set_num_threads(max(1, int(os.environ["OMP_NUM_THREADS"])))
        argv = req["argv"]
        mi = eligible(argv)
        mod = argv[mi]
        sys.argv = [mod] + argv[mi + 1:]
        pp = os.environ.get("PYTHONPATH")
        if pp:
            for p in reversed(pp.split(os.pathsep)):
                if p and p not in sys.path:
                    sys.path.insert(0, p)
        import runpy
        runpy.run_module(mod, run_name="__main__", alter_sys=True)
    except SystemExit as e:
        code = e.code if isinstance(e.code, int) else (0 if e.code is None else 1)
    except BaseException:  # noqa: BLE001 - report like an uncaught exception in python
        import traceback
        traceback.print_exc()
        code = 1
    finally:
        try:
            sys.stdout.flush()
            sys.stderr.flush()
        except Exception:
            pass
        os._exit(code)


def serve(sock_path: str) -> None:
    for m in PRELOAD:
        try:
            __import__(m)
        except Exception as e:  # a missing optional worker must not kill the zygote
            print(f"zygote: preload {m} failed: {e}", file=sys.stderr, flush=True)
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    try:
        os.unlink(sock_path)
    except FileNotFoundError:
        pass
    srv.bind(sock_path)
    srv.listen(64)
    print(f"zygote: ready on {sock_path}", flush=True)
    while True:
        conn, _ = srv.accept()
        try:
            data = b""
            while not data.endswith(b"\n"):
                chunk = conn.recv(65536)
                if not chunk:
                    break
                data += chunk
            if not data.strip():
                continue
            req = json.loads(data)
            if req.get("op") == "ping":
                conn.sendall(b'{"ok": true}\n')
                continue
            r, w = os.pipe()
            pid = os.fork()
            if pid == 0:
                os.close(r)
                _child_main(req, w)
            os.close(w)
            msg = b""
            while True:
                chunk = os.read(r, 4096)
                if not chunk:
                    break
                msg += chunk
            os.close(r)
            os.waitpid(pid, 0)  # the intermediate exits right after forking the rank
            conn.sendall((msg.decode() or '{"error": "fork failed"}').encode() + b"\n")
        except Exception as e:  # keep serving
            try:
                conn.sendall(json.dumps({"error": str(e)}).encode() + b"\n")
            except OSError:
                pass
        finally:
            conn.close()


# Device libraries a rank maps on its first GPU work (librccl.so is ~340 MB,
# nearly all of it gfx code objects): the node runtime reads them once at
# start-up -- pure file IO in the kubelet process, no GPU initialisation.  The
# first communicator's 3.5 s on a fresh node (vs 0.9 s after) turned out NOT to
# be this read (prefetched, it stayed 3.4 s) but the code-object manager's disk
# cache, which the node warm-up below fills (runtime/node_warm.py,
# profiles/r04_comgr_cache.txt).
PREFETCH_LIBS = ("librccl.so", "libamdhip64.so", "libhsa-runtime64.so")


def device_library_paths() -> List[str]:
    import importlib.util
    out = []
    spec = importlib.util.find_spec("torch")
    for d in (spec.submodule_search_locations or []) if spec else []:
        for name in PREFETCH_LIBS:
            p = os.path.join(d, "lib", name)
            if os.path.exists(p):
                out.append(p)
    ext = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")
    if os.path.exists(ext):
        out.append(ext)
    return out


def prefetch_files(paths: List[str], chunk: int = 8 << 20) -> int:
    """Read every file through once (page cache); returns the bytes read."""
    n = 0
    for p in paths:
        try:
            fd = os.open(p, os.O_RDONLY)
        except OSError:
            continue
        try:
            while True:
                b = os.read(fd, chunk)
                if not b:
                    break
                n += len(b)
        finally:
            os.close(fd)
    return n


def warm_node(env: dict, timeout: float = 180.0, gpu: Optional[int] = None, procs: Optional[list] = None) -> dict:
    """Run runtime/node_warm.py in a child process (one world-1 RCCL
    communicator on GPU ``gpu`` of the node's inventory) and return its JSON
    result.  ``procs``: the live child is appended while it runs (the kubelet
    kills it when it stops)."""
    import subprocess
    t0 = time.time()
    env = dict(env or os.environ)
    if gpu is not None:
        env["HIP_VISIBLE_DEVICES"] = str(gpu)  # the warm-up's one GPU, from the inventory
    try:
        p = subprocess.Popen([sys.executable, "-m", "kubedl_amd.runtime.node_warm"], env=env,
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
        if procs is not None:
            procs.append(p)
        try:
            out, err = p.communicate(timeout=timeout)
        finally:
            if procs is not None and p in procs:
                procs.remove(p)
        lines = [ln for ln in (out or "").splitlines() if ln.startswith("{")]
        res = json.loads(lines[-1]) if lines else {"warm": False, "error": (err or "")[-300:]}
    except subprocess.TimeoutExpired as e:
        p.kill()
        p.wait()
        res = {"warm": False, "error": f"TimeoutExpired: {e}"}
    except (OSError, ValueError) as e:
        res = {"warm": False, "error": f"{type(e).__name__}: {e}"}
    res["wall_s"] = round(time.time() - t0, 3)
    if gpu is not None:
        res["gpu"] = gpu
    return res


class ZygoteClient:
    """Kubelet side: start the zygote lazily and ask it for rank processes."""

    def __init__(self, root: str, native, warm_gpu: Optional[int] = None):
        """``warm_gpu``: the inventory GPU the node warm-up may use (None: no
        warm-up -- a node without GPUs in its inventory)."""
        self.warm_gpu = warm_gpu
        self._warm_procs: list = []
        self.sock = os.path.join(root, "zygote.sock")
        self.log = os.path.join(root, "zygote.log")
        self.native = native
        self.pid: Optional[int] = None
        self._lock = threading.Lock()
        self.ready = threading.Event()
        self.prefetched = threading.Event()
        self.prefetch_s: Optional[float] = None
        self.warm: Optional[dict] = None
        self._env: dict = {}
        # held exclusively while the warm-up runs: ranks wait on it (shared)
        # before their first communicator build, after their Ready
        self.warm_lock = os.path.join(root, "node_warm.lock")
        self._warm_fd: Optional[int] = None

    def start(self, env: dict) -> None:
        with self._lock:
            if self.pid is not None:
                return
            self.native.set_child_subreaper()
            env = dict(env)
            for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
                env.pop(k, None)
            argv = [sys.executable, "-u", "-m", "kubedl_amd.runtime.zygote", self.sock]
            self.pid = self.native.spawn(argv, [f"{k}={v}" for k, v in env.items()], None, self.log, self.log)
            self._env = env
            mode = os.environ.get("KDL_NODE_WARM", "1")  # 0 off; force: without /dev/kfd too (tests)
            if mode != "0" and (mode == "force" or os.path.exists("/dev/kfd")) and self.warm_gpu is not None:
                self._hold_warm_lock()
        threading.Thread(target=self._wait_ready, daemon=True).start()
        threading.Thread(target=self._prefetch, daemon=True).start()

    def _hold_warm_lock(self) -> None:
        """Take the warm-up lock before any pod can start (synchronously in
        start()), so a rank started right after the node runtime sees it held."""
        import fcntl
        fd = os.open(self.warm_lock, os.O_RDWR | os.O_CREAT | os.O_CLOEXEC, 0o644)
        fcntl.flock(fd, fcntl.LOCK_EX)
        self._warm_fd = fd

    def _release_warm_lock(self) -> None:
        import fcntl
        fd, self._warm_fd = self._warm_fd, None
        if fd is not None:
            try:
                fcntl.flock(fd, fcntl.LOCK_UN)
            finally:
                os.close(fd)

    def _prefetch(self) -> None:
        t0 = time.time()
        try:
            prefetch_files(device_library_paths())
            self.prefetch_s = time.time() - t0
            if self._warm_fd is not None:
                self.warm = warm_node(self._env, gpu=self.warm_gpu, procs=self._warm_procs)
        finally:
            if self.prefetch_s is None:
                self.prefetch_s = time.time() - t0
            self._release_warm_lock()
            self.prefetched.set()

    def _wait_ready(self, timeout: float = 300.0) -> None:
        t_end = time.time() + timeout
        while time.time() < t_end:
            try:
                if self._call({"op": "ping"}).get("ok"):
                    self.ready.set()
                    return
            except OSError:
                time.sleep(0.05)

    def _call(self, req: dict, timeout: float = 30.0) -> dict:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.settimeout(timeout)
        try:
            s.connect(self.sock)
            s.sendall(json.dumps(req).encode() + b"\n")
            data = b""
            while not data.endswith(b"\n"):
                chunk = s.recv(65536)
                if not chunk:
                    break
                data += chunk
            return json.loads(data or b"{}")
        finally:
            s.close()

    def launch(self, argv: List[str], env: dict, cwd: str, log: str) -> Optional[int]:
        """pid of the forked rank, or None when the zygote is not (yet) usable."""
        if not self.ready.is_set():
            return None
        try:
            r = self._call({"argv": argv, "env": env, "cwd": cwd, "log": log})
        except OSError:
            return None
        return int(r["pid"]) if "pid" in r else None

    def stop(self) -> None:
        for p in list(self._warm_procs):  # a warm-up still running: it must not outlive the node runtime
            try:
                p.kill()
                p.wait(timeout=5)
            except Exception:
                pass
        self._release_warm_lock()
        if self.pid is not None:
            try:
                self.native.kill_group(self.pid, 9)
            except Exception:
                pass
            self.native.reap([self.pid])
            self.pid = None


if __name__ == "__main__":
    serve(sys.argv[1])
