"""Is the ResNet-50 step's host issue throttled by GPU progress?

Builds the bench's trainer (batch 256, 224 px, world 1 without a process
group), warms up, then queues a ~60 ms spin kernel on the step's compute
stream and times the host issue of the next steps.  Unthrottled, the host
issues a whole step (hundreds of launches) during the spin; throttled by a cap
on outstanding work, it blocks once the cap is reached and its issue time
tracks the GPU.  Also prints the per-call issue time of every binding call of
one step (monkeypatched _C functions) to locate the slow launches."""
import collections
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubedl_amd.parallel.dist import DistInfo  # noqa: E402
from kubedl_amd.workers.resnet50 import ResNetTrainer  # noqa: E402


def main():
    torch.cuda.set_device(0)
    info = DistInfo(0, 1, 0, torch.device("cuda", 0), "nccl")
    tr = ResNetTrainer(info, batch=256, image=224, bn_backend="auto", engine="fused")
    for _ in range(6):
        tr.step()
    torch.cuda.synchronize()
    s = tr.stream
    for spin in (0, int(1.2e8)):
        torch.cuda.synchronize()
        if spin:
            with torch.cuda.stream(s):
                torch.cuda._sleep(spin)
        hs = []
        for _ in range(3):
            t0 = time.perf_counter()
            tr.step()
            hs.append((time.perf_counter() - t0) * 1e3)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(f"spin={spin:>10d}: host issue per step {[round(h, 2) for h in hs]} ms; then waited "
              f"{(time.perf_counter() - t1) * 1e3:.1f} ms for the GPU", flush=True)
    # a long unsynchronised run, as the bench's timed loop: host issue per step,
    # allocator activity (segments, retries) over it
    torch.cuda.synchronize()
    m0 = torch.cuda.memory_stats()
    hs = []
    t0 = time.perf_counter()
    for _ in range(30):
        th = time.perf_counter()
        tr.step()
        hs.append((time.perf_counter() - th) * 1e3)
    issued = time.perf_counter()
    torch.cuda.synchronize()
    m1 = torch.cuda.memory_stats()
    print(f"30 steps: host per step {[round(h, 1) for h in hs]}", flush=True)
    print(f"  issue {(issued - t0) * 1e3:.1f} ms, wall {(time.perf_counter() - t0) * 1e3:.1f} ms; "
          + ", ".join(f"{k} {m1.get(k, 0) - m0.get(k, 0)}" for k in (
              "num_alloc_retries", "segment.all.allocated", "segment.all.freed", "num_sync_all_streams",
              "num_device_alloc", "num_device_free")), flush=True)
    # per binding call host time over one step (GPU busy ahead with a spin)
    import kubedl_amd.ops._ext as E
    ext = E.load()
    stats = collections.defaultdict(list)
    orig = {}
    for name in dir(ext):
        f = getattr(ext, name)
        if callable(f) and not name.startswith("_"):
            orig[name] = f

            def wrap(*a, __f=f, __n=name, **k):
                t0 = time.perf_counter_ns()
                r = __f(*a, **k)
                stats[__n].append((time.perf_counter_ns() - t0) / 1e3)
                return r
            try:
                setattr(ext, name, wrap)
            except (AttributeError, TypeError):
                pass
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        torch.cuda._sleep(int(1.2e8))
    t0 = time.perf_counter()
    tr.step()
    h = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    tot = sum(sum(v) for v in stats.values()) / 1e3
    print(f"wrapped step: host {h:.2f} ms, {sum(len(v) for v in stats.values())} binding calls = {tot:.2f} ms")
    for n, v in sorted(stats.items(), key=lambda kv: -sum(kv[1]))[:25]:
        v.sort()
        print(f"  {n:28s} n={len(v):3d} total {sum(v) / 1e3:6.2f} ms  median {v[len(v) // 2]:6.1f} us  max {v[-1]:7.1f} us")


if __name__ == "__main__":
    main()
