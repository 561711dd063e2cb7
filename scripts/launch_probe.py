"""When does hipLaunchKernel take its slow (~56 us) path?  Times each launch of
a tiny kernel from Python (perf_counter_ns around the call) while the GPU is
busy (a spin kernel ahead in the queue) vs idle, on one stream and alternating
two streams with cross-stream waits.  Prints the launch-time distribution and
the launch index at which slow launches start (a queue-depth cap shows as a
threshold)."""
import statistics
import time

import torch


def probe(tag, n, busy, two_streams=False, sync_each=False, prio=0):
    s1 = torch.cuda.Stream(priority=prio)
    s2 = torch.cuda.Stream()
    x = torch.zeros(1024, device="cuda")
    y = torch.zeros(1024, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        if busy:
            torch.cuda._sleep(int(2e9))  # ~1 s spin ahead of every launch below
        ts = []
        for i in range(n):
            if sync_each:
                torch.cuda.synchronize()
            if two_streams and i % 2:
                s2.wait_stream(s1)
                with torch.cuda.stream(s2):
                    t0 = time.perf_counter_ns()
                    y.add_(1.0)
                    ts.append(time.perf_counter_ns() - t0)
                s1.wait_stream(s2)
            else:
                t0 = time.perf_counter_ns()
                x.add_(1.0)
                ts.append(time.perf_counter_ns() - t0)
    torch.cuda.synchronize()
    us = [t / 1e3 for t in ts]
    slow = [i for i, u in enumerate(us) if u > 40]
    print(f"{tag:28s} n={n} median {statistics.median(us):6.1f} mean {sum(us) / n:6.1f} us  slow(>40us) "
          f"{len(slow):4d}  first slow at {slow[0] if slow else None}  p90 {sorted(us)[int(0.9 * n)]:6.1f}", flush=True)


def main():
    torch.ones(1, device="cuda").add_(1)
    torch.cuda.synchronize()
    probe("idle, sync each", 200, busy=False, sync_each=True)
    probe("idle, back-to-back", 400, busy=False)
    probe("busy, one stream", 400, busy=True)
    probe("busy, one stream (again)", 2000, busy=True)
    probe("busy, two streams + waits", 400, busy=True, two_streams=True)
    probe("idle, two streams + waits", 400, busy=False, two_streams=True)
    probe("busy, high-prio stream", 400, busy=True, prio=-1)
    probe("busy, high-prio + waits", 400, busy=True, two_streams=True, prio=-1)
    probe("idle, high-prio + waits", 400, busy=False, two_streams=True, prio=-1)


if __name__ == "__main__":
    main()
