"""Where the GBDT cut fitting's ~0.1 s goes on a fresh process (first calls) vs
a second call: each torch op of GBDT.fit_cuts timed with a sync around it."""
import time

import torch


def timed(tag, fn, log):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    log.append((tag, (time.perf_counter() - t) * 1e3))
    return r


def once(X, log, B=256, k=65536):
    n = X.shape[0]
    idx = timed("arange+mul", lambda: (torch.arange(k, device=X.device, dtype=torch.int64) * n) // k + 3, log)
    samp = timed("gather+float", lambda: X[idx.clamp_(max=n - 1)].float(), log)
    q = timed("linspace", lambda: torch.linspace(0, 1, B + 1, device=X.device, dtype=torch.float64)[1:-1], log)
    srt = timed("transpose+sort", lambda: torch.sort(samp.T.contiguous(), dim=1)[0], log)
    pos = timed("pos", lambda: q * (srt.shape[1] - 1), log)
    lo, hi = timed("floor/ceil/long", lambda: (pos.floor().long(), pos.ceil().long()), log)
    w = timed("w", lambda: (pos - lo.double()).float(), log)
    return timed("lerp", lambda: (srt[:, lo] * (1 - w) + srt[:, hi] * w).contiguous(), log)


def main():
    X = torch.randn(2_000_000, 28).cuda()
    torch.cuda.synchronize()
    for rep in range(2):
        log = []
        t = time.perf_counter()
        once(X, log)
        print(f"call {rep}: total {(time.perf_counter() - t) * 1e3:.1f} ms: " +
              ", ".join(f"{a} {b:.1f}" for a, b in log), flush=True)


if __name__ == "__main__":
    main()
