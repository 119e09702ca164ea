#!/usr/bin/env python3
"""Fixed cost of a host-timed region around chained graph replays (the bench.py contract: sync,
perf_counter, run(n), sync): median host µs vs HIP-event µs for several n, at B=256, so the gap
between short and long timed runs can be split into per-step time and per-region overhead."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc.engine.fused import FusedCifarEngine  # noqa: E402


def main():
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g)
    eng = FusedCifarEngine(256, data, labels, device="cuda", lr=1e-4)
    eng.step()
    eng.capture(32)
    ns = [1, 2, 4, 16, 20, 32, 64]
    eng.add_chain(20)
    for k in sorted(eng.chains):
        eng.run(k)
    torch.cuda.synchronize()
    out = {}
    for n in ns:
        host, ev = [], []
        for _ in range(15):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a.record()
            eng.run(n)
            b.record()
            torch.cuda.synchronize()
            host.append((time.perf_counter() - t0) * 1e6)
            ev.append(a.elapsed_time(b) * 1e3)
        h, e = statistics.median(host), statistics.median(ev)
        out[n] = {"host_us": round(h, 1), "event_us": round(e, 1), "host_per_step": round(h / n, 2),
                  "event_per_step": round(e / n, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
