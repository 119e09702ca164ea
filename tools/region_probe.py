#!/usr/bin/env python3
"""Fixed cost of a timed region: how long do k chained training steps take when bracketed exactly as
bench.py brackets them (synchronize -> t0 -> one graph replay of k steps -> synchronize -> t1)?
A linear fit over k separates the per-step time (slope) from the per-region overhead (intercept:
graph launch submission, the first kernel's dispatch after an idle queue, the final sync).

  python tools/region_probe.py [--batch 256] [--reps 5] [--poll] [--spin]

--poll: busy-poll an event recorded after the replay (event.query()) before the closing synchronize
        -- does the region's fixed cost sit in the host's wake-up from a blocking wait?
--events: HIP events around the replay (GPU-side time of the k steps) + the replay call's host time
--spin: hipSetDeviceFlags(hipDeviceScheduleSpin) on torch's HIP runtime before the device is
        initialised (the runtime then spins instead of sleeping in every synchronize)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc.engine.fused import FusedCifarEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--poll", action="store_true")
    ap.add_argument("--spin", action="store_true")
    ap.add_argument("--events", action="store_true", help="also: GPU time between events recorded around the "
                    "replay, and the host time of the replay call itself")
    a = ap.parse_args()
    if a.spin:
        import ctypes
        lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        rc = lib.hipSetDeviceFlags(ctypes.c_uint(1))      # hipDeviceScheduleSpin
        print(f"hipSetDeviceFlags(spin) -> {rc}", file=sys.stderr)
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g).cuda()
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g).cuda()
    eng = FusedCifarEngine(a.batch, data, labels, device="cuda", seed=0, lr=1e-4, relu_logits=False)
    for _ in range(3):
        eng.step()
    eng.capture(32)
    ks = [1, 2, 4, 8, 16, 20, 32, 40, 64]
    for k in ks:
        eng.add_chain(k)
    for k in sorted(eng.chains):
        eng.run(k)
    eng.run(256)
    torch.cuda.synchronize()
    res, host_us, ev_us = {}, {}, {}
    for k in ks:
        ts = []
        for _ in range(a.reps):
            eng.run(64)                          # busy before, as after bench.py's warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if a.events:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
            th = time.perf_counter()
            eng.chains[k].replay()
            host_us.setdefault(k, []).append((time.perf_counter() - th) * 1e6)
            eng.host_step += k
            if a.events:
                e1.record()
            if a.poll:
                ev = torch.cuda.Event()
                ev.record()
                while not ev.query():
                    pass
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e6)
            if a.events:
                ev_us.setdefault(k, []).append(e0.elapsed_time(e1) * 1000.0)
        res[k] = min(ts)
    x = np.array(ks, dtype=float)
    y = np.array([res[k] for k in ks])
    slope, icpt = np.polyfit(x, y, 1)
    # the empty region: sync -> t0 -> sync
    torch.cuda.synchronize()
    e = []
    for _ in range(20):
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        e.append((time.perf_counter() - t0) * 1e6)
    print(json.dumps({"mode": "spin" if a.spin else "poll" if a.poll else "sync", "us_per_region": {str(k): round(v, 1) for k, v in res.items()},
                      "fit_us_per_step": round(float(slope), 2), "fit_region_overhead_us": round(float(icpt), 1),
                      "empty_sync_us": round(float(min(e)), 1),
                      "replay_call_us": {str(k): round(min(v), 1) for k, v in host_us.items()},
                      "event_us": {str(k): round(min(v), 1) for k, v in ev_us.items()}}))


if __name__ == "__main__":
    main()
