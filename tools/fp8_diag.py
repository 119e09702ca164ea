#!/usr/bin/env python3
"""fp8 path diagnostics: loss / scales over a bench-like run, and the conv1 forward's cost with and
without the activation-amax epilogue, for the fp8 conv2 dgrad on and off (engine variant fp8_dgrad)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc.engine.fused import FusedCifarEngine  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / iters


def main():
    B = int(os.environ.get("B", "1024"))
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g)
    for dg in (True, False):
        eng = FusedCifarEngine(B, data, labels, device="cuda", dtype="fp8", variant={"fp8_dgrad": dg})
        eng.step()
        eng.capture()
        eng.run(60)
        torch.cuda.synchronize()
        st = [eng.read_stats(k) for k in (1, 10, 30, 61)]
        o, p = eng.ops, eng.pv
        t_amax = timeit(lambda: o.conv1_fwd(eng.data, eng.bidx, None, 1, eng.cy, eng.cx, eng.w1f, p["conv1_bias"],
                                            eng.p1, eng.am1, eng.amax_x, eng.xraw))
        t_none = timeit(lambda: o.conv1_fwd(eng.data, eng.bidx, None, 1, eng.cy, eng.cx, eng.w1f, p["conv1_bias"],
                                            eng.p1, eng.am1, None, eng.xraw))
        p1 = eng.p1.float()
        print(json.dumps({"fp8_dgrad": dg, "loss": [s["loss"] for s in st], "amax_x": float(eng.amax_x.max()),
                          "scale_w": eng.scale_w.tolist(), "p1_nonzero": float((p1 != 0).float().mean()),
                          "p1_finite": bool(torch.isfinite(p1).all()),
                          "conv1_fwd_amax_us": round(t_amax, 2), "conv1_fwd_us": round(t_none, 2)}), flush=True)
        del eng


if __name__ == "__main__":
    main()
