#!/usr/bin/env python3
"""fp8 (BASELINE config 5) step time against the conv2 weight-gradient split g2 (image groups; the
wgrad launch runs 4*g2 conv2 blocks and g1 = 256 - 4*g2 conv1 blocks).  Same-process sweep, each
engine graph-captured, settled and timed (interleaved rounds, min per g2).
  python tools/fp8_g2_sweep.py [--batch 1024] [--g2 16,24,32] [--steps 200]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc.engine.fused import FusedCifarEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--g2", default="16,24,32")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--dtype", default="fp8")
    a = ap.parse_args()
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g)
    g2s = [int(x) for x in a.g2.split(",")]
    best = {}
    for r in range(a.rounds):
        for g2 in (g2s if r % 2 == 0 else g2s[::-1]):
            eng = FusedCifarEngine(a.batch, data, labels, device="cuda", lr=1e-4, relu_logits=False, dtype=a.dtype,
                                   g2=g2)
            eng.step()
            eng.capture(steps_per_graph=32)
            eng.run(256)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(a.steps)
            torch.cuda.synchronize()
            us = 1e6 * (time.perf_counter() - t0) / a.steps
            assert torch.isfinite(eng.master).all()
            best[g2] = min(best.get(g2, 1e30), us)
            print(json.dumps({"g2": g2, "g1": eng.g1, "round": r, "us_per_step": round(us, 2),
                              "images_per_s": round(a.batch / us * 1e6)}), flush=True)
            del eng
            torch.cuda.empty_cache()
    print(json.dumps({"batch": a.batch, "dtype": a.dtype, "min_us_per_step": {str(k): round(v, 2) for k, v in best.items()}}))


if __name__ == "__main__":
    main()
