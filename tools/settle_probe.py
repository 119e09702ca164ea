#!/usr/bin/env python3
"""Why does the bench's step time depend on how many steps ran before the timed region?
(profiles/r3_settle_steps_ab.txt: 20 timed steps after 1,024 settle steps measured 2.76-2.90 M
img/s, after 256 or 4,096 steps 3.12 M.)  This runs the bench's exact configuration (synthetic
uint8 data, random labels, lr 0.1, B=256, 32-step graph chains) for --steps steps in windows of
--window steps and prints, per window: us/step (HIP events around the replays), the training loss
and accuracy from the device stats ring, the fraction of exactly-zero pooled conv2 activations
(p2) and conv1 activations (p1), max |w| and whether every weight is finite -- i.e. whether the
timing follows the network's state (dead ReLUs make MFMA operands zero, and the chip then holds a
higher clock: MI355X_MICROARCH.md, DVFS give-back).

  python tools/settle_probe.py [--steps 4096] [--window 128] [--lr 0.1]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc.engine.fused import FusedCifarEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4096)
    ap.add_argument("--window", type=int, default=128)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--learnable", action="store_true", help="learnable synthetic labels instead of random")
    ap.add_argument("--no-relu-logits", action="store_true", help="no ReLU on the logits (reference D4 off)")
    a = ap.parse_args()
    g = torch.Generator().manual_seed(0)
    if a.learnable:
        from dmlc.data import synthetic
        data, labels = synthetic(50000, seed=0, learnable=True)
    else:
        data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g)
        labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g)
    eng = FusedCifarEngine(a.batch, data.cuda(), labels.cuda(), device="cuda", seed=0, lr=a.lr,
                           relu_logits=not a.no_relu_logits)
    for _ in range(3):
        eng.step()
    eng.capture(32)
    eng.run(32)
    torch.cuda.synchronize()
    done = eng.host_step
    while done < a.steps:
        n = min(a.window, a.steps - done)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.run(n)
        e1.record()
        torch.cuda.synchronize()
        done = eng.host_step
        st = eng.read_stats(done)
        rec = {"step": done, "us_per_step": round(e0.elapsed_time(e1) * 1000.0 / n, 2),
               "loss": st["loss"], "acc": st["accuracy"], "lr": st["lr"],
               "p2_zero": round(float((eng.p2 == 0).float().mean()), 4),
               "p1_zero": round(float((eng.p1 == 0).float().mean()), 4),
               "dl_nonzero": round(float((eng.dl[:, :10] != 0).float().mean()), 4),
               "dp2_nonzero": round(float((eng.dp2 != 0).float().mean()), 4),
               "dy2_nonzero": round(float((eng.dy2 != 0).float().mean()), 4),
               "w_absmax": float(eng.master.abs().max()), "finite": bool(torch.isfinite(eng.master).all())}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
