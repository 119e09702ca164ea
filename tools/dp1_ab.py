#!/usr/bin/env python3
"""Time the data-parallel step on ONE GPU against the single-GPU step:
   python tools/dp1_ab.py [--batch 256] [--steps 300] [--rounds 2]
Variants, each a fresh engine, graph-captured, 256 settle steps, then --steps timed (interleaved
rounds, min per variant):
  single      the single-GPU step (wgrad launch applies the SGD)
  xgmi_sgd    dp_force on a one-rank xGMI context: wgrad reduce mode | exchange kernel with the SGD
              in its epilogue (k_xgmi_allreduce_sgd) -- the r5 DP step
  xgmi_ar     the same exchange without the epilogue + the SGD launch (r4's xGMI DP step)
  rccl        dp_force on a 1-rank nccl group: captured RCCL all-reduce + SGD launch
  rccl_ov     the same, overlap schedule (fc all-reduce on a comm stream beside the wgrad launch, conv
              SGD on the main stream, fc SGD beside the next forward)
  xgmi_ov     the overlap schedule over the one-rank xGMI context
--wire bf16: the gradient crosses as bf16 (bench.py's default wire)
Prints one JSON line per measurement and a summary line."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc.cli import free_port  # noqa: E402
from dmlc.engine.fused import FusedCifarEngine  # noqa: E402


def make(name, B, data, labels, wire="fp32"):
    kw = dict(device="cuda:0", lr=1e-4, relu_logits=False)
    if name == "single":
        return FusedCifarEngine(B, data, labels, **kw)
    sched = "overlap" if name.endswith("_ov") else "serial"
    if name.startswith("rccl"):
        return FusedCifarEngine(B, data, labels, **kw, dp_force=True, dp_schedule=sched, allreduce="rccl",
                                comm_dtype=wire)
    return FusedCifarEngine(B, data, labels, **kw, dp_force=True, dp_schedule=sched, allreduce="xgmi",
                            variant={"comm_sgd": name == "xgmi_sgd"}, comm_dtype=wire)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variants", default="single,xgmi_sgd,xgmi_ar,rccl")
    ap.add_argument("--wire", choices=["fp32", "bf16"], default="fp32")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g)
    names = a.variants.split(",")
    best = {}
    for r in range(a.rounds):
        for name in (names if r % 2 == 0 else names[::-1]):
            eng = make(name, a.batch, data, labels, a.wire)
            eng.step()
            eng.capture(steps_per_graph=32)
            eng.run(256)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(a.steps)
            torch.cuda.synchronize()
            us = 1e6 * (time.perf_counter() - t0) / a.steps
            eng.check_comm() if eng.dp else eng.check_barriers()
            assert torch.isfinite(eng.master).all()
            best[name] = min(best.get(name, 1e30), us)
            print(json.dumps({"variant": name, "round": r, "us_per_step": round(us, 2), "dp": eng.dp,
                              "comm": eng.comm_info, "comm_sgd": getattr(eng, "comm_sgd", False)}), flush=True)
            del eng
            torch.cuda.empty_cache()
    print(json.dumps({"batch": a.batch, "wire": a.wire, "steps": a.steps, "min_us_per_step": {k: round(v, 2) for k, v in best.items()},
                      "delta_vs_single_us": {k: round(v - best["single"], 2) for k, v in best.items()}
                      if "single" in best else {}}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
