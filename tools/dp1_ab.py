#!/usr/bin/env python3
"""Time the data-parallel step (dp_force, 1-rank nccl group, graph-captured all-reduce) on one GPU:
   python tools/dp1_ab.py [--batch 256] [--steps 300] [--schedule serial]
Prints one JSON line {us_per_step, wgrad_reduce, ...}.  DMLC_WGRAD_SGD=0 selects the reduce-only SGD
launch instead of the in-wgrad-launch reduction (A/B)."""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--schedule", default="serial")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g)
    eng = FusedCifarEngine(a.batch, data, labels, device="cuda:0", lr=1e-4, dp_force=True,
                           dp_schedule=a.schedule, allreduce="rccl")
    eng.step()
    eng.capture(steps_per_graph=32)
    eng.run(256)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run(a.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    eng.check_barriers()
    print(json.dumps({"batch": a.batch, "schedule": a.schedule, "us_per_step": 1e6 * dt / a.steps,
                      "wgrad_reduce": eng.wgrad_reduce, "backend": eng.comm_info.get("backend")}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
