#!/usr/bin/env python3
"""Per-kernel timing of the fused CIFAR CNN step (each launch repeated back to back, HIP events).

  python tools/kbench.py [--batch 256] [--iters 200] [--g1 N] [--g2 N] [--fc1-split N]
                         [--wgrad-sweep G1:G2,G1:G2,...]
Prints one JSON line per kernel with the mean µs per launch, plus the whole eager step and the
graph-replayed step, so kernel changes can be A/B'd on the GPU box without rocprof.
"""
import argparse
import json
import re
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc.engine.fused import FusedCifarEngine  # noqa: E402


def timeit(fn, iters):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--g1", type=int, default=None)
    ap.add_argument("--g2", type=int, default=None)
    ap.add_argument("--fc1-split", type=int, default=None)
    ap.add_argument("--dtype", choices=["bf16", "fp8"], default="bf16")
    ap.add_argument("--wgrad-sweep", default="", help="merged weight-gradient launch at other (g1, g2) "
                    "splits, plus each body alone on g1 / 4*g2 workgroups")
    a = ap.parse_args()
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g)
    eng = FusedCifarEngine(a.batch, data, labels, device="cuda", g1=a.g1, g2=a.g2, fc1_split=a.fc1_split,
                           lr=1e-4, dtype=a.dtype)
    eng.step()
    torch.cuda.synchronize()
    o, p = eng.ops, eng.pv
    res = {}
    res["conv1_fwd"] = timeit(lambda: o.conv1_fwd(eng.data, eng.bidx, None, 1, eng.cy, eng.cx, eng.w1f,
                                                  p["conv1_bias"], eng.p1, eng.am1, None, eng.xraw), a.iters)
    res["conv2_fwd"] = timeit(lambda: o.conv2_fwd(eng.p1, eng.w2f, p["conv2_bias"], eng.p2, eng.am2), a.iters)
    if eng.fp8:
        res["conv2_fwd_fp8"] = timeit(lambda: o.conv2_fwd_fp8(eng.p1, eng.w2f8[0], p["conv2_bias"], eng.amax_x, eng.scale_w,
                                                              None, eng.p2, eng.am2), a.iters)
    res["conv12_fwd"] = timeit(lambda: o.conv12_fwd(eng.data, eng.bidx, None, 1, eng.cy, eng.cx,
                                                    eng.w1f, p["conv1_bias"], eng.p1, eng.am1, eng.w2f,
                                                    p["conv2_bias"], eng.p2, eng.am2, eng.xraw), a.iters)
    f = eng._fc1_fwd
    res["fc1_fwd_gemm"] = timeit(lambda: eng._gemm(f), a.iters)
    B = eng.B
    res["head"] = timeit(lambda: o.head(eng.h1part, p["full_bias_1"], eng.fc2t, p["full_bias_2"], eng.fc3t,
                                        p["full_bias_3"], eng.fc3d, eng.fc2n, eng.labels, eng.bidx, None,
                                        1, 1.0 / B, True, True, eng.h1, eng.h2, eng.dl, eng.dh1, eng.dh2,
                                        eng.loss_part, eng.correct_part, None), a.iters)
    res["fc_bwd_gemm"] = timeit(eng._fc_backward, a.iters)
    res["conv2_dgrad"] = timeit(lambda: o.conv2_dgrad(eng.dp2, eng.am2, eng.w2d, eng.dp1, eng.dy2), a.iters)
    if eng.fp8:
        res["conv2_dgrad_fp8"] = timeit(lambda: o.conv2_dgrad_fp8(eng.dp2, eng.am2, eng.w2f8[1], eng.scale_w, eng.dp1,
                                                                  eng.dy2), a.iters)
    res["wgrad_merged"] = timeit(lambda: o.wgrad(eng.data, eng.bidx, None, 1, eng.cy, eng.cx,
                                                 eng.dp1, eng.am1, eng.part1, eng.partb1, eng.p1, eng.dy2,
                                                 eng.part2, eng.partb2, eng.groups2, eng.xraw), a.iters)
    for pair in filter(None, a.wgrad_sweep.split(",")):
        g1, g2 = (int(v) for v in pair.split(":"))
        z = lambda *sh: torch.zeros(*sh, device=eng.device, dtype=torch.float32)
        p1, pb1, p2, pb2 = z(g1, 80, 64), z(g1, 64), z(g2, 1600, 64), z(g2, 64)
        res[f"wgrad_{g1}_{g2}"] = timeit(lambda: o.wgrad(eng.data, eng.bidx, None, 1, eng.cy, eng.cx, eng.dp1, eng.am1,
                                                         p1, pb1, eng.p1, eng.dy2, p2, pb2, g2, eng.xraw), a.iters)
    res["conv_bwd"] = timeit(eng._conv_backward, a.iters)
    res["sgd_reduce_only"] = timeit(lambda: eng._sgd(mode=1), a.iters)
    res["sgd_full"] = timeit(lambda: eng._sgd(mode=0), a.iters)
    res["step_eager"] = timeit(eng._eager_step, a.iters)
    eng.capture()
    res["step_graph"] = timeit(lambda: eng.graphs[0].replay(), a.iters)
    res["sum_kernels"] = sum(v for k, v in res.items()
                             if not k.startswith("step") and not re.match(r"wgrad_\d", k)
                             and k not in ("sgd_reduce_only", "conv_bwd")
                             and k not in (("conv1_fwd", "conv2_fwd") if eng.fused_fwd else ("conv12_fwd",)))
    cfg = dict(batch=a.batch, g1=eng.g1, g2=eng.g2, fc1_split=eng.fc1_split, dtype=a.dtype)
    print(json.dumps({"config": cfg, "us": {k: round(v, 2) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
