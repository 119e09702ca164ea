#!/usr/bin/env python3
"""Isolation timings of the fc GEMM problems of the fused CNN step (grouped-GEMM kernel, cnn_gemm.hip):
each configuration launched back to back (HIP events, mean us per launch, the ~1.5 us dependent-launch
boundary included), so problem shapes / splits / tile orders can be compared without the step around
them.  usage: python tools/gemm_probe.py [--batch 256] [--iters 300]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc.engine.fused import FusedCifarEngine, _gemm_params, FC1_NUMEL  # noqa: E402


def timeit(fn, iters, reps=5):
    """us per launch of ``fn`` replayed from a HIP graph of ``iters`` back-to-back launches (device
    time: eager back-to-back launches are host-bound at ~5.6 us each); min over ``reps`` replays."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(gr, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    gr.replay()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        gr.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1000.0 / iters)
    return round(best, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=100)
    a = ap.parse_args()
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (4096, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (4096,), dtype=torch.int32, generator=g)
    eng = FusedCifarEngine(a.batch, data, labels, device="cuda", lr=1e-4)
    eng.step()
    torch.cuda.synchronize()
    B = eng.B
    o = eng.ops
    res = {}

    def run(name, f, sgd=False):
        sched = [eng.lr0, eng.decay, eng.decay_steps, 1.0, 0.0, 1.0]
        if sgd:
            fn = lambda: o.gemm_grouped(f["A"], f["B"], f["C"], f["bias"], f["params"], eng.step_t, eng.fc1n, sched)
        else:
            fn = lambda: o.gemm_grouped(f["A"], f["B"], f["C"], f["bias"], f["params"], eng.step_t)
        res[name] = timeit(fn, a.iters)

    # the null kernel: one 64x64 tile, K = 32 (launch + boundary floor)
    tiny = torch.zeros(64, 64, dtype=torch.bfloat16, device="cuda")
    tout = torch.zeros(64, 64, dtype=torch.float32, device="cuda")
    run("null_1tile", dict(A=[tiny], B=[tiny], C=[tout], bias=[None],
                           params=_gemm_params(64, 64, 32, 64, 1, 64, 1, 64, 0)))
    big = torch.zeros(max(1, 256 * 8), 64, 64, dtype=torch.float32, device="cuda")
    # fc1 forward at several splits
    for s in (1, 2, 4, 8, 9, 16):
        part = torch.zeros(s, B, 384, dtype=torch.float32, device="cuda")
        f = dict(A=[eng.p2.view(B, 2304)], B=[eng.fc1n], C=[part], bias=[None],
                 params=_gemm_params(B, 384, 2304, 2304, 1, 384, 0, 384, 2, s, b_par=FC1_NUMEL))
        run(f"fc1_fwd_split{s}", f)
    fb = eng._fc_bwd
    for i, nm in enumerate(["dp2", "dW1", "dW2", "dW3", "db1", "db2", "db3"]):
        f = {k: fb[k][i:i + 1] for k in ("A", "B", "C", "bias")}
        f["params"] = fb["params"][14 * i:14 * i + 14]
        run(f"bwd_{nm}", f)
    run("bwd_all7", fb)
    run("bwd_all7_sgd", eng._fc_bwd_sgd, sgd=True)
    dw = eng._fc_bwd_sgd
    f = {k: dw[k][1:2] for k in ("A", "B", "C", "bias")}
    f["params"] = dw["params"][14:28]
    run("bwd_dW1_sgd", f, sgd=True)
    # the head alone
    p = eng.pv
    res["head"] = timeit(lambda: o.head(eng.h1part, p["full_bias_1"], eng.fc2t, p["full_bias_2"], eng.fc3t,
                                        p["full_bias_3"], eng.fc3d, eng.fc2n, eng.labels, eng.bidx, None, 1,
                                        1.0 / eng.Bv, eng.relu_logits, True, eng.h1, eng.h2, eng.dl, eng.dh1,
                                        eng.dh2, eng.loss_part, eng.correct_part, None, eng.Bv, eng.step_t,
                                        eng.step_sgd), a.iters)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
