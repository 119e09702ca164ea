#!/usr/bin/env python3
"""Per-kernel timing of the fused ResNet-20 step (each launch repeated back to back, HIP events).

  python tools/rn_kbench.py [--batch 256] [--iters 100]
One JSON line: µs per launch for every layer's fwd / dgrad / wgrad, head, sgd, the eager step and
the graph-replayed step.  Kernel variants: build with DMLC_VARIANT="name:-DFLAG" and run with the
same env (see _build.py)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc.engine.fused_resnet import FusedResNetEngine, LAYERS, _block_sc_mode  # noqa: E402


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
    return round(a.elapsed_time(b) * 1000.0 / iters, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=100)
    a = ap.parse_args()
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g)
    eng = FusedResNetEngine(a.batch, data, labels, device="cuda", lr=1e-3)
    eng.step()
    torch.cuda.synchronize()
    o = eng.ops
    res = {"variant": os.environ.get("DMLC_VARIANT", ""), "batch": a.batch}
    for l, (_, ci, co, h, s) in enumerate(LAYERS):
        if l == 0:
            f = lambda: o.rn_fwd(ci, co, h, s, eng.data, eng.order_desc, eng.step_t, eng.period, 0, 0, None, None, None,
                                 None, None, 0, None, eng.wf[0], eng.z[0], eng.stat[0])
        else:
            p = l - 1
            scm, scs = (_block_sc_mode(p), eng.a[p - 2]) if (p >= 2 and p % 2 == 0) else (0, None)
            f = (lambda l=l, p=p, ci=ci, co=co, h=h, s=s, scm=scm, scs=scs:
                 o.rn_fwd(ci, co, h, s, None, None, None, 1, 0, 0, eng.z[p], eng.stat[p], eng.gamma[p], eng.beta[p],
                          scs, scm, eng.a[p], eng.wf[l], eng.z[l], eng.stat[l]))
        res[f"fwd{l}"] = timeit(f, a.iters)
        res[f"wgrad{l}"] = timeit(lambda l=l: eng._wgrad(l), a.iters)
        if l > 0:
            p = l - 1
            scm, gsc = (_block_sc_mode(l + 1), eng.gy[l + 1]) if l % 2 == 1 else (0, None)
            res[f"dgrad{l}"] = timeit(
                lambda l=l, p=p, ci=ci, co=co, h=h, s=s, scm=scm, gsc=gsc:
                o.rn_dgrad(ci, co, h, s, eng.gy[l], eng.z[l], eng.stat[l], eng.red[l], eng.gamma[l], eng.wd[l],
                           eng.a[p], eng.z[p], eng.stat[p], gsc, scm, eng.gy[p], eng.red[p]), a.iters)
    res["head"] = timeit(lambda: o.rn_head(eng.z[18], eng.stat[18], eng.gamma[18], eng.beta[18], eng.a[16], eng.fcw,
                                           eng.fcb, eng.labels, eng.order_desc, eng.step_t, eng.period, 1.0 / eng.B,
                                           eng.gy[18], eng.red[18], eng.fc_part, eng.loss_img, eng.correct_img,
                                           None), a.iters)
    res["sgd"] = timeit(lambda: eng._sgd(mode=0), a.iters)
    res["fwd_sum"] = round(sum(v for k, v in res.items() if k.startswith("fwd")), 1)
    res["dgrad_sum"] = round(sum(v for k, v in res.items() if k.startswith("dgrad")), 1)
    res["wgrad_sum"] = round(sum(v for k, v in res.items() if k.startswith("wgrad")), 1)
    res["step_eager"] = timeit(eng.step, 20)
    eng.capture()
    res["step_graph"] = timeit(eng.step, 50)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
