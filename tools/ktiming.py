#!/usr/bin/env python3
"""Per-phase timing of every fused-step kernel from in-kernel s_memrealtime stamps (100 MHz).

  DMLC_TIMING=1 python tools/ktiming.py [--batch 256] [--eager]
Builds/loads the diagnostic library (libdmlc_hip_timing.so), replays a 2-step graph chain (bench.py's
launch pattern; --eager: one eager step), and prints for
each kernel: span (first entry -> last stamp), and per slot the median / max over blocks of the time
since the block's own entry stamp.  Slot meanings are documented at each DMLC_STAMP call site.
"""
import argparse
import ctypes
import json
import os
import sys

os.environ["DMLC_TIMING"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc import _build  # noqa: E402
from dmlc.engine.fused import FusedCifarEngine  # noqa: E402

NAMES = ["conv1_fwd", "conv2_fwd", "gemm(last)", "head", "conv2_dgrad", "conv1_wgrad", "conv2_wgrad", "sgd"]
NK, NB, NS = 8, 1024, 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--raw", default="", help="comma list of kernel names whose per-block stamps (us since "
                    "the step's first stamp, -1 = not stamped) are dumped too, as raw_<name>")
    ap.add_argument("--eager", action="store_true",
                    help="time an eager step instead of the second step of a 2-step graph chain (eager "
                         "launches leave host gaps: the first kernel's workgroups then enter up to ~4 us "
                         "apart, 0.4 us in the graph)")
    ap.add_argument("--graph", action="store_true", help="(the default; kept for old command lines)")
    ap.add_argument("--variant", default="", help="engine variant keys, key=0|1,... (bench.py --variant)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    a = ap.parse_args()
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g)
    var = {k: bool(int(v)) for k, v in (kv.split("=") for kv in filter(None, a.variant.split(",")))}
    eng = FusedCifarEngine(a.batch, data, labels, device="cuda", lr=1e-4, variant=var, dtype=a.dtype)
    lib = ctypes.CDLL(_build.HIP_LIB)
    assert lib.dmlc_timing_enabled() == 1, "not a timing build"
    for _ in range(5):
        eng.step()
    torch.cuda.synchronize()
    if not a.eager:
        eng.capture(steps_per_graph=2)
        eng.run(4)
        torch.cuda.synchronize()
        lib.dmlc_timing_clear()
        eng.chains[2].replay()
    else:
        lib.dmlc_timing_clear()
        eng.step()
    torch.cuda.synchronize()
    buf = np.zeros(NK * NB * NS, dtype=np.uint64)
    assert lib.dmlc_timing_read(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    t = buf.reshape(NK, NB, NS).astype(np.int64)
    out = {}
    base = None
    for k in range(NK):
        blocks = t[k][t[k][:, 0] > 0]
        if len(blocks) == 0:
            continue
        ent = blocks[:, 0]
        if base is None or ent.min() < base:
            base = ent.min()
    for k in range(NK):
        blocks = t[k][t[k][:, 0] > 0]
        if len(blocks) == 0:
            continue
        ent = blocks[:, 0]
        rec = {"blocks": int(len(blocks)), "start_us": round((ent.min() - base) / 100.0, 2)}
        last = blocks.max()
        rec["span_us"] = round((last - ent.min()) / 100.0, 2)
        rec["entry_spread_us"] = round((ent.max() - ent.min()) / 100.0, 2)
        slots = {}
        for sl in range(1, NS):
            v = blocks[:, sl]
            ok = v > 0
            if ok.sum() == 0:
                continue
            d = (v[ok] - ent[ok]) / 100.0
            slots[sl] = [round(float(np.median(d)), 2), round(float(d.max()), 2)]
        rec["slot_med_max_us"] = slots
        if NAMES[k] == "sgd":      # per block-role breakdown (see cnn_sgd.hip block ranges)
            nfc1 = 1 if getattr(eng, "fc1_epilogue", False) else 217     # fc1 bias only / weight + bias
            roles = {"conv1_rows": (0, 150), "conv_bias": (150, 152), "conv2_rows": (152, 552),
                     "fc1": (552, 552 + nfc1), "fc2": (552 + nfc1, 576 + nfc1), "fc_tail": (576 + nfc1, 585 + nfc1)}
            raw = t[k]
            for name, (lo, hi) in roles.items():
                sub = raw[lo:hi]
                sub = sub[sub[:, 0] > 0]
                if len(sub):
                    d = (sub[:, 1] - sub[:, 0]) / 100.0
                    rec[f"role_{name}_work_us_med_max"] = [round(float(np.median(d)), 2), round(float(d.max()), 2)]
                    rec[f"role_{name}_start_us_max"] = round(float((sub[:, 0].max() - ent.min()) / 100.0), 2)
                    rec[f"role_{name}_work_q10_50_90"] = [round(float(np.percentile(d, q)), 2) for q in (10, 50, 90)]
                    ids = np.nonzero(raw[lo:hi, 0] > 0)[0] + lo
                    rec[f"role_{name}_slowest_blocks"] = [int(i) for i in ids[np.argsort(-d)[:8]]]
                    rec[f"role_{name}_work_by_xcd"] = [round(float(d[(ids % 8) == x].mean()), 2) if ((ids % 8) == x).any()
                                                       else None for x in range(8)]
        out[NAMES[k]] = rec
        if NAMES[k] in a.raw.split(","):
            raw = t[k]
            out["raw_" + NAMES[k]] = [[round(float((x - base) / 100.0), 2) if x > 0 else -1 for x in row]
                                      for row in raw[: int(np.nonzero(raw[:, 0] > 0)[0].max()) + 1]]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
