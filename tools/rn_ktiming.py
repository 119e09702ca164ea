#!/usr/bin/env python3
"""Per-phase timing of the stage-1 ResNet-20 kernels (16->16 channels, 32x32) from in-kernel
s_memrealtime stamps (100 MHz); timing build only.

  DMLC_TIMING=1 python tools/rn_ktiming.py [--batch 256]
Stamp ids / slots (csrc/kernels/resnet.hip, `TS` sites): 0 = k_rn_fwd<16,16,32,1> (1 input staged,
2 weights + barrier, 3 MFMAs issued, 4 z stored, 5 statistics flushed); 1 = its dgrad body (1 g_z
staged, 2 MFMAs, 3 g_y stored, 4 reductions flushed); 2 = its wgrad body (1 first staging step,
2 MFMAs, 3 slab written).  The last launch of each shape in one training step wins the slots.
Prints per kernel: blocks, span (first entry -> last stamp), entry spread, and per slot the median /
max over blocks of the time since the block's own entry."""
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
from dmlc.engine.fused_resnet import FusedResNetEngine  # noqa: E402

NAMES = {0: "rn_fwd16", 1: "rn_dgrad16", 2: "rn_wgrad16"}
NK, NB, NS = 8, 1024, 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g)
    eng = FusedResNetEngine(a.batch, data, labels, device="cuda", lr=1e-3)
    lib = ctypes.CDLL(_build.HIP_LIB)
    assert lib.dmlc_timing_enabled() == 1, "not a timing build"
    for _ in range(5):
        eng.step()
    torch.cuda.synchronize()
    lib.dmlc_timing_clear()
    eng.step()
    torch.cuda.synchronize()
    buf = np.zeros(NK * NB * NS, dtype=np.uint64)
    assert lib.dmlc_timing_read(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    t = buf.reshape(NK, NB, NS).astype(np.int64)
    out = {}
    for k, name in NAMES.items():
        blocks = t[k][t[k][:, 0] > 0]
        if len(blocks) == 0:
            continue
        ent = blocks[:, 0]
        rec = {"blocks": int(len(blocks)), "span_us": round((blocks.max() - ent.min()) / 100.0, 2),
               "entry_spread_us": round((ent.max() - ent.min()) / 100.0, 2)}
        slots = {}
        for sl in range(1, NS):
            v = blocks[:, sl]
            ok = v > 0
            if ok.sum() == 0:
                continue
            d = (v[ok] - ent[ok]) / 100.0
            slots[sl] = [round(float(np.median(d)), 2), round(float(d.max()), 2)]
        rec["slot_med_max_us"] = slots
        out[name] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
