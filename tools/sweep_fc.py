"""Sweep the fc1 forward split-K factor of the fused CNN step (three-launch fc path) at one batch
size: whole captured steps timed, one JSON line per setting.
usage: python tools/sweep_fc.py [B] [split ...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc.engine.fused import FusedCifarEngine, head_rows  # noqa: E402  (head_rows: the three-launch head)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    splits = [int(v) for v in sys.argv[2:]] or [4, 6, 8, 9]
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g).cuda()
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g).cuda()
    for sp in splits:
        eng = FusedCifarEngine(B, data, labels, seed=0, fc1_split=sp)
        eng.step()
        eng.capture()
        eng.run(40)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            eng.run(400)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / 400)
        print(json.dumps({"B": B, "head_rows": head_rows(B), "fc1_split": sp,
                          "us_per_step": round(best * 1e6, 2)}), flush=True)
        del eng


if __name__ == "__main__":
    main()
