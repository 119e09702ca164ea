"""Timed-region anatomy of bench.py: wall time of run(k) for several k after capture + warm-up, to
separate the fixed cost of a timed region (first graph launch after an idle queue) from the
per-step cost.  Prints one JSON object: {k: us}, plus the least-squares fit us = fixed + k * per_step."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc.engine.fused import FusedCifarEngine  # noqa: E402


def main():
    B = int(os.environ.get("B", "256"))
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g).cuda()
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g).cuda()
    eng = FusedCifarEngine(B, data, labels, device="cuda:0")
    for _ in range(3):
        eng.step()
    eng.capture(int(os.environ.get("SPG", "8")))
    eng.run(64)
    torch.cuda.synchronize()
    res = {}
    for k in (1, 2, 4, 8, 16, 20, 40, 80, 160, 400):
        best = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(k)
            torch.cuda.synchronize()
            best.append((time.perf_counter() - t0) * 1e6)
        res[k] = round(min(best), 1)
    ks = torch.tensor(list(res), dtype=torch.float64)
    ts = torch.tensor(list(res.values()), dtype=torch.float64)
    A = torch.stack([torch.ones_like(ks), ks], 1)
    fit = torch.linalg.lstsq(A, ts.unsqueeze(1)).solution.squeeze(1).tolist()
    print(json.dumps({"B": B, "us": res, "fixed_us": round(fit[0], 1), "per_step_us": round(fit[1], 2)}))


if __name__ == "__main__":
    main()
