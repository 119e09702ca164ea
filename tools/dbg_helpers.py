"""Debug: compare fused engines (eager / graph, helpers on / off) segment by segment."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dmlc  # noqa: F401
from dmlc.engine.fused import FusedCifarEngine
from dmlc.models import cifar_cnn as M

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
g = torch.Generator().manual_seed(7)
data = torch.randint(0, 256, (8 * B, 32, 32, 3), dtype=torch.uint8, generator=g)
labels = torch.randint(0, 10, (8 * B,), dtype=torch.int32, generator=g)


def run(graph, wsgd="1", steps=int(os.environ.get("STEPS", "1"))):
    os.environ["DMLC_WGRAD_SGD"] = wsgd
    e = FusedCifarEngine(B, data, labels, seed=8, lr=1e-4)
    if graph:
        e.capture()
    for _ in range(steps):
        e.step()
    torch.cuda.synchronize()
    return e


ref = run(False, "0")
for name, e in [("eager", run(False)), ("graph", run(True)), ("eager2", run(False))]:
    print(name, "err", int(e.wbar[320]), "claims", e.wbar[352:352 + 8].tolist(), "gens", e.wbar[6 * 32:10 * 32:32].tolist())
    for s in M.PARAM_SPECS:
        a, b = e.master[s.offset:s.offset + s.numel], ref.master[s.offset:s.offset + s.numel]
        d = (a - b).abs()
        if d.max() > 0:
            idx = torch.nonzero(d).flatten()
            print(f"  {s.name}: {idx.numel()} differ, max {float(d.max()):.3e} (|w| {float(b.abs().max()):.3e}), first idx {idx[:8].tolist()}")
            if s.numel == 102400:   # conv2 HWIO: idx = krow * 64 + co, krow = tap * 64 + ci
                krow, co = idx // 64, idx % 64
                print("    taps", sorted(set((krow // 64).tolist()))[:30], "ci", sorted(set((krow % 64).tolist()))[:70],
                      "co", sorted(set(co.tolist()))[:70])
            if s.numel == 4800:
                row, co = idx // 64, idx % 64
                print("    rows", sorted(set(row.tolist()))[:80], "co", sorted(set(co.tolist()))[:70])
