"""Repeat compute_gradients() with the in-launch slab reduction and compare each result with the
two-launch path (bitwise): finds intermittent races.  usage: dbg_race.py B dtype reps"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dmlc  # noqa: F401
from dmlc.engine.fused import FusedCifarEngine

B, dt, reps = int(sys.argv[1]), sys.argv[2], int(sys.argv[3])
g = torch.Generator().manual_seed(4)
data = torch.randint(0, 256, (1024, 32, 32, 3), dtype=torch.uint8, generator=g)
labels = torch.randint(0, 10, (1024,), dtype=torch.int32, generator=g)
os.environ["DMLC_WGRAD_SGD_FP8"] = "1"
fused = FusedCifarEngine(B, data, labels, seed=2, dtype=dt)
os.environ["DMLC_WGRAD_SGD"] = "0"
ref = FusedCifarEngine(B, data, labels, seed=2, dtype=dt)
assert fused._grad_in_launch and not ref._grad_in_launch
want = ref.compute_gradients().clone()
bad = 0
for r in range(reps):
    got = fused.compute_gradients().clone()
    torch.cuda.synchronize()
    if not torch.equal(got, want):
        bad += 1
        d = (got - want).abs()
        idx = torch.nonzero(d).flatten()
        print(f"rep {r}: {idx.numel()} differ, max {float(d.max()):.3e}, first {idx[:6].tolist()}", flush=True)
print(f"B={B} {dt}: {bad}/{reps} mismatching, err word {int(fused.wbar[320])}", flush=True)
