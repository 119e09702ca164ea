"""Compare one single-GPU step with the fc weight-gradient tiles in the wgrad launch
(DMLC_FC_DW_WGRAD=1) against the tiles in the fc chain + SGD (=0): per-segment max |diff|, and the
fc1 update of each against p2^T dh1 computed by torch from the step's own buffers."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dmlc  # noqa: F401
from dmlc.engine.fused import FusedCifarEngine
from dmlc.models import cifar_cnn as M
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
g = torch.Generator().manual_seed(5)
data = torch.randint(0, 256, (4 * B, 32, 32, 3), dtype=torch.uint8, generator=g)
labels = torch.randint(0, 10, (4 * B,), dtype=torch.int32, generator=g)
s1 = M.PARAM_SPECS[4]
for v in ("0", "1"):
    os.environ["DMLC_FC_DW_WGRAD"] = v
    e = FusedCifarEngine(B, data, labels, seed=4, lr=0.01)
    before = e.master[s1.offset:s1.offset + s1.numel].clone()
    e.step()
    torch.cuda.synchronize()
    after = e.master[s1.offset:s1.offset + s1.numel]
    upd = (before - after) / 0.01
    ref = (e.p2.view(e.B, 2304).float().t() @ e.dh1.float()).reshape(-1)
    rel = float((upd - ref).norm() / ref.norm())
    ratio = float((upd * ref).sum() / (ref * ref).sum())
    print(f"DMLC_FC_DW_WGRAD={v}: fc1 update vs p2^T dh1: rel {rel:.3e}, scale {ratio:.4f}, err {int(e.wbar[320])}", flush=True)
