import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import dmlc
from dmlc.engine.fused import FusedCifarEngine
from dmlc.models import cifar_cnn as M
g = torch.Generator().manual_seed(41)
B = 128
data = torch.randint(0, 256, (8 * B, 32, 32, 3), dtype=torch.uint8, generator=g)
labels = torch.randint(0, 10, (8 * B,), dtype=torch.int32, generator=g)
ref = FusedCifarEngine(B, data, labels, seed=40, lr=0.01)
os.environ["DMLC_FC_BRANCH"] = "1"
br = FusedCifarEngine(B, data, labels, seed=40, lr=0.01)
def cmp(tag):
    torch.cuda.synchronize()
    out = [tag, ref.global_step(), br.global_step(), "nan_br", bool(torch.isnan(br.master).any()), "nan_ref", bool(torch.isnan(ref.master).any())]
    for s in M.PARAM_SPECS:
        a = ref.master[s.offset:s.offset+s.numel]; b = br.master[s.offset:s.offset+s.numel]
        out.append((M.short(s.name), int((a != b).sum())))
    for n in ("p1", "p2", "h1", "dh1", "dp2", "dp1", "dy2", "part2", "part1", "fc1n", "w2f", "bidx"):
        out.append((n, bool(torch.equal(getattr(ref, n), getattr(br, n)))))
    print(out, flush=True)
ref.step(); br.step(); cmp("eager1")
for e in (ref, br): e.capture(steps_per_graph=2)
cmp("after-capture")
ref.graphs[0].replay(); br.graphs[0].replay(); cmp("graph1")
ref.graphs[0].replay(); br.graphs[0].replay(); cmp("graph1b")
ref.chains[2].replay(); br.chains[2].replay(); cmp("chain2")
ref.step(); br.step(); cmp("step-after")
