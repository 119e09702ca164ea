"""ResNet-20 (BASELINE config 4): structure, numerics vs an independent torch.nn build, training
step, checkpoint names/round trip through the CLI trainer (CPU)."""
import os
import subprocess
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

from dmlc import checkpoint as CK
from dmlc.models import resnet as R

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_param_count_and_names():
    assert R.NUM_PARAMS == 269722       # 267,696 conv + 1,376 BN affine + 650 fc
    names = [s.name for s in R.PARAM_SPECS]
    assert names[0] == "resnet20/stem/conv/kernel" and names[-1] == "resnet20/fc/biases"
    assert sum(1 for n in names if n.endswith("/conv/kernel")) == 19
    assert all(s.offset % 64 == 0 for s in R.PARAM_SPECS + R.STATE_SPECS)


class _RefBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, cout, 3, stride, 0, bias=False)
        self.b1 = nn.BatchNorm2d(cout, eps=1e-3)
        self.c2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.b2 = nn.BatchNorm2d(cout, eps=1e-3)
        self.stride, self.cin, self.cout = stride, cin, cout

    def forward(self, x):
        pad = (0, 1, 0, 1) if self.stride == 2 else (1, 1, 1, 1)
        y = F.relu(self.b1(self.c1(F.pad(x, pad))))
        y = self.b2(self.c2(y))
        sc = x[:, :, ::2, ::2] if self.stride == 2 else x
        sc = F.pad(sc, (0, 0, 0, 0, 0, self.cout - self.cin))
        return F.relu(y + sc)


def test_matches_independent_torch_nn_build():
    torch.manual_seed(0)
    m = R.ResNet20(seed=3)
    p = R._views(m.flat.detach(), R.PARAM_SPECS)
    stem = nn.Conv2d(3, 16, 3, 1, 1, bias=False)
    stem_bn = nn.BatchNorm2d(16, eps=1e-3)
    blocks, cin = [], 16
    for s, w in enumerate(R.WIDTHS):
        for b in range(3):
            blocks.append(_RefBlock(cin, w, 2 if (s > 0 and b == 0) else 1))
            cin = w
    with torch.no_grad():
        stem.weight.copy_(p["stem/conv/kernel"].permute(3, 2, 0, 1))
        i = 0
        for s in range(3):
            for b in range(3):
                blk = blocks[i]
                blk.c1.weight.copy_(p[f"stage{s}/block{b}/a/conv/kernel"].permute(3, 2, 0, 1))
                blk.c2.weight.copy_(p[f"stage{s}/block{b}/b/conv/kernel"].permute(3, 2, 0, 1))
                i += 1
    x = torch.rand(4, 32, 32, 3) * 255
    h = F.relu(stem_bn(stem(x.permute(0, 3, 1, 2))))
    for blk in blocks:
        h = blk(h)
    ref = h.mean(dim=(2, 3)) @ p["fc/weights"] + p["fc/biases"]
    got = m(x)
    assert torch.allclose(got, ref, rtol=1e-4, atol=1e-4)
    # train-mode BN moved the moving stats
    mm = R._views(m.state, R.STATE_SPECS)["stem/bn/moving_mean"]
    assert float(mm.abs().sum()) > 0


def test_training_step_reduces_loss_and_eval_mode():
    from dmlc.data import synthetic
    from dmlc.engine.eager import EagerTrainer
    torch.manual_seed(0)
    x, y = synthetic(256, seed=2, learnable=True)
    tr = EagerTrainer("resnet20", 64, x, y, lr=0.05, crop=32, seed=1)
    losses = []
    for _ in range(12):
        tr.step()
        losses.append(float(tr.last_loss))
    assert losses[-1] < losses[0]
    acc = tr.evaluate(x, y, max_batches=1)
    assert 0.0 <= acc <= 1.0


def test_cli_resnet20_checkpoint_roundtrip(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="4")
    cmd = [sys.executable, os.path.join(REPO, "cifar10cnn.py"), "--model=resnet20", "--crop=32", "--synthetic",
           "--synthetic_size=256", "--batch_size=32", "--device=cpu", "--generations=4", "--output_every=2",
           "--eval_every=4", "--eval_batches=1", "--learning_rate=0.05", f"--log_dir={tmp_path}"]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=240)
    assert r.returncode == 0, r.stdout
    t = CK.read_bundle(CK.latest_checkpoint(str(tmp_path)))
    assert int(t["global_step"]) == 4
    assert tuple(t["resnet20/stage2/block0/a/conv/kernel"].shape) == (3, 3, 32, 64)
    assert "resnet20/stem/bn/moving_variance" in t
    m = R.ResNet20()
    assert CK.load_module_tensors(m, t) == 4
    r2 = subprocess.run(cmd[:-5] + ["--generations=6", "--output_every=2", "--eval_every=100", "--eval_batches=1",
                                    "--learning_rate=0.05", f"--log_dir={tmp_path}"],
                        env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=240)
    assert r2.returncode == 0 and "Restored" in r2.stdout, r2.stdout
    assert int(CK.read_bundle(CK.latest_checkpoint(str(tmp_path)))["global_step"]) == 6


def test_fused_resnet_layer_table_matches_model():
    """The fused engine's execution order / shortcut wiring (CPU-checkable part of engine/fused_resnet.py)."""
    from dmlc.engine import fused_resnet as FR
    from dmlc.models import resnet as R
    convs = [s.name for s in R.PARAM_SPECS if s.name.endswith("/conv/kernel")]
    assert [f"{R.SCOPE}/{n}/conv/kernel" for n, *_ in FR.LAYERS] == convs
    shapes = {s.name: s.shape for s in R.PARAM_SPECS}
    for n, ci, co, h, s in FR.LAYERS:
        assert shapes[f"{R.SCOPE}/{n}/conv/kernel"] == (3, 3, ci, co)
    assert [l for l, (*_, s) in enumerate(FR.LAYERS) if s == 2] == [7, 13]
    assert [FR._block_sc_mode(b) for b in range(2, 19, 2)] == [1, 1, 1, 2, 1, 1, 2, 1, 1]
    # every conv offset is float4-aligned (the SGD kernel updates HWIO rows 4 c_out at a time)
    P = {s.name: s.offset for s in R.PARAM_SPECS}
    assert all(P[f"{R.SCOPE}/{n}/conv/kernel"] % 4 == 0 for n, *_ in FR.LAYERS)
    for B in (16, 256, 1024):
        for _, ci, co, _, _ in FR.LAYERS:
            g = FR.FusedResNetEngine._pick_groups(B, ci, co)
            assert 1 <= g <= B and g & (g - 1) == 0


def test_fixed_point_bn_slots_are_order_independent():
    """The fused engine's BatchNorm sums are fixed-point (resnet.hip fx_add / fx_total): integer part +
    48-bit fraction per fp32 partial.  Any add order gives the same bits, the total matches an fp64 sum,
    and a poisoned slot (non-finite partial) decodes to NaN.  Host mirror of the encoding."""
    from dmlc.engine import fused_resnet as FR
    g = torch.Generator().manual_seed(0)
    parts = (torch.randn(256, 128, generator=g) * torch.logspace(-6, 4, 128)).float()   # one row per block
    hi, lo = FR.fx_encode(parts)
    assert int(lo.min()) >= 0 and int(lo.max()) <= 2 ** 48

    def accumulate(order):
        slots = torch.zeros(FR.NSLOT, 256, dtype=torch.int64)
        for b in order.tolist():
            slots[b % FR.NSLOT, :128] += hi[b]
            slots[b % FR.NSLOT, 128:] += lo[b]
        return slots

    s1 = accumulate(torch.arange(256))
    s2 = accumulate(torch.randperm(256, generator=g))
    assert torch.equal(s1, s2)
    tot = FR.fx_decode(s1)
    ref = parts.double().sum(0)
    # each add rounds its fraction to 2^-48 (error <= 2^-49): an absolute bound, far below the fp32
    # partials' own relative rounding (2^-24)
    assert bool(((tot - ref).abs() <= 256 * 2.0 ** -49 + 1e-13 * ref.abs()).all())
    s1[3, 5] += 1 << 56                                      # a non-finite partial's poison
    t = FR.fx_decode(s1)
    assert torch.isnan(t[5]) and torch.isfinite(t[:5]).all()
