"""fp8 (OCP e4m3fn) conv2 forward path (BASELINE config 5): converter format, forward numerics vs the
fp32 PyTorch reference, delayed-scaling bookkeeping and training."""
import pytest
import torch

from dmlc.engine.fused import FusedCifarEngine
from dmlc.models import cifar_cnn as M

pytestmark = pytest.mark.gpu


def _synthetic(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, generator=g),
            torch.randint(0, 10, (n,), dtype=torch.int32, generator=g))


def test_converter_is_ocp_e4m3fn():
    import dmlc.ops._ext as E
    E.hip()
    x = (torch.rand(100000, device="cuda") * 2 - 1) * 440
    x[:8] = torch.tensor([0.0, 1.0, -1.0, 0.0625, 448.0, -448.0, 1e-3, 240.0], device="cuda")
    y = torch.empty_like(x)
    torch.ops.dmlc.fp8_roundtrip(x, y, 1.0)
    ref = x.to(torch.float8_e4m3fn).float()
    assert torch.equal(y, ref), (y - ref).abs().max()
    # saturation instead of NaN beyond the e4m3fn range
    big = torch.tensor([1000.0, -1e6], device="cuda")
    yb = torch.empty_like(big)
    torch.ops.dmlc.fp8_roundtrip(big, yb, 1.0)
    assert yb.tolist() == [448.0, -448.0]


def test_fp8_forward_matches_reference():
    B = 64
    data, labels = _synthetic(512, seed=3)
    eng = FusedCifarEngine(B, data, labels, seed=1, dtype="fp8")
    idx = torch.randperm(data.shape[0])[:B].to(torch.int32)
    eng.forward_logits(idx)                 # first call populates the activation amax slot
    got = eng.forward_logits(idx)
    x = data[idx.long()].cuda()[:, 4:28, 4:28, :].float()
    ref = M.cnn_forward(x, M.views(eng.flat_params().cuda()), True)
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 8e-2, rel
    assert float(eng.scale_w[eng.host_step & 1]) > 0


def test_fp8_training_tracks_scales_and_reduces_loss():
    from dmlc.data import synthetic
    data, labels = synthetic(2048, seed=9, learnable=True)
    eng = FusedCifarEngine(128, data, labels, seed=10, lr=0.0005, relu_logits=False, dtype="fp8")
    eng.step()
    eng.capture()
    losses = []
    for i in range(60):
        eng.step()
        if (i + 1) % 10 == 0:
            torch.cuda.synchronize()
            losses.append(eng.read_stats(eng.host_step)["loss"])
    s = eng.host_step & 1
    w2 = M.views(eng.flat_params())["conv2_kernel"]
    amax = float(w2.abs().max())
    assert abs(float(eng.amax_w[s]) - amax) <= 1e-6 * max(1.0, amax)       # exact running amax
    assert abs(float(eng.scale_w[s]) * amax - 224.0) / 224.0 < 0.05        # 2x headroom scale
    assert losses[-1] < 0.9 * losses[0], losses


def test_fp8_loss_curve_tracks_bf16_over_300_steps():
    """BASELINE config 5 acceptance: 300 steps of the same run in fp8 (conv2 forward on the f8f6f4
    MFMA) and in bf16 -- same weights, same batches (the generated order is shared) -- must give loss
    curves within 5 % of each other on 25-step windows, and both must learn."""
    from dmlc.data import synthetic
    B, steps, win = 128, 300, 25
    data, labels = synthetic(8192, seed=5, learnable=True)
    curves = {}
    for dt in ("bf16", "fp8"):
        eng = FusedCifarEngine(B, data, labels, seed=6, lr=1e-4, relu_logits=False, staircase=False, dtype=dt)
        eng.step()
        eng.capture()
        eng.run(steps - 1)
        torch.cuda.synchronize()
        curves[dt] = torch.tensor([eng.read_stats(k)["loss"] for k in range(1, steps + 1)]).view(-1, win).mean(1)
    wb, wf = curves["bf16"], curves["fp8"]
    assert torch.isfinite(wf).all() and wf[-1] < 0.5 * wf[0] and wb[-1] < 0.5 * wb[0], (wf.tolist(), wb.tolist())
    dev = float(((wf - wb).abs() / wb).max())
    assert dev < 0.05, (dev, wf.tolist(), wb.tolist())


def test_lr_warmup_and_linear_scaling_on_device():
    """The fused SGD kernel's learning rate (lr_of) with the large-batch recipe: a linear warm-up
    over the first steps times the staircase decay, read back from the on-device stats ring."""
    from dmlc.data import synthetic
    data, labels = synthetic(256, seed=3)
    eng = FusedCifarEngine(16, data, labels, seed=4, lr=0.4, lr_decay=0.5, decay_steps=3, warmup_steps=4)
    for _ in range(8):
        eng.step()
    torch.cuda.synchronize()
    want = [0.4 * 0.5 ** (s // 3) * (min(s + 1, 4) / 4) for s in range(8)]
    assert [eng.read_stats(s)["lr"] for s in range(1, 9)] == pytest.approx(want, rel=1e-6)
