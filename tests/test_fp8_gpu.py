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
