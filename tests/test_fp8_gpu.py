"""fp8 (OCP e4m3fn) conv2 forward + input-gradient path (BASELINE config 5): converter format, forward
and dgrad numerics vs the fp32 PyTorch reference, delayed-scaling bookkeeping and training."""
import json
import os

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


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


@pytest.mark.parametrize("B", [64, 320])
def test_fp8_dgrad_matches_reference(B):
    """The fp8 conv2 input gradient (k_conv2_dgrad_fp8: per-image dY2 scale, e4m3 flipped weights,
    weight-stationary blocks looping over images for B > 256) against fp32 PyTorch fed with the
    kernel's own bf16 dY2 and the fp32 master W2; the bf16 kernel on the same inputs sets the scale of
    the comparison, and the conv1 weight gradient downstream must keep its direction."""
    data, labels = _synthetic(1024, seed=4)
    eng = FusedCifarEngine(B, data, labels, seed=2, dtype="fp8")
    assert eng.fp8_dgrad
    g8 = eng.compute_gradients().clone()
    torch.cuda.synchronize()
    dy = eng.dy2.float().view(B, 12, 12, 64).permute(0, 3, 1, 2)
    w = M.views(eng.flat_params().cuda())["conv2_kernel"].float()                # HWIO
    ref = torch.nn.grad.conv2d_input((B, 64, 12, 12), w.permute(3, 2, 0, 1).contiguous(), dy, padding=2)
    ref = ref.permute(0, 2, 3, 1)
    rel8 = _rel(eng.dp1, ref)
    dp1b, dy2b = torch.empty_like(eng.dp1), torch.empty_like(eng.dy2)
    eng.ops.conv2_dgrad(eng.dp2, eng.am2, eng.w2d, dp1b, dy2b)
    torch.cuda.synchronize()
    assert torch.equal(dy2b, eng.dy2)                  # the same pool2 / ReLU backward, bit for bit
    relb = _rel(dp1b, ref)
    per_img = ((eng.dp1.float() - ref).flatten(1).norm(dim=1) / ref.flatten(1).norm(dim=1).clamp_min(1e-30))
    eng.fp8_dgrad = False
    gb = eng.compute_gradients().clone()
    c1 = slice(M.PARAM_SPECS[0].offset, M.PARAM_SPECS[0].offset + M.PARAM_SPECS[0].numel)
    cos = float(torch.nn.functional.cosine_similarity(g8[c1], gb[c1], dim=0))
    out = {"B": B, "rel_fp8": rel8, "rel_bf16": relb, "per_image_rel_max": float(per_img.max()), "conv1_grad_cos": cos}
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/fp8_dgrad_numerics_b{B}.json", "w") as f:
        json.dump(out, f)
    assert rel8 < 6e-2 and float(per_img.max()) < 1e-1, out
    assert relb < 1e-2, out
    assert cos > 0.995, out


@pytest.mark.parametrize("B", [64, 100, 1024])
def test_fp8_wgrad_matches_reference(B):
    """The fp8 conv2 weight gradient (cnn_wgrad.hip w2_fp8_main: e4m3 operands quantised in the
    staging with per-batch scales from the per-image maxima, scaled 16x16x128 MFMA over units of two
    images) against fp32 PyTorch fed with the kernel's own bf16 p1 and dY2; the bf16 weight gradient
    on the same inputs sets the scale of the comparison.  B = 100 leaves groups with an odd image count
    (a half-empty last unit); B = 1024 runs 16 units per block."""
    data, labels = _synthetic(2048, seed=14)
    eng = FusedCifarEngine(B, data, labels, seed=12, dtype="fp8")
    assert eng.fp8_wgrad
    g8 = eng.compute_gradients().clone()
    torch.cuda.synchronize()
    Bv = eng.Bv
    x = eng.p1[:Bv].float().permute(0, 3, 1, 2)
    dy = eng.dy2[:Bv].float().view(Bv, 12, 12, 64).permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(x, (64, 64, 5, 5), dy, padding=2).permute(2, 3, 1, 0).reshape(-1)   # HWIO
    refb = dy.sum(dim=(0, 2, 3))
    s2, sb = M.PARAM_SPECS[2], M.PARAM_SPECS[3]
    got = g8[s2.offset:s2.offset + s2.numel]
    gotb = g8[sb.offset:sb.offset + sb.numel]
    eng._w8 = {}                                   # the bf16 conv2 weight gradient, same batch
    gbf = eng.compute_gradients().clone()[s2.offset:s2.offset + s2.numel]
    torch.cuda.synchronize()
    out = {"B": B, "rel_fp8": _rel(got, ref), "rel_bf16": _rel(gbf, ref), "rel_bias": _rel(gotb, refb),
           "cos_fp8": float(torch.nn.functional.cosine_similarity(got, ref, dim=0))}
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/fp8_wgrad_numerics_b{B}.json", "w") as f:
        json.dump(out, f)
    assert out["rel_bf16"] < 1e-2, out
    assert out["rel_fp8"] < 6e-2 and out["cos_fp8"] > 0.998, out
    assert out["rel_bias"] < 2e-2, out             # (from the e4m3 dY bytes, one ones-MFMA per chunk)


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
    assert abs(float(eng.amax_w[s].max()) - amax) <= 1e-6 * max(1.0, amax)  # exact amax (block maxima)
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


@pytest.mark.parametrize("B", [64, 100, 1024])
def test_fp8_sgd_in_wgrad_launch_is_bit_identical(B):
    """fp8 (BASELINE config 5) on one GPU: the SGD inside the wgrad launch also writes the e4m3
    shadows (forward w2f8, the dgrad's flipped copy) with the delayed per-tensor scale and the new
    weights' amax slots.  After eager + graph-replayed steps the parameters, both fp8 shadows, the
    scales and the stats equal the SGD-launch path bit for bit."""
    data, labels = _synthetic(8 * B, seed=51)
    kw = dict(seed=52, lr=1e-4, relu_logits=False, dtype="fp8")
    fused = FusedCifarEngine(B, data, labels, **kw, variant={"wgrad_sgd_fp8": True})   # opt-in (measured slower)
    ref = FusedCifarEngine(B, data, labels, **kw, variant={"wgrad_sgd": False})
    assert fused.wgrad_apply and not ref.wgrad_apply and fused.fp8
    for eng in (ref, fused):
        eng.step()
        eng.step()
        eng.capture(steps_per_graph=4)
        eng.run(5)
    torch.cuda.synchronize()
    fused.check_barriers()
    assert ref.global_step() == fused.global_step() == 7
    assert torch.isfinite(ref.master).all()
    assert torch.equal(ref.master, fused.master)
    assert torch.equal(ref.w2f8, fused.w2f8)
    assert torch.equal(ref.scale_w, fused.scale_w)
    assert float(ref.amax_w[1].max()) == float(fused.amax_w[1].max())   # step 7: slot 1 holds the new amax
    assert ref.read_stats(7) == fused.read_stats(7)


@pytest.mark.parametrize("B", [64, 100, 1024])
def test_fp8_conv_grad_reduction_in_wgrad_launch_is_bit_identical(B):
    """fp8 compute_gradients() through the in-launch conv-slab reduction (reduce mode, the data-parallel
    path; helpers included at B=64) against the reduce-only SGD launch, bit for bit over the whole flat
    gradient, for the generated batch and an explicit index list -- the case round 3 excluded after a
    wrong conv1 gradient (cosine 0.24 at B=64) on an intermediate build."""
    data, labels = _synthetic(8 * B, seed=47)
    kw = dict(seed=48, lr=1e-4, relu_logits=False, dtype="fp8")
    fused = FusedCifarEngine(B, data, labels, **kw, variant={"wgrad_sgd_fp8": True})   # single GPU: the opt-in
    ref = FusedCifarEngine(B, data, labels, **kw, variant={"wgrad_sgd": False})
    assert fused._grad_in_launch and not ref._grad_in_launch and fused.fp8
    idx = torch.randperm(8 * B, generator=torch.Generator().manual_seed(3))[:B].to(torch.int32)
    for explicit in (None, idx, None):
        g_ref = ref.compute_gradients(explicit).clone()
        g_fused = fused.compute_gradients(explicit).clone()
        torch.cuda.synchronize()
        assert torch.isfinite(g_ref).all() and float(g_ref.abs().max()) > 0
        assert torch.equal(g_ref, g_fused)
    assert torch.equal(ref.scale_w, fused.scale_w)            # reduce mode leaves the fp8 state alone
    fused.check_barriers()


def test_check_barriers_raises_in_reduce_mode():
    """The sticky error word of the wgrad sub-grid barriers is checked in reduce mode too (a timed-out
    barrier there would all-reduce partial conv gradients that every replica agrees on), through the
    device read and through the pinned copy the trainer reads at every progress point."""
    data, labels = _synthetic(512, seed=5)
    eng = FusedCifarEngine(64, data, labels, seed=6, dp_force=True, allreduce="rccl")   # no step taken
    assert eng.wgrad_reduce and not eng.wgrad_apply and eng.barriers_in_use
    eng.wbar[320] = 1                                         # as bar_wait's give-up path sets it
    with pytest.raises(RuntimeError, match="sub-grid barrier timed out"):
        eng.check_barriers()
    eng.queue_error_copy()
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="sub-grid barrier timed out"):
        eng.check_barriers(cached=True)
    with pytest.raises(RuntimeError):
        eng.check_comm()
    eng.wbar[320] = 0
    eng.check_barriers()
