"""Numerics of the HIP kernels vs a plain PyTorch fp32 reference of the same ops (TF semantics).

Every check goes through the fused engine, i.e. exactly the kernels the benchmark runs."""
import pytest
import torch

from dmlc.engine.fused import FusedCifarEngine
from dmlc.models import cifar_cnn as M

pytestmark = pytest.mark.gpu


def _synthetic(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    data = torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (n,), dtype=torch.int32, generator=g)
    return data, labels


def _ref_grads(flat, data, labels, idx, relu_logits=True):
    dev = "cuda"
    flat = flat.to(dev).clone().requires_grad_(True)
    x = data[idx.long()].to(dev)[:, 4:28, 4:28, :].float()
    logits = M.cnn_forward(x, M.views(flat), relu_logits)
    loss = M.cifar_loss(logits, labels[idx.long()].to(dev))
    loss.backward()
    return logits.detach(), loss.detach(), flat.grad.detach()


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


@pytest.mark.parametrize("B", [16, 64, 128])
def test_forward_logits_match_reference(B):
    data, labels = _synthetic(max(256, 2 * B))
    eng = FusedCifarEngine(B, data, labels, seed=1)
    idx = torch.randperm(data.shape[0])[:B].to(torch.int32)
    got = eng.forward_logits(idx)
    ref, _, _ = _ref_grads(eng.flat_params(), data, labels, idx)
    assert _rel(got, ref) < 3e-2, _rel(got, ref)


@pytest.mark.parametrize("B", [32, 128])
def test_gradients_match_reference(B):
    data, labels = _synthetic(4 * B, seed=3)
    eng = FusedCifarEngine(B, data, labels, seed=2)
    idx = eng.batch_indices(eng.host_step)
    grad = eng.compute_gradients().cpu()
    _, _, gref = _ref_grads(eng.flat_params(), data, labels, idx)
    gref = gref.cpu()
    for s in M.PARAM_SPECS:
        a = grad[s.offset:s.offset + s.numel]
        b = gref[s.offset:s.offset + s.numel]
        if b.norm() < 1e-8:
            assert a.norm() < 1e-4, s.name
            continue
        # end-to-end: bf16 error compounds through 7 kernels (and can flip ReLU / pool decisions),
        # so this is a direction check; the per-kernel 1e-2 checks are tests/test_cnn_kernels_gpu.py
        cos = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
        assert cos > 0.995, (s.name, cos, _rel(a, b))


def test_multi_step_graph_run_equals_eager_steps():
    """run(n) replays chains of 8/4/2/1 captured steps straight across epoch boundaries (the batch
    order is generated in-kernel from the step counter); the result is bit-identical to n eager
    steps (same batches, same LR schedule)."""
    B = 32
    data, labels = _synthetic(5 * B, seed=9)          # period 5: every chain crosses an epoch boundary
    kw = dict(seed=11, lr=1e-4, decay_steps=4, relu_logits=False)     # stays finite: NaN != NaN
    a = FusedCifarEngine(B, data, labels, **kw)
    b = FusedCifarEngine(B, data, labels, **kw)
    a.step()
    a.capture(steps_per_graph=8)
    assert sorted(a.chains) == [1, 2, 4, 8]
    a.run(20)
    assert a.add_chain(7) and not a.add_chain(7)       # exact-length chain (bench's short regions)
    a.run(7)                                           # ONE replay of the 7-step graph
    for _ in range(28):
        b.step()
    torch.cuda.synchronize()
    assert a.global_step() == b.global_step() == 28 and a.host_step == 28
    assert torch.isfinite(a.flat_params()).all()
    assert torch.equal(a.flat_params(), b.flat_params())
    assert a.read_stats(28) == b.read_stats(28) and a.read_stats(21) == b.read_stats(21)


def test_sgd_step_matches_reference_update():
    B = 64
    data, labels = _synthetic(4 * B, seed=5)
    eng = FusedCifarEngine(B, data, labels, seed=4, lr=0.01)
    before = eng.flat_params().clone()
    idx = eng.batch_indices(eng.host_step)
    eng.step()
    torch.cuda.synchronize()
    after = eng.flat_params()
    _, loss, gref = _ref_grads(before, data, labels, idx)
    expect = before - 0.01 * gref.cpu()
    assert eng.global_step() == 1
    st = eng.read_stats(1)
    assert abs(st["loss"] - float(loss)) / max(1.0, abs(float(loss))) < 2e-2
    assert abs(st["lr"] - 0.01) < 1e-7
    delta, dref = after - before, expect - before
    assert float(torch.nn.functional.cosine_similarity(delta, dref, dim=0)) > 0.99


def test_graph_replay_equals_eager_and_is_deterministic():
    B = 64
    data, labels = _synthetic(8 * B, seed=7)
    a = FusedCifarEngine(B, data, labels, seed=8)
    b = FusedCifarEngine(B, data, labels, seed=8)
    for _ in range(3):
        a.step()
    b.capture()
    for _ in range(3):
        b.step()
    torch.cuda.synchronize()
    assert a.global_step() == b.global_step() == 3
    assert torch.equal(a.flat_params(), b.flat_params())


def test_training_reduces_loss():
    # The reference model (raw 0..255 pixels, ReLU on the logits) dies at most learning rates; the
    # convergence check runs the same kernels with linear logits (the --relu_logits=false variant).
    from dmlc.data import synthetic
    B = 128
    data, labels = synthetic(2048, seed=9, learnable=True)
    eng = FusedCifarEngine(B, data, labels, seed=10, lr=0.0005, relu_logits=False)
    eng.capture()
    losses = []
    for i in range(60):
        eng.step()
        if (i + 1) % 10 == 0:
            torch.cuda.synchronize()
            losses.append(eng.read_stats(eng.host_step)["loss"])
    assert losses[-1] < 0.9 * losses[0], losses


def test_lr_staircase_schedule_on_device():
    B = 16
    data, labels = _synthetic(64, seed=11)
    eng = FusedCifarEngine(B, data, labels, seed=12, lr=0.1, lr_decay=0.5, decay_steps=2)
    for _ in range(5):
        eng.step()
    torch.cuda.synchronize()
    lrs = [eng.read_stats(s)["lr"] for s in range(1, 6)]
    assert lrs == pytest.approx([0.1, 0.1, 0.05, 0.05, 0.025])


def test_fused_conv12_forward_equals_two_launches():
    """ops.conv12_fwd (conv1 -> pool1 -> conv2 -> pool2 of an image in one workgroup, pool1 handed to
    conv2 through LDS) produces bit-identical p1 / argmax / p2 / logits to the two separate launches."""
    B = 64
    data, labels = _synthetic(4 * B, seed=21)
    fused = FusedCifarEngine(B, data, labels, seed=20, conv_split=1)
    assert fused.fused_fwd
    idx = torch.randperm(data.shape[0])[:B].to(torch.int32)
    lf = fused.forward_logits(idx).clone()
    split = FusedCifarEngine(B, data, labels, seed=20, conv_split=1, variant={"split_fwd": True})
    assert not split.fused_fwd
    ls = split.forward_logits(idx).clone()
    for n in ("p1", "am1", "p2", "am2"):
        assert torch.equal(getattr(fused, n), getattr(split, n)), n
    assert torch.equal(lf, ls)



@pytest.mark.parametrize("B,split1", [(128, 2), (128, 4), (256, 2), (48, 4)])
def test_channel_split_kernels_match_per_image_kernels(B, split1):
    """The channel-split kernels (cnn_split.hip, S workgroups per image) against the one-workgroup-
    per-image kernels on the same weights and batch.  conv1 accumulates every output in the same K
    order in both, so p1 and its argmax bytes are bit-identical; conv2 adds two K halves, so p2 /
    logits / gradients agree to fp32 summation order (then bf16 rounding)."""
    data, labels = _synthetic(4 * B, seed=31)
    ref = FusedCifarEngine(B, data, labels, seed=30, conv_split=1)
    spl = FusedCifarEngine(B, data, labels, seed=30, conv_split=2, conv1_split=split1)
    idx = torch.randperm(data.shape[0], generator=torch.Generator().manual_seed(2))[:B].to(torch.int32)
    gr = ref.compute_gradients(idx=idx).clone()
    gs = spl.compute_gradients(idx=idx).clone()
    torch.cuda.synchronize()
    assert torch.equal(ref.p1, spl.p1) and torch.equal(ref.am1, spl.am1)
    # the split forward copies the explicit rows' images out for its wgrad (the per-image engine's
    # xraw is restored to its own step's rows afterwards: it prefetches them)
    assert torch.equal(spl.xraw, data[idx.long()].view(B, 3072).to(spl.xraw.device))
    assert _rel(spl.p2, ref.p2) < 1e-2
    assert float((spl.am2 != ref.am2).float().mean()) < 1e-3
    assert _rel(spl.dy2, ref.dy2) < 2e-2 and _rel(spl.dp1, ref.dp1) < 2e-2
    assert _rel(gs, gr) < 2e-2, _rel(gs, gr)


def test_generated_order_in_kernels_matches_host_twin():
    """The kernels' in-place Feistel order (common.h order_perm) picks exactly the rows the host
    twin (data/order.py) names, at epoch starts, ends and far-away steps: the forward through the
    generated order is bit-identical to the forward through the explicit index list."""
    B = 32
    data, labels = _synthetic(1000, seed=13)           # period 31
    eng = FusedCifarEngine(B, data, labels, seed=14)
    for step in (0, 1, 30, 31, 62, 1000, 123457):
        eng.set_step(step)
        eng._forward(eng.order_desc, eng.step_t, eng.period, train=False, logits_out=eng.logits_buf)
        gen = eng.logits_buf.clone()
        ref = eng.forward_logits(eng.batch_indices(step))
        assert torch.equal(gen, ref), step


def test_chained_run_across_n8_shard_epochs_equals_eager():
    """The N=8 shard case: 50k rows / 8 ranks at B=256 is a 24-step epoch per rank.  A 6250-row
    dataset gives one rank that epoch length; 48 steps as chained graph replays (two epoch
    boundaries inside chains, no host work between them) are bit-identical to 48 eager steps."""
    B = 256
    data, labels = _synthetic(6250, seed=15)
    kw = dict(seed=16, lr=1e-4, relu_logits=False)
    a = FusedCifarEngine(B, data, labels, **kw)
    b = FusedCifarEngine(B, data, labels, **kw)
    assert a.period == 24
    a.step()
    a.capture()
    a.run(47)
    for _ in range(48):
        b.step()
    torch.cuda.synchronize()
    assert a.global_step() == b.global_step() == 48
    assert torch.isfinite(a.flat_params()).all()
    assert torch.equal(a.flat_params(), b.flat_params())


@pytest.mark.parametrize("B", [1, 2, 100, 127])
def test_any_batch_size_masked_tail(B):
    """Batches that are not a multiple of the 16-row tile: the kernels run on the padded batch, the
    head gives padding rows zero weight -- gradients, loss and accuracy are those of the B real rows."""
    data, labels = _synthetic(max(512, 4 * B), seed=17)
    eng = FusedCifarEngine(B, data, labels, seed=18, lr=0.01)
    assert eng.Bv == B and eng.B % 16 == 0 and eng.B - B < 16
    idx = eng.batch_indices(0)
    assert idx.numel() == B
    grad = eng.compute_gradients().cpu().clone()
    logits, loss, gref = _ref_grads(eng.flat_params(), data, labels, idx)
    got_logits = eng.forward_logits(idx)
    assert got_logits.shape == (B, 10)
    assert _rel(got_logits, logits) < 1e-2, _rel(got_logits, logits)
    g = gref.cpu()
    cos = float(torch.nn.functional.cosine_similarity(grad, g, dim=0))
    assert cos > 0.995, cos                          # bf16 kernels vs fp32 autograd on the real rows
    # exact masking check: the same real rows in a full 16-row tile (rows repeated, so the batch mean
    # is unchanged) -- padding rows must contribute nothing at all
    Bp = eng.B
    rep = idx.repeat((Bp + B - 1) // B)[:Bp] if Bp % B == 0 else None
    if rep is not None:
        full = FusedCifarEngine(Bp, data, labels, seed=18, lr=0.01)
        gfull = full.compute_gradients(idx=rep).cpu()
        assert _rel(grad, gfull) < 1e-3, _rel(grad, gfull)
    # the masked loss / accuracy in the stats ring are those of the kernel's own logits of the B rows
    y = labels[idx.long()].long().cuda()
    want_loss = float(torch.nn.functional.cross_entropy(got_logits.cuda(), y))
    want_acc = float((got_logits.cuda().argmax(1) == y).float().mean())
    eng.step()
    torch.cuda.synchronize()
    st = eng.read_stats(1)
    assert abs(st["loss"] - want_loss) < 1e-4 * max(1.0, abs(want_loss)), (st, want_loss, float(loss))
    assert abs(st["accuracy"] - want_acc) < 1e-6, (st, want_acc)


@pytest.mark.parametrize("B", [100, 256])
def test_fc1_update_in_gemm_epilogue_is_bit_identical(B):
    """Single GPU: the fc1 weight update runs in the dW1 GEMM's epilogue (c_mode 4) and the SGD kernel
    updates only the fc1 bias; the fc1 shadow is double-buffered by step parity.  After eager and
    graph-replayed steps (odd and even counts, a mid-run set_step, an eval forward) everything equals
    the plain path (fp32 gradient through HBM, fc1 in the SGD kernel) bit for bit."""
    data, labels = _synthetic(8 * B, seed=43)
    kw = dict(seed=44, lr=1e-4, relu_logits=False)
    fused = FusedCifarEngine(B, data, labels, **kw)
    ref = FusedCifarEngine(B, data, labels, **kw, variant={"fc1_epilogue": False})
    assert fused.fc1_epilogue and not ref.fc1_epilogue
    idx = torch.arange(B, dtype=torch.int32)
    for eng in (ref, fused):
        eng.step()
        eng.step()
        eng.capture(steps_per_graph=4)
        eng.run(5)
        eng.set_step(eng.global_step() + 1)     # parity flip from the host
        eng.run(3)
    torch.cuda.synchronize()
    assert ref.global_step() == fused.global_step() == 11
    assert torch.isfinite(ref.master).all()
    assert torch.equal(ref.master, fused.master)
    assert torch.equal(ref.fc1n_current(), fused.fc1n_current())
    w1 = ref.pv["full_weight_1"].view(2304, 384)
    assert torch.equal(fused.fc1n_current(), w1.to(torch.bfloat16))
    assert ref.read_stats(11) == fused.read_stats(11)
    assert torch.equal(ref.forward_logits(idx), fused.forward_logits(idx))


@pytest.mark.parametrize("B", [16, 100, 128, 192, 256, 1024])
def test_sgd_in_wgrad_launch_is_bit_identical(B):
    """Single GPU: the merged weight-gradient launch also runs the SGD (cnn_wgrad.hip apply mode:
    sub-grid barriers per slab family, each block reduces its share of the slabs in the SGD kernel's
    order, the conv1 blocks run the fc roles / stats / global_step / next batch rows) and the step has
    no SGD launch.  After eager and graph-replayed steps (a host set_step in between) the parameters,
    every bf16 shadow, the stats, the step counter and the next batch rows equal the two-launch step
    bit for bit, and no barrier timed out."""
    data, labels = _synthetic(8 * B, seed=45)
    kw = dict(seed=46, lr=1e-4, relu_logits=False)
    fused = FusedCifarEngine(B, data, labels, **kw)
    ref = FusedCifarEngine(B, data, labels, **kw, variant={"wgrad_sgd": False})
    assert fused.wgrad_apply and not ref.wgrad_apply
    idx = torch.arange(min(B, 64), dtype=torch.int32)
    for eng in (ref, fused):
        eng.step()
        eng.step()
        eng.capture(steps_per_graph=4)
        eng.run(5)
        eng.set_step(eng.global_step() + 3)
        eng.run(3)
    torch.cuda.synchronize()
    fused.check_barriers()
    assert int(fused.wbar[320]) == 0
    assert ref.global_step() == fused.global_step() == 13
    assert torch.isfinite(ref.master).all()
    assert torch.equal(ref.master, fused.master)
    for name in ("w1f", "w2f", "w2d", "fc2t", "fc2n", "fc3t", "fc3d", "bidx"):
        assert torch.equal(getattr(ref, name), getattr(fused, name)), name
    assert torch.equal(ref.fc1n_current(), fused.fc1n_current())
    for s in (10, 11, 12, 13):
        assert ref.read_stats(s) == fused.read_stats(s), s
    assert torch.equal(ref.forward_logits(idx), fused.forward_logits(idx))


@pytest.mark.parametrize("B", [16, 100, 256])
def test_conv_grad_reduction_in_wgrad_launch_is_bit_identical(B):
    """Data-parallel / compute_gradients path: the merged weight-gradient launch reduces its own conv
    slabs into the flat gradient (SGD mode 1 inside cnn_wgrad.hip, helpers included) instead of a
    reduce-only SGD launch.  The whole flat gradient equals the two-launch path bit for bit, for the
    generated batch and for an explicit index list."""
    data, labels = _synthetic(8 * B, seed=47)
    kw = dict(seed=48, lr=1e-4, relu_logits=False)
    fused = FusedCifarEngine(B, data, labels, **kw)
    ref = FusedCifarEngine(B, data, labels, **kw, variant={"wgrad_sgd": False})
    assert fused._grad_in_launch and not ref._grad_in_launch
    idx = torch.randperm(8 * B, generator=torch.Generator().manual_seed(3))[:B].to(torch.int32)
    for explicit in (None, idx):
        g_ref = ref.compute_gradients(explicit).clone()
        g_fused = fused.compute_gradients(explicit).clone()
        torch.cuda.synchronize()
        assert torch.isfinite(g_ref).all() and float(g_ref.abs().max()) > 0
        assert torch.equal(g_ref, g_fused)
    fused.check_barriers()


@pytest.mark.parametrize("B", [16, 100, 128, 256])
def test_fc_chain_launch_matches_three_launch_path(B):
    """The persistent fc-chain launch (cnn_fc.hip: fc1 forward + head + fc backward, 256 co-resident
    workgroups, in-launch hand-offs) against the three-launch path (grouped GEMM, head, grouped
    GEMM) on the same weights and batch: loss, accuracy, the conv backward's input dp2 and every
    gradient segment agree to bf16 rounding (the fc1 split-K order differs: 8 slices, not 9)."""
    data, labels = _synthetic(8 * B, seed=61)
    kw = dict(seed=62, lr=1e-4, relu_logits=False)
    fused = FusedCifarEngine(B, data, labels, **kw, variant={"fc_fused": True})
    ref = FusedCifarEngine(B, data, labels, **kw, variant={"fc_fused": False})
    assert fused.fc_fused and not ref.fc_fused
    idx = torch.randperm(8 * B, generator=torch.Generator().manual_seed(5))[:B].to(torch.int32)
    for explicit in (None, idx):
        g_ref = ref.compute_gradients(explicit).clone()
        g_fus = fused.compute_gradients(explicit).clone()
        torch.cuda.synchronize()
        fused.check_barriers()
        n = B // 4
        assert abs(float(fused.loss_part[:n].sum()) - float(ref.loss_part.sum())) <= 1e-3 * max(1.0, float(ref.loss_part.sum()))
        assert int(fused.correct_part[:n].sum()) == int(ref.correct_part.sum())
        assert _rel(fused.dp2[:fused.Bv], ref.dp2[:ref.Bv]) < 2e-2
        for spec in M.PARAM_SPECS:
            sl = slice(spec.offset, spec.offset + spec.numel)
            assert _rel(g_fus[sl], g_ref[sl]) < 2e-2, spec.name
    # counters re-arm: many launches (eager and graph-replayed) keep giving the eager step's weights
    for eng in (fused, ref):
        eng.step()
        eng.capture(steps_per_graph=4)
        eng.run(9)
    torch.cuda.synchronize()
    fused.check_barriers()
    assert _rel(fused.master, ref.master) < 1e-3
    # (the loss after 10 steps at ~18 nats rides on logits in the hundreds: weights within 1e-3 of
    # each other move it by up to ~2 %, depending on where the bf16 roundings of the run fall)
    assert abs(fused.read_stats(10)["loss"] - ref.read_stats(10)["loss"]) < 3e-2 * max(1.0, abs(ref.read_stats(10)["loss"]))


@pytest.mark.parametrize("B", [64, 128])
def test_fused_split_forward_is_bit_identical(B):
    """B <= 128: conv1 -> conv2 forward as ONE launch whose two workgroups per image swap their pool1
    halves in-launch (cnn_split.hip k_conv12_fwd_split) against the two channel-split launches: p1,
    am1, p2, am2, the gradients and the weights after eager + graph-replayed steps are bit-identical
    (the same conv1 / conv2 split bodies; only the hand-off of the pool1 halves differs)."""
    data, labels = _synthetic(8 * B, seed=67)
    kw = dict(seed=68, lr=1e-3, relu_logits=False)
    fused = FusedCifarEngine(B, data, labels, **kw, variant={"fwd12_split": True})
    ref = FusedCifarEngine(B, data, labels, **kw, variant={"fwd12_split": False})
    assert fused.fwd12_split and not ref.fwd12_split and ref.conv_split == 2
    idx = torch.randperm(8 * B, generator=torch.Generator().manual_seed(7))[:B].to(torch.int32)
    for explicit in (None, idx):
        g_ref = ref.compute_gradients(explicit).clone()
        g_fus = fused.compute_gradients(explicit).clone()
        torch.cuda.synchronize()
        fused.check_barriers()
        for name in ("p1", "am1", "p2", "am2"):
            assert torch.equal(getattr(fused, name), getattr(ref, name)), name
        assert torch.equal(g_fus, g_ref)
    for eng in (fused, ref):
        eng.step()
        eng.capture(steps_per_graph=4)
        eng.run(9)
    torch.cuda.synchronize()
    fused.check_barriers()
    assert torch.equal(fused.master, ref.master)
    assert int(fused.c12_flags.abs().sum()) == 0          # every flag re-armed


@pytest.mark.parametrize("B", [64, 256])
def test_fc_sgd_in_chain_is_bit_identical(B):
    """Every fc SGD in the fc chain's dW tile epilogues (fc2 / fc3 / biases too, variant fc_sgd_in_chain)
    vs as SGD roles of the wgrad launch: parameters, every shadow and the stats bit for bit after eager
    and graph-replayed steps."""
    data, labels = _synthetic(8 * B, seed=73)
    kw = dict(seed=74, lr=1e-3, relu_logits=False)
    on = FusedCifarEngine(B, data, labels, **kw, variant={"fc_sgd_in_chain": True})
    off = FusedCifarEngine(B, data, labels, **kw, variant={"fc_sgd_in_chain": False})
    assert on.fc_sgd_in_chain and not off.fc_sgd_in_chain
    for eng in (on, off):
        eng.step()
        eng.capture(steps_per_graph=4)
        eng.run(6)
    torch.cuda.synchronize()
    on.check_barriers()
    assert torch.equal(on.master, off.master)
    for name in ("fc2t", "fc2n", "fc3t", "fc3d", "w1f", "w2f", "w2d"):
        assert torch.equal(getattr(on, name), getattr(off, name)), name
    assert torch.equal(on.fc1n_current(), off.fc1n_current())
    assert torch.equal(on.stats, off.stats)


@pytest.mark.parametrize("B", [64, 128, 160, 256])
def test_dgrad_in_fc_chain_is_bit_identical(B):
    """The conv2 input gradient inside the fc chain launch (each workgroup's image -- at B <= 128 each
    pair of workgroups' image halves, as the split dgrad launch -- once its dp2 row tile's 18 column
    tasks have published) against the separate dgrad launch: dP1, dY2, every gradient segment and the
    weights after eager + graph-replayed steps are bit-identical (the same device function on the
    same operands; only the hand-off differs)."""
    data, labels = _synthetic(8 * B, seed=63)
    kw = dict(seed=64, lr=1e-3, relu_logits=False)
    fused = FusedCifarEngine(B, data, labels, **kw, variant={"fc_dgrad": True})
    ref = FusedCifarEngine(B, data, labels, **kw, variant={"fc_dgrad": False})
    assert fused.fc_dgrad and not ref.fc_dgrad
    idx = torch.randperm(8 * B, generator=torch.Generator().manual_seed(6))[:B].to(torch.int32)
    for explicit in (None, idx):
        g_ref = ref.compute_gradients(explicit).clone()
        g_fus = fused.compute_gradients(explicit).clone()
        torch.cuda.synchronize()
        fused.check_barriers()
        assert torch.equal(fused.dp2, ref.dp2)
        assert torch.equal(fused.dy2, ref.dy2)
        assert torch.equal(fused.dp1, ref.dp1)
        assert torch.equal(g_fus, g_ref)
    for eng in (fused, ref):
        eng.step()
        eng.capture(steps_per_graph=4)
        eng.run(9)
    torch.cuda.synchronize()
    fused.check_barriers()
    assert torch.equal(fused.master, ref.master)


@pytest.mark.parametrize("B", [128, 256])
def test_fc_dw_tiles_in_wgrad_launch_are_bit_identical(B):
    """The fc weight-gradient tiles + every fc SGD epilogue run in the wgrad launch's conv1 blocks
    (variant fc_dw_in_wgrad) or in the fc chain: every epilogue applies the SGD kernel's expression,
    so the weights after eager + graph-replayed steps are bit-identical either way."""
    data, labels = _synthetic(8 * B, seed=65)
    kw = dict(seed=66, lr=1e-3, relu_logits=False)
    engs = []
    for v in (True, False):
        engs.append(FusedCifarEngine(B, data, labels, **kw, variant={"fc_dw_in_wgrad": v}))
    assert engs[0].fc_dw_in_wgrad and not engs[1].fc_dw_in_wgrad
    for eng in engs:
        eng.step()
        eng.capture(steps_per_graph=4)
        eng.run(7)
    torch.cuda.synchronize()
    for eng in engs:
        eng.check_barriers()
    assert torch.isfinite(engs[0].master).all()
    assert torch.equal(engs[0].master, engs[1].master)


def test_fc_chain_graph_replay_is_deterministic():
    """Two engines, same seed, same steps through the persistent fc chain: bit-identical weights
    (fixed-order split-K sums, no atomics on data)."""
    data, labels = _synthetic(2048, seed=71)
    engs = [FusedCifarEngine(256, data, labels, seed=72, lr=1e-3) for _ in range(2)]
    for eng in engs:
        assert eng.fc_fused
        eng.step()
        eng.capture(steps_per_graph=8)
        eng.run(23)
    torch.cuda.synchronize()
    assert torch.equal(engs[0].master, engs[1].master)
    assert engs[0].read_stats(24) == engs[1].read_stats(24)


@pytest.mark.parametrize("B", [144, 256])
def test_xraw_prefetch_is_bit_identical(B):
    """r5: the training forward reads its raw images from xraw, gathered for it by the previous step's
    finalizer (the wgrad launch's conv1 blocks on one GPU), instead of index -> image loads.  Chained
    graph replays across an epoch boundary, a host set_step, an explicit-index compute_gradients()
    and an evaluation in between: weights and stats equal the gathering forward bit for bit."""
    data, labels = _synthetic(3 * B, seed=81)          # 3 steps per epoch: the chains cross epochs
    kw = dict(seed=82, lr=1e-4, relu_logits=False)
    pre = FusedCifarEngine(B, data, labels, **kw)
    ref = FusedCifarEngine(B, data, labels, **kw, variant={"xraw_prefetch": False})
    assert pre.xraw_prefetch and not ref.xraw_prefetch
    idx = torch.randperm(3 * B, generator=torch.Generator().manual_seed(7))[:B].to(torch.int32)
    for eng in (pre, ref):
        eng.step()
        eng.capture(steps_per_graph=4)
        eng.run(5)
        eng.compute_gradients(idx)
        eng.evaluate(data[:B], labels[:B])
        eng.run(3)
        eng.set_step(eng.global_step() + 1)
        eng.run(4)
    torch.cuda.synchronize()
    assert pre.global_step() == ref.global_step() == 14
    assert torch.isfinite(ref.master).all()
    assert torch.equal(pre.master, ref.master)
    # the prefetching engine's xraw already holds the NEXT step's images (its bidx rows)
    assert torch.equal(pre.xraw, pre.data[pre.bidx.long()].view(pre.B, 3072))
    assert torch.equal(pre.bidx, ref.bidx)
    for s in (9, 14):
        assert pre.read_stats(s) == ref.read_stats(s), s


_SPIN0 = "spin0:-DDMLC_SPIN_LIMIT=0"
_SPIN0_SCRIPT = r"""
import json, sys, torch
sys.path.insert(0, sys.argv[1])
import dmlc  # noqa: F401
from dmlc.engine.fused import FusedCifarEngine
B = int(sys.argv[2])
g = torch.Generator().manual_seed(0)
x = torch.randint(0, 256, (4 * B, 32, 32, 3), dtype=torch.uint8, generator=g)
y = torch.randint(0, 10, (4 * B,), dtype=torch.int32, generator=g)
eng = FusedCifarEngine(B, x, y, device="cuda", lr=1e-4, relu_logits=False)
flags = {"fc_fused": eng.fc_fused, "wgrad_apply": eng.wgrad_apply, "fwd12_split": eng.fwd12_split}
for _ in range(3):
    eng.step()
torch.cuda.synchronize()
word = int(eng.wbar[320])
try:
    eng.check_barriers()
    msg = ""
except RuntimeError as e:
    msg = str(e)
print(json.dumps({"flags": flags, "word": word, "msg": msg, "flags_rezeroed": int(eng.c12_flags.abs().sum())}))
"""


def _spin0(B, **env):
    import json
    import os
    import subprocess
    import sys
    from dmlc import _build
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(_build.LIB_DIR, "libdmlc_hip_spin0.so")
    if not os.path.exists(lib):
        pytest.skip("diagnostic library not built: DMLC_VARIANT='" + _SPIN0 + "' python -c 'import __graft_entry__'"
                    " ... _build.build()")
    r = subprocess.run([sys.executable, "-c", _SPIN0_SCRIPT, repo, str(B)], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, DMLC_VARIANT=_SPIN0, **env))
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("B", [256, 64])
def test_forced_spin_timeouts_name_kernel_and_switch(B):
    """Round-6 hardening: a diagnostic build whose in-launch waits give up at the first
    unsatisfied poll (-DDMLC_SPIN_LIMIT=0: the wgrad sub-grid barriers, the fc chain seams, the split
    forward's flags) drives the REAL timeout paths.  The sticky error word then carries the wgrad bit
    (1) and the hand-off bit (2), check_barriers() names the kernels and the environment switch that
    turns each persistent launch off -- and with those three switches set the same library runs the
    step with no wait left to time out (error word 0).  The kernels then read partial data: the
    weights are garbage, which is what the error reports."""
    got = _spin0(B)
    f = got["flags"]
    assert f["fc_fused"] and f["wgrad_apply"] and f["fwd12_split"] == (B <= 128), got
    assert got["word"] & 1 and got["word"] & 2, got
    m = got["msg"]
    assert "k_wgrad" in m and "DMLC_WGRAD_SGD=0" in m, m
    assert "k_fc_chain" in m and "DMLC_FC_FUSED=0" in m and "DMLC_FWD12_SPLIT=0" in m, m
    assert got["flags_rezeroed"] == 0, got                 # check_barriers re-armed the split flags
    off = _spin0(B, DMLC_FC_FUSED="0", DMLC_WGRAD_SGD="0", DMLC_FWD12_SPLIT="0")
    assert not any(off["flags"].values()), off
    assert off["word"] == 0 and off["msg"] == "", off
