"""Fused ResNet-20 HIP kernels (csrc/kernels/resnet.hip) vs the fp32 PyTorch model (models/resnet.py,
train-mode BatchNorm): forward logits, every parameter gradient, one SGD step incl. BN running
statistics, graph replay vs eager launches, and a short convergence run."""
import pytest
import torch
import torch.nn.functional as F

from dmlc.data.cifar import synthetic
from dmlc.engine.fused_resnet import FusedResNetEngine
from dmlc.models import resnet as R

pytestmark = pytest.mark.gpu


def _data(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, generator=g),
            torch.randint(0, 10, (n,), dtype=torch.int32, generator=g))


def _ref(flat, state, data, labels, idx):
    dev = "cuda"
    flat = flat.to(dev).clone().requires_grad_(True)
    st = state.to(dev).clone()
    x = data[idx.long()].to(dev).float()
    logits = R.resnet20_forward(x, R._views(flat, R.PARAM_SPECS), R._views(st, R.STATE_SPECS), training=True)
    loss = F.cross_entropy(logits, labels[idx.long()].to(dev).long())
    loss.backward()
    return logits.detach(), loss.detach(), flat.grad.detach().cpu(), st.cpu()


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def local_layer_errors(eng, data, labels, idx):
    """Per-kernel numerics: every fused kernel's output vs fp32 PyTorch ops fed with the fused
    engine's OWN inputs for that kernel (so bf16 error does not compound across 19 layers and ReLU
    mask flips cannot occur).  Call after ``eng.compute_gradients()``.  Returns {check: rel error}."""
    from dmlc.engine.fused_resnet import LAYERS, _block_sc_mode
    dev = eng.device
    P = {s.name[len(R.SCOPE) + 1:]: s for s in R.PARAM_SPECS}
    flat = eng.flat_params().to(dev)
    grad = eng.grad
    f = lambda t: t.float().permute(0, 3, 1, 2)          # NHWC bf16 -> NCHW fp32
    out = {}
    ximg = data[idx.long()].to(dev).float().permute(0, 3, 1, 2)

    def bn_train(z, name):
        g = flat[P[f"{name}/bn/gamma"].offset:][:z.shape[1]].clone().requires_grad_(True)
        b = flat[P[f"{name}/bn/beta"].offset:][:z.shape[1]].clone().requires_grad_(True)
        return F.batch_norm(z, None, None, g, b, training=True, eps=R.BN_EPS), g, b

    for l, (name, ci, co, h, s) in enumerate(LAYERS):
        spec = P[f"{name}/conv/kernel"]
        w = flat[spec.offset:spec.offset + spec.numel].view(spec.shape).clone().requires_grad_(True)
        x = (ximg if l == 0 else f(eng.a[l - 1])).clone().requires_grad_(True)
        z = R._conv3x3(x, w, s)
        out[f"fwd{l}"] = _rel(f(eng.z[l]), z)
        y, g, b = bn_train(f(eng.z[l]), name)
        y.backward(f(eng.gy[l]))
        zz = f(eng.z[l]).detach().requires_grad_(True)
        yz, _, _ = bn_train(zz, name)
        yz.backward(f(eng.gy[l]))
        z2 = R._conv3x3(x, w, s)
        z2.backward(zz.grad)
        out[f"wgrad{l}"] = _rel(grad[spec.offset:spec.offset + spec.numel].view(spec.shape), w.grad)
        out[f"gamma{l}"] = _rel(grad[P[f"{name}/bn/gamma"].offset:][:co], g.grad)
        out[f"beta{l}"] = _rel(grad[P[f"{name}/bn/beta"].offset:][:co], b.grad)
        if l == 0:
            continue
        ga = x.grad.clone()
        if l % 2 == 1:                                   # a-conv: + shortcut gradient of its block
            gsc = f(eng.gy[l + 1])
            if _block_sc_mode(l + 1) == 2:
                up = torch.zeros_like(ga)
                up[:, :, ::2, ::2] = gsc[:, :ci]
                gsc = up
            ga = ga + gsc
        gy_prev = ga * (f(eng.a[l - 1]) > 0).float()
        out[f"dgrad{l}"] = _rel(f(eng.gy[l - 1]), gy_prev)
    # head: BN_18 + residual + ReLU + pool + fc + xent -> g_y18
    z18 = f(eng.z[18])
    y18, _, _ = bn_train(z18, LAYERS[18][0])
    y18 = y18.detach().requires_grad_(True)
    a18 = F.relu(y18 + f(eng.a[16]))
    fw = flat[P["fc/weights"].offset:][:640].view(64, 10)
    fb = flat[P["fc/biases"].offset:][:10]
    logits = a18.mean(dim=(2, 3)) @ fw + fb
    F.cross_entropy(logits, labels[idx.long()].to(dev).long()).backward()
    out["head"] = _rel(f(eng.gy[18]), y18.grad)
    return out


@pytest.mark.parametrize("B", [16, 128])
def test_forward_logits_match_reference(B):
    data, labels = _data(2 * B)
    eng = FusedResNetEngine(B, data, labels, seed=1)
    idx = torch.randperm(data.shape[0])[:B].to(torch.int32)
    got = eng.forward_logits(idx).cpu()
    ref, loss, _, _ = _ref(eng.flat_params(), eng.state.cpu(), data, labels, idx)
    assert _rel(got, ref.cpu()) < 5e-2, _rel(got, ref.cpu())
    # per-image loss / accuracy published by the head kernel
    assert abs(float(eng.loss_img.mean()) - float(loss)) < 5e-2 * max(1.0, float(loss))


@pytest.mark.parametrize("B", [32, 128])
def test_each_kernel_matches_fp32_ops(B):
    data, labels = _data(4 * B, seed=3)
    eng = FusedResNetEngine(B, data, labels, seed=2)
    idx = eng.batch_indices(eng.host_step)
    eng.compute_gradients()
    errs = local_layer_errors(eng, data, labels, idx)
    bad = {k: v for k, v in errs.items() if v > 3e-2}
    assert not bad, bad


def test_end_to_end_gradients_close_to_fp32_model():
    """End to end the bf16 forward drifts ~2-3 % by layer 18, which flips a few ReLU masks, so the
    deepest gradients agree only to cos ~0.95; this pins that level (a wrong kernel gives ~0)."""
    B = 64
    data, labels = _data(4 * B, seed=3)
    eng = FusedResNetEngine(B, data, labels, seed=2)
    idx = eng.batch_indices(eng.host_step)
    grad = eng.compute_gradients().cpu()
    _, _, gref, _ = _ref(eng.flat_params(), eng.state.cpu(), data, labels, idx)
    cos = float(F.cosine_similarity(grad, gref, dim=0))
    assert cos > 0.9, cos
    for s in R.PARAM_SPECS:
        a, b = grad[s.offset:s.offset + s.numel], gref[s.offset:s.offset + s.numel]
        assert float(F.cosine_similarity(a, b, dim=0)) > 0.8, s.name


def test_sgd_step_and_bn_running_stats():
    B = 64
    data, labels = _data(4 * B, seed=5)
    eng = FusedResNetEngine(B, data, labels, seed=4, lr=0.05)
    before, st0 = eng.flat_params().clone(), eng.state.cpu().clone()
    idx = eng.batch_indices(eng.host_step)
    eng.step()
    torch.cuda.synchronize()
    _, loss, gref, st_ref = _ref(before, st0, data, labels, idx)
    assert eng.global_step() == 1
    st = eng.read_stats(1)
    assert abs(st["loss"] - float(loss)) / max(1.0, float(loss)) < 5e-2
    delta, dref = eng.flat_params() - before, -0.05 * gref
    assert float(F.cosine_similarity(delta, dref, dim=0)) > 0.98
    assert _rel(eng.state.cpu(), st_ref) < 2e-2


@pytest.mark.parametrize("B", [32, 256])
def test_graph_replay_matches_eager_launches_bitwise(B):
    """Deterministic BN statistics (fixed-point slots added with integer atomics): chained graph
    replays == eager launches bit for bit -- weights, BN moving statistics and published losses --
    across 10 steps (SURVEY.md §5.2 determinism goal)."""
    data, labels = _data(8 * B, seed=7)
    e1 = FusedResNetEngine(B, data, labels, seed=6, lr=0.02)
    e2 = FusedResNetEngine(B, data, labels, seed=6, lr=0.02)
    e2.capture()
    for _ in range(10):
        e1.step()
    e2.run(10)
    torch.cuda.synchronize()
    assert e1.global_step() == e2.global_step() == 10
    assert torch.equal(e2.flat_params(), e1.flat_params())
    assert torch.equal(e2.state, e1.state)
    assert [e1.read_stats(k) for k in range(1, 11)] == [e2.read_stats(k) for k in range(1, 11)]


def test_fixed_point_bn_sums_match_activations():
    """The fixed-point slot totals (integer atomics, resnet.hip fx_add) equal an fp64 sum of the stored
    pre-BN activations per channel, up to their bf16 rounding."""
    B = 64
    data, labels = _data(4 * B, seed=9)
    eng = FusedResNetEngine(B, data, labels, seed=8)
    eng.compute_gradients()
    torch.cuda.synchronize()
    sums = eng.bn_sums().cpu()
    assert torch.isfinite(sums).all()
    for l in (0, 7, 18):
        z = eng.z[l].double().cpu()
        co = z.shape[-1]
        s1, s2 = z.sum((0, 1, 2)), (z * z).sum((0, 1, 2))
        assert _rel(sums[0, l, :co], s1) < 2e-2, l
        assert _rel(sums[0, l, 64:64 + co], s2) < 2e-2, l
        if co < 64:
            assert float(sums[0, l, co:64].abs().max()) == 0.0


def test_short_training_reduces_loss():
    B = 128
    data, labels = synthetic(32 * B, seed=11, learnable=True)
    eng = FusedResNetEngine(B, data, labels, seed=3, lr=0.05, staircase=False)
    eng.capture()
    eng.run(150)
    torch.cuda.synchronize()
    first = sum(eng.read_stats(k)["loss"] for k in range(1, 11)) / 10
    last = sum(eng.read_stats(k)["loss"] for k in range(141, 151)) / 10
    assert last < 0.8 * first, (first, last)
    acc = eng.evaluate(data[:1024], labels[:1024])
    assert 0.0 <= acc <= 1.0


def test_cli_fused_resnet20_checkpoint_resume(tmp_path):
    """cifar10cnn.py --model=resnet20 on the GPU picks the fused engine; the checkpoint holds the
    parameters + BN moving statistics under the eager model's names, and a rerun resumes from it."""
    import os
    import subprocess
    import sys
    from dmlc import checkpoint as CK
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(repo, "cifar10cnn.py"), "--model=resnet20", "--synthetic",
           "--synthetic_size=1024", "--batch_size=64", "--generations=6", "--output_every=3", "--eval_every=6",
           "--eval_batches=2", "--learning_rate=0.05", f"--log_dir={tmp_path}"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "engine=fused model=resnet20" in r.stdout, r.stdout[-2000:]
    t = CK.read_bundle(CK.latest_checkpoint(str(tmp_path)))
    assert int(t["global_step"]) == 6
    m = R.ResNet20()
    assert CK.load_module_tensors(m, t) == 6
    mv = t["resnet20/stem/bn/moving_variance"]
    assert not torch.allclose(mv, torch.ones_like(mv))          # running stats were updated and saved
    r2 = subprocess.run(cmd[:-6] + ["--generations=9", "--output_every=3", "--eval_every=100", "--eval_batches=1",
                                    "--learning_rate=0.05", f"--log_dir={tmp_path}"],
                        stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r2.returncode == 0 and "Restored" in r2.stdout, r2.stdout[-3000:]
    assert int(CK.read_bundle(CK.latest_checkpoint(str(tmp_path)))["global_step"]) == 9


def test_merged_backward_launch_matches_separate_launches():
    """rn_bwd (dgrad_l + wgrad_l as one launch, block roles) computes the same gradients as the two
    separate launches (up to the order of the fp64 BN-statistics atomics)."""
    B = 32
    data, labels = _data(4 * B, seed=13)
    merged = FusedResNetEngine(B, data, labels, seed=12)
    assert merged.merged_bwd and not merged.wgrad_branch
    g_m = merged.compute_gradients().cpu().clone()
    split = FusedResNetEngine(B, data, labels, seed=12, merged_bwd=False)
    assert not split.merged_bwd
    g_s = split.compute_gradients().cpu().clone()
    assert _rel(g_m, g_s) < 1e-4, _rel(g_m, g_s)
    for lm, ls in zip(merged.part, split.part):
        assert _rel(lm, ls) < 1e-3


def test_branch_sgd_split_equals_single_sgd_launch():
    """The layer-range SGD launches on a graph branch (stage 3 after its last backward launch, stage
    2 after its) + the tail SGD give bitwise the same parameters, BN state and step as one SGD
    launch, eagerly and under graph replay."""
    B = 32
    data, labels = _data(8 * B, seed=21)
    split = FusedResNetEngine(B, data, labels, seed=5, lr=0.01, sgd_split=True)
    assert split.sgd_split
    one = FusedResNetEngine(B, data, labels, seed=5, lr=0.01)
    assert not one.sgd_split
    for e in (split, one):
        for _ in range(3):
            e.step()
        e.capture()
        for _ in range(4):
            e.step()
    torch.cuda.synchronize()
    assert split.global_step() == one.global_step() == 7
    assert torch.equal(split.master, one.master)
    assert torch.equal(split.state, one.state)


@pytest.mark.parametrize("B", [20, 1, 100])
def test_any_batch_size_masked_tail(B):
    """Any batch size (BASELINE config 4 at the reference's arbitrary BATCH_SIZE): the kernels run on the
    batch padded to 16 images; the padding images must not enter any BatchNorm statistic and must get
    exactly zero gradient.  Checked: g_y of every padding image is exactly 0 at every layer; logits,
    loss, gradients and the BN running statistics of one step agree with the fp32 eager model at batch B."""
    data, labels = _data(4 * max(B, 16), seed=31)
    eng = FusedResNetEngine(B, data, labels, seed=7, lr=0.05)
    assert eng.Bv == B and eng.B % 16 == 0 and eng.B >= B
    idx = eng.batch_indices(eng.host_step)
    assert idx.numel() == B
    got = eng.forward_logits(idx).cpu()
    ref_logits, loss, gref, _ = _ref(eng.flat_params(), eng.state.cpu(), data, labels, idx)
    assert got.shape == (B, 10)
    assert _rel(got, ref_logits.cpu()) < 5e-2, _rel(got, ref_logits.cpu())
    grad = eng.compute_gradients().cpu()
    for l in range(len(eng.gy)):
        assert int(eng.gy[l][B:].float().abs().sum()) == 0, l
    cos = float(F.cosine_similarity(grad, gref, dim=0))
    assert cos > 0.9, cos
    before, st0 = eng.flat_params().clone(), eng.state.cpu().clone()
    eng.step()
    torch.cuda.synchronize()
    st = eng.read_stats(1)
    assert abs(st["loss"] - float(loss)) / max(1.0, float(loss)) < 5e-2, (st, float(loss))
    _, _, _, st_ref = _ref(before, st0, data, labels, idx)
    assert _rel(eng.state.cpu(), st_ref) < 2e-2


@pytest.mark.parametrize("B,level", [(32, 1), (256, 1), (64, 2), (256, 2)])
def test_per_image_backward_is_bit_identical(B, level):
    """The stride-1 layers' dgrad + wgrad from one workgroup per image (k_rn_bwd_img: the staged g_z and
    layer input serve both, one weight-gradient slab per image; level 1: the 16->16 layers, level 2:
    also the 32->32 ones) train exactly like the merged launch with separate wgrad blocks over the
    same slabs (bwd_img_level=0): the same per-image sums in the same k-step order, so parameters,
    BN state and stats agree bit for bit after eager and graph-replayed steps."""
    data, labels = _data(4 * B, seed=31)
    img = FusedResNetEngine(B, data, labels, seed=30, bwd_img_level=level)
    assert all(img._per_image(l) for l in range(1, 7))
    assert all(img._per_image(l) for l in (8, 9, 10, 11, 12)) == (level == 2)
    ref = FusedResNetEngine(B, data, labels, seed=30, groups=list(img.groups), bwd_img_level=0)
    assert not any(ref._per_image(l) for l in range(1, 7))
    for eng in (ref, img):
        eng.step()
        eng.capture(steps_per_graph=2)
        eng.run(3)
    torch.cuda.synchronize()
    assert ref.global_step() == img.global_step() == 4
    assert torch.isfinite(ref.master).all()
    assert torch.equal(ref.master, img.master)
    assert torch.equal(ref.state, img.state)
    assert ref.read_stats(4) == img.read_stats(4)
