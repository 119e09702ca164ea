"""Per-kernel numerics of the fused CIFAR-10 CNN step (csrc/kernels/cnn_*.hip).

Every kernel's output is compared with fp32 PyTorch ops fed with THAT kernel's own inputs (the bf16
activations the previous kernel wrote, the bf16 weight shadows the kernels read), so bf16 error does
not compound along the step and ReLU / max-pool decisions cannot flip between the two sides.  What
remains is the kernel's own rounding (bf16 outputs, fp32 accumulation order): ~2e-3 expected,
1e-2 asserted.  The layers are the reference model's (/root/reference/cifar10cnn.py:94-176)."""
import json
import os

import pytest
import torch
import torch.nn.functional as F

from dmlc.engine.fused import FusedCifarEngine
from dmlc.models import cifar_cnn as M

pytestmark = pytest.mark.gpu
TOL = 1e-2


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _pool_bwd(dp, am, H):
    """TF-SAME 3x3/2 max-pool backward through the kernel's argmax bytes (255 = no gradient)."""
    B, HO, _, C = dp.shape
    out = torch.zeros(B, 2 * HO + 1, 2 * HO + 1, C, device=dp.device)
    dp = dp.float()
    for d in range(9):
        dy, dx = divmod(d, 3)
        out[:, dy:dy + 2 * HO:2, dx:dx + 2 * HO:2, :] += dp * (am == d)
    return out[:, :H, :H, :]


def cnn_local_errors(eng, data, labels, idx):
    """{check: rel error} for every kernel of one training step on dataset rows ``idx``."""
    dev = eng.device
    B = eng.Bv
    eng.keep_dp1 = True                  # the fused dgrad keeps dp1 in LDS unless asked for a copy
    eng.compute_gradients(idx=idx)
    torch.cuda.synchronize()
    flat = eng.flat_params().to(dev)
    bfw = {k: v.to(torch.bfloat16).float() for k, v in M.views(flat).items()}    # what the kernels read
    p = M.views(flat)
    g = M.views(eng.grad)
    nchw = lambda t: t.float().permute(0, 3, 1, 2)
    nhwc = lambda t: t.permute(0, 2, 3, 1)
    out = {}
    o = eng.cy
    x = data[idx.long()].to(dev)[:, o:o + 24, o:o + 24, :].float()

    # conv12_fwd: conv1 + ReLU + pool1, then conv2 + ReLU + pool2 from the kernel's own p1
    w1 = bfw["conv1_kernel"].permute(3, 2, 0, 1)
    w2 = bfw["conv2_kernel"].permute(3, 2, 0, 1)
    y1 = F.relu(F.conv2d(nchw(x), w1, p["conv1_bias"], padding=2))
    out["conv1_fwd"] = _rel(nchw(eng.p1[:B]), M.tf_same_maxpool_3x3s2(y1))
    p1 = nchw(eng.p1[:B])
    y2 = F.relu(F.conv2d(p1, w2, p["conv2_bias"], padding=2))
    out["conv2_fwd"] = _rel(nchw(eng.p2[:B]), M.tf_same_maxpool_3x3s2(y2))
    # argmax bytes: 255 exactly where the pooled (post-ReLU) value is 0
    out["argmax_mask"] = float(((eng.am2[:B] == 255) != (eng.p2[:B] == 0)).float().mean())

    # fc1 forward (split-K partial slabs, summed by the head)
    p2 = eng.p2[:B].reshape(B, 2304).float()
    # fc1 split-K partials: the persistent fc chain's (8 slices) or the grouped GEMM's
    h1pre = (eng.h1part8 if eng.fc_fused else eng.h1part)[:, :B].sum(0)
    out["fc1_fwd"] = _rel(h1pre, p2 @ bfw["full_weight_1"])

    # head: fc1 bias+ReLU, fc2, fc3 (+ReLU logits), softmax-xent, dlogits, dh2, dh1
    h1 = eng.h1[:B].float()
    h2 = eng.h2[:B].float()
    dl = eng.dl[:B, :10].float()
    dh2 = eng.dh2[:B].float()
    out["head_h1"] = _rel(h1, F.relu(h1pre + p["full_bias_1"]))
    out["head_h2"] = _rel(h2, F.relu(h1 @ bfw["full_weight_2"] + p["full_bias_2"]))
    logits = (h2 @ bfw["full_weight_3"] + p["full_bias_3"]).detach().requires_grad_(True)
    lg = F.relu(logits) if eng.relu_logits else logits
    y = labels[idx.long()].to(dev).long()
    loss = F.cross_entropy(lg, y)
    loss.backward()
    out["head_dlogits"] = _rel(dl, logits.grad)
    out["head_loss"] = abs(float(eng.loss_part.sum()) / B - float(loss)) / max(1.0, abs(float(loss)))
    out["head_dh2"] = _rel(dh2, (dl @ bfw["full_weight_3"].t()) * (h2 > 0))
    dh1 = eng.dh1[:B].float()
    out["head_dh1"] = _rel(dh1, (dh2 @ bfw["full_weight_2"].t()) * (h1 > 0))

    # grouped fc backward GEMM: dp2 and the fc weight / bias gradients
    out["fc1_dgrad"] = _rel(eng.dp2[:B].reshape(B, 2304), dh1 @ bfw["full_weight_1"].t())
    out["fc1_wgrad"] = _rel(g["full_weight_1"], p2.t() @ dh1)
    out["fc2_wgrad"] = _rel(g["full_weight_2"], h1.t() @ dh2)
    out["fc3_wgrad"] = _rel(g["full_weight_3"], h2.t() @ dl)
    out["fc1_bgrad"] = _rel(g["full_bias_1"], dh1.sum(0))
    out["fc2_bgrad"] = _rel(g["full_bias_2"], dh2.sum(0))
    out["fc3_bgrad"] = _rel(g["full_bias_3"], dl.sum(0))

    # conv2_dgrad: pool2/ReLU backward (-> dy2) and the conv2 input gradient (-> dp1)
    dy2_ref = _pool_bwd(eng.dp2[:B], eng.am2[:B], 12)
    out["pool2_bwd"] = _rel(eng.dy2[:B].view(B, 12, 12, 64), dy2_ref)
    dy2 = nchw(eng.dy2[:B].view(B, 12, 12, 64))
    xin = p1.clone().requires_grad_(True)
    wv = w2.clone().requires_grad_(True)
    F.conv2d(xin, wv, None, padding=2).backward(dy2)
    out["conv2_dgrad"] = _rel(nchw(eng.dp1[:B]), xin.grad)

    # wgrad: conv2 weight/bias gradients from the kernel's p1 and dy2; conv1 from its dp1 / am1
    out["conv2_wgrad"] = _rel(g["conv2_kernel"], wv.grad.permute(2, 3, 1, 0))
    out["conv2_bgrad"] = _rel(g["conv2_bias"], dy2.sum((0, 2, 3)))
    dy1 = nchw(_pool_bwd(eng.dp1[:B], eng.am1[:B], 24).to(torch.bfloat16))   # the kernel keeps dY1 in bf16
    xv = nchw(x).requires_grad_(False)
    w1v = w1.clone().requires_grad_(True)
    F.conv2d(xv, w1v, None, padding=2).backward(dy1)
    out["conv1_wgrad"] = _rel(g["conv1_kernel"], w1v.grad.permute(2, 3, 1, 0))
    out["conv1_bgrad"] = _rel(g["conv1_bias"], dy1.sum((0, 2, 3)))

    # sgd (apply mode from the flat gradient): fp32 master update + every bf16 shadow refreshed
    lr = eng.lr0
    want = flat - lr * eng.grad
    eng._sgd(mode=2)
    torch.cuda.synchronize()
    new = M.views(eng.master)
    out["sgd_master"] = _rel(eng.master, want)
    nb = {k: v.to(torch.bfloat16) for k, v in new.items()}
    out["sgd_shadows"] = max(
        _rel(eng.fc1n_current(), nb["full_weight_1"]), _rel(eng.fc2n, nb["full_weight_2"]),
        _rel(eng.fc2t, nb["full_weight_2"].t()), _rel(eng.fc3t[:10], nb["full_weight_3"].t()),
        _rel(eng.w2f.view(64, 25, 64), nb["conv2_kernel"].reshape(25, 64, 64).permute(2, 0, 1)))
    return out


# (batch, ReLU on the logits, conv_split, conv1_split): the channel-split kernels (cnn_split.hip) at
# the reference batch 128 and below / at 256 / with a masked tail (100), and the one-workgroup-per-
# image kernels (cnn_conv.hip) they replace at small batches
@pytest.mark.parametrize("B,relu_logits,split,split1", [
    (64, True, 2, 4), (128, False, 2, 4), (128, True, 2, 2), (256, False, 2, 2),
    (100, False, 2, 2), (256, False, 1, 2), (128, False, 1, 2)])
def test_every_kernel_matches_fp32_on_its_own_inputs(B, relu_logits, split, split1):
    g = torch.Generator().manual_seed(3)
    data = torch.randint(0, 256, (2048, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (2048,), dtype=torch.int32, generator=g)
    eng = FusedCifarEngine(B, data, labels, seed=4, lr=0.01, relu_logits=relu_logits, conv_split=split,
                           conv1_split=split1)
    idx = eng.batch_indices(0)
    errs = cnn_local_errors(eng, data, labels, idx)
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/cnn_local_errors_b{B}_s{split}{split1}.json", "w") as f:
        json.dump({k: float(f"{v:.3e}") for k, v in errs.items()}, f, indent=1)
    assert errs["argmax_mask"] == 0.0
    bad = {k: v for k, v in errs.items() if not v <= TOL}
    assert not bad, (bad, errs)
    assert errs["sgd_master"] < 1e-6 and errs["head_loss"] < 1e-4, errs


@pytest.mark.parametrize("relu_logits,lr", [(True, 1e-5), (False, 1e-4)])
def test_training_curve_fused_bf16_tracks_eager_fp32(relu_logits, lr):
    """300 training steps on learnable synthetic data: the fused bf16 engine and the eager fp32
    PyTorch engine start from the same weights and see the same batches (the generated order is
    shared); their loss curves must stay within 8 % of each other (25-step windows).  With linear
    logits both must learn (last window below chance, ln 10).  With the reference's ReLU on the
    logits (D4) and its raw 0..255 pixels, BOTH engines collapse to chance within ~50 steps at every
    learning rate tried (1e-5 .. 2e-4, profiles/r2_curve_parity.txt) -- parity is asserted through
    the collapse, and the loss must still fall from its start."""
    from dmlc.data import synthetic
    from dmlc.engine.eager import EagerTrainer
    B, steps, win = 128, 300, 25
    data, labels = synthetic(8192, seed=5, learnable=True)
    kw = dict(seed=6, lr=lr, relu_logits=relu_logits, staircase=False)
    fused = FusedCifarEngine(B, data, labels, **kw)
    fused.step()
    fused.capture()
    fused.run(steps - 1)
    torch.cuda.synchronize()
    lf = torch.tensor([fused.read_stats(k)["loss"] for k in range(1, steps + 1)])
    eager = EagerTrainer("cifar_cnn", B, data, labels, device="cuda", dtype="fp32", **kw)
    le = []
    for _ in range(steps):
        eager.step()
        le.append(float(eager.last_loss))
    le = torch.tensor(le)
    wf, we = lf.view(-1, win).mean(1), le.view(-1, win).mean(1)
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/curve_parity_relu{int(relu_logits)}_lr{lr:g}.json", "w") as f:
        json.dump({"fused": wf.tolist(), "eager": we.tolist()}, f)
    assert torch.isfinite(lf).all() and torch.isfinite(le).all()
    assert wf[-1] < 0.5 * wf[0] and we[-1] < 0.5 * we[0], (wf.tolist(), we.tolist())
    if not relu_logits:
        assert wf[-1] < 2.2 and we[-1] < 2.2, (wf.tolist(), we.tolist())
    # 8 %: the eager fp32 side (PyTorch / MIOpen convolutions) is not run-to-run reproducible -- its
    # second window read 3.79 and 4.09 in two runs of the same tree while the fused curve was
    # bit-identical (30.974, 3.844, ...); the steep early descent amplifies that to 6 %
    dev = ((wf - we).abs() / we).max()
    assert dev < 0.08, (float(dev), wf.tolist(), we.tolist())
