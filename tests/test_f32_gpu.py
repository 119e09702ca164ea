"""fp32-accurate HIP mode (``--dtype fp32`` / ``--impl hipf32``, ops/f32.py): the fp32 MFMA GEMM,
im2col / col2im and column sums against float64 references, the whole CNN's logits and gradients
against the fp32/fp64 PyTorch model at <= 1e-4 relative error, several batch sizes, determinism, and
training steps of the eager engine on the HIP backend (graph-captured) against the PyTorch fp32
engine."""
import pytest
import torch
import torch.nn.functional as F

from dmlc.models import cifar_cnn as M

pytestmark = pytest.mark.gpu


def _ops():
    import dmlc.ops._ext as E
    E.hip()
    return torch.ops.dmlc


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("M_,N_,K_", [(77, 50, 33), (256, 384, 2304), (75, 64, 20000), (1, 10, 192), (300, 130, 64)])
def test_gemm_f32_matches_fp64(ta, tb, M_, N_, K_):
    ops = _ops()
    g = torch.Generator(device="cuda").manual_seed(M_ * 7 + N_)
    a = torch.randn((K_, M_) if ta else (M_, K_), device="cuda", generator=g)
    b = torch.randn((N_, K_) if tb else (K_, N_), device="cuda", generator=g)
    bias = torch.randn(N_, device="cuda", generator=g)
    for relu in (False, True):
        got = ops.f32_gemm(a, b, bias, ta, tb, relu)
        ref = (a.double().t() if ta else a.double()) @ (b.double().t() if tb else b.double()) + bias.double()
        if relu:
            ref = ref.clamp_min(0)
        assert got.shape == (M_, N_)
        # fp32 products and fp32 accumulation: error ~ sqrt(K) * 2^-24 relative
        assert _rel(got, ref) < 2e-6, (ta, tb, relu, _rel(got, ref))
    # no bias, and bitwise reproducible (split-K slices summed in a fixed order)
    x1 = ops.f32_gemm(a, b, None, ta, tb, False)
    x2 = ops.f32_gemm(a, b, None, ta, tb, False)
    assert torch.equal(x1, x2)


def test_im2col_col2im_are_adjoint_and_match_conv():
    ops = _ops()
    B, H, W, C, CO, k = 3, 12, 12, 64, 64, 5
    x = torch.randn(B, H, W, C, device="cuda", dtype=torch.float64).float()
    w = torch.randn(k, k, C, CO, device="cuda").float() * 0.05
    cols = ops.f32_im2col(x, k, k, 2)
    assert cols.shape == (B * H * W, k * k * C)
    y = (cols.double() @ w.double().view(-1, CO)).view(B, H, W, CO)
    ref = F.conv2d(x.double().cpu().permute(0, 3, 1, 2), w.double().cpu().permute(3, 2, 0, 1), padding=2)
    assert _rel(y.cpu(), ref.permute(0, 2, 3, 1)) < 1e-12
    g = torch.randn_like(cols)
    dx = ops.f32_col2im(g, B, H, W, C, k, k, 2)
    lhs = float((dx.double() * x.double()).sum())
    rhs = float((g.double() * cols.double()).sum())
    assert abs(lhs - rhs) / abs(rhs) < 1e-5


@pytest.mark.parametrize("H,C,CO", [(24, 3, 64), (12, 64, 64)])
def test_implicit_conv_gemm_matches_explicit_im2col(H, C, CO):
    ops = _ops()
    B = 5
    g = torch.Generator(device="cuda").manual_seed(H)
    x = torch.randn(B, H, H, C, device="cuda", generator=g)
    w = torch.randn(25 * C, CO, device="cuda", generator=g) * 0.05
    dy = torch.randn(B * H * H, CO, device="cuda", generator=g)
    cols = ops.f32_im2col(x, 5, 5, 2).double()
    y = ops.f32_conv_gemm(x, w, None, False, False)
    assert _rel(y, cols @ w.double()) < 2e-6
    gwb = ops.f32_conv_gemm(x, dy, None, True, True)          # [25C + 1, CO]: weights + bias row
    assert gwb.shape == (25 * C + 1, CO)
    assert _rel(gwb[:25 * C], cols.t() @ dy.double()) < 2e-6
    assert _rel(gwb[25 * C], dy.double().sum(0)) < 2e-6
    assert torch.equal(gwb, ops.f32_conv_gemm(x, dy, None, True, True))


def test_implicit_conv_autograd_matches_explicit_path():
    from dmlc.ops import f32 as F32
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(4, 12, 12, 64, device="cuda", generator=g, requires_grad=True)
    w = (torch.randn(5, 5, 64, 64, device="cuda", generator=g) * 0.05).requires_grad_()
    b = torch.randn(64, device="cuda", generator=g, requires_grad=True)
    outs = []
    for implicit in (True, False):
        y = F32.conv_same(x, w, b, implicit=implicit)
        gx, gw, gb = torch.autograd.grad((y * y).sum(), (x, w, b))
        outs.append((y.detach(), gx, gw, gb))
    for a, e in zip(outs[0], outs[1]):
        assert _rel(a, e) < 1e-5


def test_colsum_is_fixed_order_and_exact_enough():
    ops = _ops()
    for M_, N_ in [(147456, 64), (256, 384), (5, 10), (1000, 1)]:
        x = torch.randn(M_, N_, device="cuda")
        s = ops.f32_colsum(x)
        assert _rel(s, x.double().sum(0)) < 1e-5
        assert torch.equal(s, ops.f32_colsum(x))


def _model_pair(relu_logits=True, seed=0):
    flat = M.init_flat_params(torch.Generator().manual_seed(seed))
    ref = M.CifarCNN(flat, relu_logits=relu_logits).cuda()
    hip = M.CifarCNN(flat, relu_logits=relu_logits, backend="hip_f32").cuda()
    return ref, hip


@pytest.mark.parametrize("B", [1, 2, 8, 100])
def test_cnn_logits_and_grads_match_fp64(B):
    ref, hip = _model_pair(relu_logits=False, seed=B)
    g = torch.Generator().manual_seed(B)
    x = torch.randint(0, 256, (B, 24, 24, 3), generator=g).float().cuda()
    y = torch.randint(0, 10, (B,), generator=g).cuda()
    logits = hip(x)
    loss = F.cross_entropy(logits, y)
    loss.backward()
    # float64 oracle on the CPU (same parameters, same TF semantics)
    ref64 = M.CifarCNN(ref.flat.detach().cpu().double(), relu_logits=False)
    ref64.flat.data = ref64.flat.data.double()
    l64 = ref64(x.cpu().double())
    F.cross_entropy(l64, y.cpu()).backward()
    assert _rel(logits.detach().cpu(), l64.detach()) < 1e-4, _rel(logits.detach().cpu(), l64.detach())
    g_hip = M.views(hip.flat.grad.detach().cpu())
    g_64 = M.views(ref64.flat.grad.detach())
    for name in g_hip:
        assert _rel(g_hip[name], g_64[name]) < 1e-4, (name, _rel(g_hip[name], g_64[name]))


def test_cnn_f32_is_deterministic():
    _, hip = _model_pair()
    x = torch.randint(0, 256, (64, 24, 24, 3)).float().cuda()
    y = torch.randint(0, 10, (64,)).cuda()
    out = []
    for _ in range(2):
        hip.flat.grad = None
        F.cross_entropy(hip(x), y).backward()
        out.append(hip.flat.grad.clone())
    assert torch.equal(out[0], out[1])


def test_eager_engine_hip_f32_graph_trains_like_torch_fp32():
    """Graph replay of the fp32 HIP step tracks the same step run eagerly (the captured SGD reads a
    device LR tensor -- addcmul instead of add(alpha) -- so the update rounds differently; the
    forward/backward themselves are bitwise reproducible, test above), and both track the PyTorch
    fp32 engine."""
    from dmlc.engine.eager import EagerTrainer
    g = torch.Generator().manual_seed(5)
    data = torch.randint(0, 256, (1024, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (1024,), dtype=torch.int32, generator=g)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    kw = dict(device="cuda", dtype="fp32", seed=2, lr=1e-5)     # reference ReLU logits, raw pixels
    a = EagerTrainer("cifar_cnn", 64, data, labels, graph=True, backend="hip_f32", **kw)
    c = EagerTrainer("cifar_cnn", 64, data, labels, backend="hip_f32", **kw)
    b = EagerTrainer("cifar_cnn", 64, data, labels, **kw)
    for i in range(8):                       # 3 eager warm-up steps, capture, 5 graph replays
        for t in (a, b, c):
            t.step()
        if i == 0:                           # one step: the fp32 paths agree to fp32 rounding
            assert _rel(c.model.flat.detach(), b.model.flat.detach()) < 1e-6
    torch.cuda.synchronize()
    assert a.graph is not None and a.global_step == b.global_step == c.global_step == 8
    assert _rel(a.model.flat.detach(), c.model.flat.detach()) < 1e-6
    lb = float(b.last_loss)
    assert abs(float(a.last_loss) - lb) < 1e-3 * max(1.0, abs(lb)), (float(a.last_loss), lb)
    assert _rel(a.model.flat.detach(), b.model.flat.detach()) < 1e-4
