"""HIP-graph capture of the eager (PyTorch-op) step equals the uncaptured step (ResNet-20 path)."""
import pytest
import torch

from dmlc.data import synthetic
from dmlc.engine.eager import EagerTrainer

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model,crop,lr", [("resnet20", 32, 0.01), ("cifar_cnn", 24, 1e-4)])
def test_graph_step_matches_eager(model, crop, lr):
    x, y = synthetic(512, seed=4, learnable=True)
    kw = dict(device="cuda", dtype="fp32", crop=crop, seed=2, lr=lr, relu_logits=False)
    a = EagerTrainer(model, 64, x, y, graph=False, **kw)
    b = EagerTrainer(model, 64, x, y, graph=True, **kw)
    for _ in range(8):
        a.step()
        b.step()
    torch.cuda.synchronize()
    assert b.graph is not None and a.global_step == b.global_step == 8
    fa, fb = a.flat_params(), b.flat_params()
    assert float((fa - fb).norm() / fa.norm()) < 1e-4
    assert abs(float(a.last_loss) - float(b.last_loss)) < 1e-3 * max(1.0, abs(float(a.last_loss)))
