"""CPU-side contract of the fp32-accurate HIP mode (ops/f32.py): routing and argument validation.
The kernels themselves are covered by tests/test_f32_gpu.py."""
import pytest
import torch

from dmlc import config as C
from dmlc.engine.trainer import pick_impl
from dmlc.models import build_model


def test_pick_impl_routes_fp32_cnn_to_hip_kernels():
    assert pick_impl(C.TrainConfig(dtype="fp32"), torch.device("cuda")) == "hipf32"
    assert pick_impl(C.TrainConfig(dtype="fp32"), torch.device("cpu")) == "eager"
    assert pick_impl(C.TrainConfig(dtype="bf16"), torch.device("cuda")) == "fused"
    assert pick_impl(C.TrainConfig(dtype="fp32", model="resnet20"), torch.device("cuda")) == "eager"


def test_backend_validation():
    m = build_model("cifar_cnn", backend="hip_f32")
    assert m.backend == "hip_f32"
    with pytest.raises(ValueError):
        build_model("cifar_cnn", backend="tf32")
    with pytest.raises(ValueError):
        build_model("resnet20", backend="hip_f32")
    from dmlc.engine.eager import EagerTrainer
    data = torch.zeros(64, 32, 32, 3, dtype=torch.uint8)
    labels = torch.zeros(64, dtype=torch.int32)
    with pytest.raises(ValueError):       # the fp32 HIP path is a GPU path
        EagerTrainer("cifar_cnn", 16, data, labels, device="cpu", dtype="fp32", backend="hip_f32")
