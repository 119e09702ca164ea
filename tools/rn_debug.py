"""Per-kernel numerics of the fused ResNet-20 engine (see tests/test_fused_resnet_gpu.py
local_layer_errors).  Run on a GPU box: python tools/rn_debug.py [B]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dmlc  # noqa: F401,E402
import torch  # noqa: E402

from dmlc.engine.fused_resnet import FusedResNetEngine  # noqa: E402
from test_fused_resnet_gpu import local_layer_errors  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    g = torch.Generator().manual_seed(3)
    data = torch.randint(0, 256, (4 * B, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (4 * B,), dtype=torch.int32, generator=g)
    eng = FusedResNetEngine(B, data, labels, seed=2)
    idx = eng.batch_indices(eng.host_step)
    eng.compute_gradients()
    for k, v in local_layer_errors(eng, data, labels, idx).items():
        print(f"{k:10s} {v:.5f}")


if __name__ == "__main__":
    main()
