"""Data-parallel fused ResNet-20 (SGD mode 1 -> all-reduce of the flat gradient -> SGD mode 2) vs the
average of two single-process gradients.  BatchNorm uses per-rank batch statistics (as the eager
model under DP), so the reference is the mean of the per-shard gradients, not the union batch.
Two ranks share the test box's GPU over gloo; on an 8-GPU node the same path runs over RCCL (or
the xGMI peer-to-peer all-reduce kernel, allreduce="xgmi")."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B, LR = 32, 0.02


def _data():
    g = torch.Generator().manual_seed(23)
    return (torch.randint(0, 256, (512, 32, 32, 3), dtype=torch.uint8, generator=g),
            torch.randint(0, 10, (512,), dtype=torch.int32, generator=g))


def _rank(rank, world, port, out, graph, allreduce):
    sys.path.insert(0, REPO)
    import datetime
    import torch.distributed as dist
    import dmlc  # noqa: F401
    from dmlc.engine.fused_resnet import FusedResNetEngine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    x, y = _data()
    eng = FusedResNetEngine(B, x, y, device="cuda:0", world_size=world, rank=rank, seed=5, lr=LR,
                            allreduce=allreduce)
    assert eng.comm_info["allreduce"] == ("xgmi" if allreduce == "xgmi" else "rccl"), eng.comm_info
    if graph:
        eng.capture()
    eng.step()
    torch.cuda.synchronize()
    torch.save({"flat": eng.flat_params(), "state": eng.state.cpu(), "step": eng.global_step(),
                "batch": eng.batch_indices(0)}, os.path.join(out, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("graph,allreduce", [(False, "rccl"), (True, "rccl"), (True, "xgmi")])
def test_resnet_dp2_matches_mean_of_rank_gradients(tmp_path, graph, allreduce):
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    from dmlc.engine.fused_resnet import FusedResNetEngine
    mp.spawn(_rank, args=(2, free_port(), str(tmp_path), graph, allreduce), nprocs=2, join=True)
    r = [torch.load(tmp_path / f"r{k}.pt", weights_only=True) for k in (0, 1)]
    assert r[0]["step"] == r[1]["step"] == 1
    assert torch.equal(r[0]["flat"], r[1]["flat"])
    x, y = _data()
    grads = []
    for k in (0, 1):
        ref = FusedResNetEngine(B, x, y, device="cuda:0", seed=5, lr=LR)
        init = ref.flat_params().clone()
        grads.append(ref.compute_gradients(idx=r[k]["batch"]).cpu().clone())   # rank k's batch of step 0
    expect = -LR * (grads[0] + grads[1]) / 2
    got = r[0]["flat"] - init
    rel = float((got - expect).norm() / expect.norm())
    assert rel < 1e-2, rel
