"""Data-parallel fused engine (two graph segments around the bucketed all-reduce + apply-only SGD)
vs a single-process fused run on the union batch.  Two ranks share the one GPU of the test box and
talk over gloo (which all-reduces GPU tensors through the host); on an 8-GPU node the same code
path runs over RCCL.  allreduce="xgmi" runs the IPC peer-to-peer all-reduce kernel instead
(parallel/xgmi.py; the two ranks map each other's gradient buffer on the shared GPU).  SURVEY.md §2.D / §4 'Distributed'."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _data():
    g = torch.Generator().manual_seed(21)
    x = torch.randint(0, 256, (1024, 32, 32, 3), dtype=torch.uint8, generator=g)
    y = torch.randint(0, 10, (1024,), dtype=torch.int32, generator=g)
    return x, y


def _rank(rank, world, port, out, B, steps, graph, comm_dtype, allreduce, schedule="overlap"):
    sys.path.insert(0, REPO)
    import torch.distributed as dist
    import dmlc  # noqa: F401
    from dmlc.engine.fused import FusedCifarEngine
    import datetime
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))   # a failing peer must not hang the suite
    x, y = _data()
    eng = FusedCifarEngine(B, x, y, device="cuda:0", world_size=world, rank=rank, seed=5, lr=1e-4,
                           relu_logits=False, comm_dtype=comm_dtype, allreduce=allreduce,
                           dp_schedule=schedule)
    assert eng.comm_info["allreduce"] == ("xgmi" if allreduce == "xgmi" else "rccl"), eng.comm_info
    if allreduce == "xgmi":
        assert eng.comm_info["wire"] == comm_dtype, eng.comm_info      # bf16 no longer forces RCCL
    eng.step()
    if graph:
        eng.capture()
    for _ in range(steps - 1):
        eng.step()
    torch.cuda.synchronize()
    torch.save({"flat": eng.flat_params(), "step": eng.global_step(),
                "batches": [eng.batch_indices(s) for s in range(steps)]}, os.path.join(out, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("graph,comm_dtype,allreduce,schedule",
                         [(False, "fp32", "rccl", "overlap"), (True, "fp32", "rccl", "overlap"),
                          (True, "bf16", "rccl", "overlap"), (False, "fp32", "xgmi", "overlap"),
                          (True, "fp32", "xgmi", "overlap"), (True, "fp32", "rccl", "serial"),
                          (False, "fp32", "xgmi", "serial"), (True, "fp32", "xgmi", "serial"),
                          (True, "bf16", "xgmi", "serial")])
def test_dp2_matches_single_process_union_batch(tmp_path, graph, comm_dtype, allreduce, schedule):
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    from dmlc.engine.fused import FusedCifarEngine
    B, steps = 32, 3
    mp.spawn(_rank, args=(2, free_port(), str(tmp_path), B, steps, graph, comm_dtype, allreduce, schedule),
             nprocs=2, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    assert r0["step"] == r1["step"] == steps
    assert torch.equal(r0["flat"], r1["flat"])           # replicas identical after every step
    # single process, batch 2B: the generated order makes its batch of every step exactly the two
    # ranks' batches of that step, in rank order (data/order.py)
    x, y = _data()
    ref = FusedCifarEngine(2 * B, x, y, device="cuda:0", seed=5, lr=1e-4, relu_logits=False)
    for s in range(steps):
        assert torch.equal(ref.batch_indices(s), torch.cat([r0["batches"][s], r1["batches"][s]]))
    init = ref.flat_params().clone()
    for _ in range(steps):
        ref.step()
    torch.cuda.synchronize()
    d_dp, d_ref = r0["flat"] - init, ref.flat_params() - init
    rel = float((d_dp - d_ref).norm() / d_ref.norm())
    assert rel < (2e-2 if comm_dtype == "bf16" else 1e-2), rel


def _tune_rank(rank, world, port, out, allreduce):
    sys.path.insert(0, REPO)
    import torch.distributed as dist
    import dmlc  # noqa: F401
    from dmlc.engine.fused import FusedCifarEngine
    import datetime
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    x, y = _data()
    eng = FusedCifarEngine(32, x, y, device="cuda:0", world_size=world, rank=rank, seed=5, lr=1e-4,
                           relu_logits=False, allreduce=allreduce)
    eng.step()
    eng.capture(steps_per_graph=2)
    best = eng.tune_schedule(iters=3, steps_per_graph=2)
    captured = eng._captured_schedule
    eng.run(3)
    torch.cuda.synchronize()
    torch.save({"flat": eng.flat_params(), "step": eng.global_step(), "best": best, "captured": captured,
                "info": dict(eng.comm_info)}, os.path.join(out, f"t{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("allreduce", ["rccl", "xgmi"])
def test_dp2_tune_schedule_agrees_across_ranks(tmp_path, allreduce):
    """tune_schedule(): both schedules timed (max over ranks), one decision on every rank, the
    replicas stay identical, the graphs kept are the winner's, and every timed step counts
    (1 + 2 rounds x 2 schedules x (2 + 3) tuning + 3 = 24 steps)."""
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    mp.spawn(_tune_rank, args=(2, free_port(), str(tmp_path), allreduce), nprocs=2, join=True)
    t0 = torch.load(tmp_path / "t0.pt", weights_only=True)
    t1 = torch.load(tmp_path / "t1.pt", weights_only=True)
    assert t0["best"] == t1["best"] in ("overlap", "serial")
    assert t0["info"]["schedule"] == t0["best"] and set(t0["info"]["schedule_us"]) == {"overlap", "serial"}
    assert t0["captured"] == t0["best"] and t1["captured"] == t1["best"]
    assert t0["step"] == t1["step"] == 24
    assert torch.equal(t0["flat"], t1["flat"])
    assert torch.isfinite(t0["flat"]).all()


def _nccl1_rank(rank, world, port, out, steps):
    sys.path.insert(0, REPO)
    import datetime
    import torch.distributed as dist
    import dmlc  # noqa: F401
    from dmlc.engine.fused import FusedCifarEngine
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60), device_id=torch.device("cuda", 0))
    x, y = _data()
    res = {}
    for sched in ("serial", "overlap"):
        eng = FusedCifarEngine(32, x, y, device="cuda:0", seed=5, lr=1e-4, relu_logits=False, dp_force=True,
                               dp_schedule=sched, allreduce="rccl")
        assert eng.dp and eng.capture_comm and eng.single_graph, (eng.dp, eng.capture_comm)
        eng.step()
        eng.capture(steps_per_graph=4)
        eng.run(steps - 1)
        torch.cuda.synchronize()
        res[sched] = {"flat": eng.flat_params(), "step": eng.global_step(), "info": dict(eng.comm_info)}
    torch.save(res, os.path.join(out, "nccl1.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_captured_rccl_allreduce_world1_equals_single_gpu(tmp_path):
    """The RCCL path with the all-reduce captured inside the step graph (capture_comm) and chained
    steps, on a 1-rank nccl group (dp_force: the DP step -- reduce-only SGD, all-reduce, apply-only
    SGD -- runs at world size 1).  A 1-rank sum is the identity, so it must equal the plain
    single-GPU step bit for bit, for both step schedules."""
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    from dmlc.engine.fused import FusedCifarEngine
    steps = 11
    mp.spawn(_nccl1_rank, args=(1, free_port(), str(tmp_path), steps), nprocs=1, join=True)
    res = torch.load(tmp_path / "nccl1.pt", weights_only=True)
    x, y = _data()
    ref = FusedCifarEngine(32, x, y, device="cuda:0", seed=5, lr=1e-4, relu_logits=False)
    for _ in range(steps):
        ref.step()
    torch.cuda.synchronize()
    for sched, r in res.items():
        assert r["step"] == steps, sched
        assert r["info"]["captured_comm"] and r["info"]["backend"] == "nccl", r["info"]
        assert torch.equal(r["flat"], ref.flat_params()), sched
