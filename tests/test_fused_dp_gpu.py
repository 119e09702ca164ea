"""Data-parallel fused engine (two graph segments around the bucketed all-reduce + apply-only SGD)
vs a single-process fused run on the union batch.  Two ranks share the one GPU of the test box and
talk over gloo (which all-reduces GPU tensors through the host); on an 8-GPU node the same code
path runs over RCCL.  allreduce="xgmi" runs the IPC peer-to-peer all-reduce kernel instead
(parallel/xgmi.py; the two ranks map each other's gradient buffer on the shared GPU).  SURVEY.md §2.D / §4 'Distributed'."""
import json
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


def _rank(rank, world, port, out, B, steps, graph, comm_dtype, allreduce, schedule="overlap", variant=None):
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
                           dp_schedule=schedule, staircase=False, variant=variant)
    assert eng.comm_info["allreduce"] == ("xgmi" if allreduce == "xgmi" else "rccl"), eng.comm_info
    if variant and variant.get("comm_sgd"):
        assert eng.comm_sgd
    if allreduce == "xgmi":
        assert eng.comm_info["wire"] == comm_dtype, eng.comm_info      # bf16 no longer forces RCCL
    eng.step()
    if graph:
        eng.capture()
    for _ in range(steps - 1):
        eng.step()
    torch.cuda.synchronize()
    torch.save({"flat": eng.flat_params(), "step": eng.global_step(), "fc_fused": eng.fc_fused,
                "batches": [eng.batch_indices(s) for s in range(steps)]}, os.path.join(out, f"r{rank}.pt"))
    dist.destroy_process_group()


def _dp_reference(world, B, steps, batches, comm_dtype, allreduce, fc_fused=False, wire_from=0):
    """Replays the data-parallel run on ONE world-1 engine: at every step each rank's gradient on its
    own batch from the shared weights (the DP kernels compute exactly it / world: the loss scale
    1/(B*world) is a power-of-two multiple of 1/B here, which commutes with every rounding), summed in
    rank order like the xGMI kernel (bf16 wire: bf16 inputs, fp32 sum, bf16 result), then the SAME
    apply-only SGD kernel.  ``wire_from``: the bf16 wire carries the flat gradient from this offset on
    (RCCL overlap schedule: the fc bucket only -- its conv bucket crosses as fp32).  Returns
    (initial, final) flat parameters."""
    from dmlc.engine.fused import FusedCifarEngine
    x, y = _data()
    # the fc kernels the ranks ran (ranks sharing one GPU run the three-launch fc path, not the
    # persistent fc chain, whose 256 workgroups must own the chip)
    ref = FusedCifarEngine(B, x, y, device="cuda:0", seed=5, lr=1e-4, relu_logits=False, staircase=False,
                           variant={"fc_fused": bool(fc_fused)})
    assert ref.fc_fused == fc_fused
    init = ref.flat_params().clone()
    def bf(t):
        if comm_dtype != "bf16":
            return t
        t = t.clone()
        t[wire_from:] = t[wire_from:].to(torch.bfloat16).float()
        return t
    for s in range(steps):
        tot = None
        for r in range(world):
            g = bf(ref.compute_gradients(idx=batches[r][s]).clone() / world)
            tot = g if tot is None else tot + g
        ref.grad.copy_(bf(tot))
        ref._sgd(mode=2)
    torch.cuda.synchronize()
    return init, ref.flat_params()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,graph,comm_dtype,allreduce,schedule",
                         [(2, False, "fp32", "rccl", "overlap"), (2, True, "fp32", "rccl", "overlap"),
                          (2, True, "bf16", "rccl", "overlap"), (2, False, "fp32", "xgmi", "overlap"),
                          (2, True, "fp32", "xgmi", "overlap"), (2, True, "fp32", "rccl", "serial"),
                          (2, False, "fp32", "xgmi", "serial"), (2, True, "fp32", "xgmi", "serial"),
                          (2, True, "bf16", "xgmi", "serial"), (4, True, "fp32", "rccl", "serial"),
                          (4, True, "fp32", "xgmi", "serial"), (4, True, "fp32", "xgmi", "overlap"),
                          (4, True, "bf16", "xgmi", "serial")])
def test_dp_matches_mean_of_rank_gradients(tmp_path, world, graph, comm_dtype, allreduce, schedule):
    """DP-2 / DP-4 (ranks sharing the test box's GPU; "rccl" runs over gloo here, RCCL on a node) for
    10 steps against the exact replay of the DP semantics on one engine (_dp_reference): a bucket
    offset, a missing or doubled 1/world or a stale bucket shows up as O(1e-2..1); what may remain is
    fp32 summation order inside the collective (gloo's ring) -- asserted at 1e-5.  The replicas are
    bit-identical to each other after every run."""
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    B, steps = 32, 10
    mp.spawn(_rank, args=(world, free_port(), str(tmp_path), B, steps, graph, comm_dtype, allreduce, schedule),
             nprocs=world, join=True)
    rs = [torch.load(tmp_path / f"r{k}.pt", weights_only=True) for k in range(world)]
    assert all(r["step"] == steps for r in rs)
    for r in rs[1:]:
        assert torch.equal(rs[0]["flat"], r["flat"])      # replicas identical
    # the RCCL overlap schedule sends its conv bucket as fp32 on any wire (fused.py _allreduce_bucket)
    from dmlc.models import cifar_cnn as M
    wire_from = M.FC_BUCKET_OFFSET if (allreduce == "rccl" and schedule == "overlap") else 0
    init, want = _dp_reference(world, B, steps, [r["batches"] for r in rs], comm_dtype, allreduce, rs[0]["fc_fused"],
                               wire_from=wire_from)
    d_dp, d_ref = rs[0]["flat"] - init, want - init
    rel = float((d_dp - d_ref).norm() / d_ref.norm())
    tol = 1e-2 if (comm_dtype == "bf16" and allreduce == "rccl") else 1e-5
    assert rel <= tol, rel
    if allreduce == "xgmi" and world == 2:
        assert torch.equal(rs[0]["flat"], want)           # same sums, same order, same kernels


@pytest.mark.timeout(300)
@pytest.mark.parametrize("comm_dtype", ["fp32", "bf16"])
def test_xgmi_sgd_epilogue_w2_equals_exchange_plus_sgd_launch(tmp_path, comm_dtype):
    """the exchange kernel with the SGD in its epilogue (variant comm_sgd) at W = 2 -- the
    per-peer barriers of its workgroups, the SGD reading the peer-pushed sums after the exchange --
    against the exchange + SGD launch, bit for bit (the ranks share the test box's GPU; the exchange
    kernel's workgroups are split between them)."""
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    B, steps = 32, 8
    res = {}
    for v in (True, False):
        d = tmp_path / f"v{int(v)}"
        d.mkdir()
        mp.spawn(_rank, args=(2, free_port(), str(d), B, steps, True, comm_dtype, "xgmi", "serial",
                              {"comm_sgd": v}), nprocs=2, join=True)
        res[v] = [torch.load(d / f"r{k}.pt", weights_only=True) for k in range(2)]
    for v in res:
        assert res[v][0]["step"] == res[v][1]["step"] == steps
        assert torch.equal(res[v][0]["flat"], res[v][1]["flat"])
    assert torch.isfinite(res[True][0]["flat"]).all()
    assert torch.equal(res[True][0]["flat"], res[False][0]["flat"])


def _rank_node(rank, world, port, out, B, steps, lockfile, schedule="serial", comm_dtype="fp32"):
    """One rank of a node rehearsal: the engine is told it has a GPU of its own (LOCAL_WORLD_SIZE=1),
    so it takes the paths an 8-GPU node runs -- the persistent fc chain with the conv2 dgrad, the
    wgrad launch reducing the conv slabs into the flat gradient, the split forward at B <= 128 --
    and the ranks take turns on the shared card (a file lock around each rank's GPU work) so every
    persistent launch has the chip to itself, as on its own GPU."""
    os.environ["LOCAL_WORLD_SIZE"] = "1"
    sys.path.insert(0, REPO)
    import datetime
    import fcntl
    import torch.distributed as dist
    import dmlc  # noqa: F401
    from dmlc.engine.fused import FusedCifarEngine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    x, y = _data()
    eng = FusedCifarEngine(B, x, y, device="cuda:0", world_size=world, rank=rank, seed=5, lr=1e-4,
                           relu_logits=False, comm_dtype=comm_dtype, allreduce="rccl", dp_schedule=schedule,
                           staircase=False)
    flags = {"fc_fused": eng.fc_fused, "fc_dgrad": eng.fc_dgrad, "wgrad_reduce": eng.wgrad_reduce,
             "fwd12_split": eng.fwd12_split, "grad16": eng.grad16 is not None}
    n = eng.master.numel()

    def gpu(fn):
        with open(lockfile, "a") as f:
            fcntl.flock(f, fcntl.LOCK_EX)
            try:
                fn()
                torch.cuda.synchronize()
            finally:
                fcntl.flock(f, fcntl.LOCK_UN)

    for _ in range(steps):
        if schedule == "serial":               # _serial_dp_step, with the GPU turns made explicit
            gpu(eng._seg_compute_ab)
            eng.check_barriers()
            eng._allreduce(eng._wire_grad()[:n])
            gpu(eng._seg_apply)
        else:                                  # _dp_step: fc bucket after the chain, conv bucket after wgrad
            gpu(lambda: (eng._seg_forward(), eng._seg_fc()))
            eng._allreduce_bucket(fc=True)
            gpu(eng._seg_compute_b_launch)
            eng._allreduce_bucket(fc=False)
            gpu(lambda: (eng._seg_apply_fc(), eng._seg_apply_conv()))
        eng.host_step += 1
    torch.save({"flat": eng.flat_params(), "step": eng.global_step(), "flags": flags,
                "batches": [eng.batch_indices(s) for s in range(steps)]}, os.path.join(out, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,B,schedule,comm_dtype", [(2, 32, "serial", "fp32"), (2, 160, "serial", "fp32"),
                                                         (4, 64, "serial", "fp32"), (2, 256, "overlap", "fp32"),
                                                         (4, 64, "overlap", "fp32"), (2, 256, "serial", "bf16"),
                                                         (2, 64, "overlap", "bf16")])
def test_dp_node_kernels_match_mean_of_rank_gradients(tmp_path, world, B, schedule, comm_dtype):
    """The data-parallel step with the kernels a node with one GPU per rank runs (fc chain + dgrad,
    reduce-mode wgrad with 1/(B*W) loss scale, split forward) -- which ranks sharing one GPU cannot
    run concurrently -- rehearsed with the ranks taking turns on the card, 6 steps, against the exact
    replay of the DP semantics on one engine with the same kernels (_dp_reference, fc chain on).
    Both step schedules: serial (one all-reduce, one SGD launch) and overlap (fc bucket after the
    chain, conv bucket after the wgrad launch, fc / conv SGD launches)."""
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    steps = 6
    mp.spawn(_rank_node, args=(world, free_port(), str(tmp_path), B, steps, str(tmp_path / "gpu.lock"), schedule,
                               comm_dtype), nprocs=world, join=True)
    rs = [torch.load(tmp_path / f"r{k}.pt", weights_only=True) for k in range(world)]
    f = rs[0]["flags"]
    assert f["fc_fused"] and f["fc_dgrad"] and f["wgrad_reduce"], f
    assert f["fwd12_split"] == (B <= 128), f
    assert f["grad16"] == (comm_dtype == "bf16"), f      # the bf16 wire: producers write bf16 (grad16)
    assert all(r["step"] == steps for r in rs)
    for r in rs[1:]:
        assert torch.equal(rs[0]["flat"], r["flat"])      # replicas identical
    init, want = _dp_reference(world, B, steps, [r["batches"] for r in rs], comm_dtype, "rccl", fc_fused=True)
    d_dp, d_ref = rs[0]["flat"] - init, want - init
    rel = float((d_dp - d_ref).norm() / d_ref.norm())
    # bf16: gloo sums the two bf16 gradients in its own order / precision (the reference: fp32 sum of
    # the bf16 inputs, rounded once) -- the tolerance of the other gloo bf16 cases
    assert rel <= (1e-5 if comm_dtype == "fp32" else 1e-2), rel


def test_dp_reference_union_batch_consistency():
    """The generated order makes the W ranks' batches of a step exactly the union batch a single
    process with batch W*B trains on (data/order.py), in rank order."""
    from dmlc.engine.fused import FusedCifarEngine
    x, y = _data()
    single = FusedCifarEngine(64, x, y, device="cuda:0", seed=5)
    from dmlc.data.order import OrderSpec
    specs = [OrderSpec(x.shape[0], 32, 2, r, 5) for r in (0, 1)]
    for s in (0, 1, 7, 15, 16, 40):
        assert torch.equal(single.batch_indices(s).long(), torch.cat([sp.batch(s).long() for sp in specs]))


def _curve_rank(rank, world, port, out, comm_dtype, steps, B):
    sys.path.insert(0, REPO)
    import datetime
    import torch.distributed as dist
    import dmlc  # noqa: F401
    from dmlc.data import synthetic
    from dmlc.engine.fused import FusedCifarEngine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=120))
    x, y = synthetic(4096, seed=5, learnable=True)
    eng = FusedCifarEngine(B, x, y, device="cuda:0", world_size=world, rank=rank, seed=6, lr=1e-4,
                           relu_logits=False, comm_dtype=comm_dtype, allreduce="xgmi", dp_schedule="serial",
                           staircase=False)
    assert eng.comm_info.get("wire") == comm_dtype, eng.comm_info
    eng.step()
    eng.capture(steps_per_graph=8)
    eng.run(steps - 1)
    torch.cuda.synchronize()
    eng.check_comm()
    torch.save({"loss": [eng.read_stats(k)["loss"] for k in range(1, steps + 1)], "flat": eng.flat_params()},
               os.path.join(out, f"c{comm_dtype}{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp2_bf16_wire_loss_curve_tracks_fp32_wire(tmp_path):
    """Round-6 check behind bench.py's default gradient wire: DP-2 over the xGMI exchange kernel (the
    ranks share the test box's GPU) trains 300 steps on learnable synthetic data with the bf16 wire
    (every summed gradient rounded to bf16, half the link bytes) and with the fp32 wire, from the same
    weights on the same batches.  Both learn, the bf16 replicas stay bit-identical, and the loss curves
    (25-step windows) agree like the fused-vs-eager parity test's (tests/test_cnn_kernels_gpu.py):
    within 8 % through the steep first 50 steps (the first run measured 5.0 % in window 2, 3.54 vs
    3.37), within 3 % from window 3 on (2.4 % max) and within 2 % in the last window (0.5 %)."""
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    steps, B, win = 300, 64, 25
    for cd in ("fp32", "bf16"):
        mp.spawn(_curve_rank, args=(2, free_port(), str(tmp_path), cd, steps, B), nprocs=2, join=True)
    c = {cd: [torch.load(tmp_path / f"c{cd}{r}.pt", weights_only=True) for r in (0, 1)] for cd in ("fp32", "bf16")}
    for cd in c:
        assert torch.equal(c[cd][0]["flat"], c[cd][1]["flat"]), cd
    lf, lb = torch.tensor(c["fp32"][0]["loss"]), torch.tensor(c["bf16"][0]["loss"])
    wf, wb = lf.view(-1, win).mean(1), lb.view(-1, win).mean(1)
    os.makedirs("gpurun_out", exist_ok=True)
    import json
    with open("gpurun_out/dp2_wire_curve.json", "w") as f:
        json.dump({"fp32": wf.tolist(), "bf16": wb.tolist()}, f)
    assert torch.isfinite(lf).all() and torch.isfinite(lb).all()
    assert wf[-1] < 0.9 * wf[0] and wb[-1] < 0.9 * wb[0], (wf.tolist(), wb.tolist())
    dev = (wb - wf).abs() / wf
    assert float(dev.max()) < 0.08, (dev.tolist(), wf.tolist(), wb.tolist())
    assert float(dev[2:].max()) < 0.03 and float(dev[-1]) < 0.02, (dev.tolist(), wf.tolist(), wb.tolist())


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


def _nccl1_rank(rank, world, port, out, steps, dtype="bf16", B=32):
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
        eng = FusedCifarEngine(B, x, y, device="cuda:0", seed=5, lr=1e-4, relu_logits=False, dp_force=True,
                               dp_schedule=sched, allreduce="rccl", dtype=dtype)
        assert eng.dp and eng.capture_comm and eng.single_graph, (eng.dp, eng.capture_comm)
        # the DP step reduces the conv slabs inside the wgrad launch (fp8 too: round 3 asserted here)
        assert eng.wgrad_reduce == eng._grad_in_launch
        assert eng.wgrad_reduce or sched == "overlap", sched
        eng.step()
        eng.capture(steps_per_graph=4)
        eng.run(steps - 1)
        torch.cuda.synchronize()
        res[sched] = {"flat": eng.flat_params(), "step": eng.global_step(), "info": dict(eng.comm_info)}
    if dtype == "fp8":
        res["fp8_state"] = {"w2f8": eng.w2f8.cpu(), "scale_w": eng.scale_w.cpu()}
    torch.save(res, os.path.join(out, "nccl1.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("dtype,B", [("bf16", 32), ("fp8", 32), ("bf16", 256)])
def test_captured_rccl_allreduce_world1_equals_single_gpu(tmp_path, dtype, B):
    """The RCCL path with the all-reduce captured inside the step graph (capture_comm) and chained
    steps, on a 1-rank nccl group (dp_force: the DP step -- conv slabs reduced in the wgrad launch,
    all-reduce, apply-only SGD -- runs at world size 1).  A 1-rank sum is the identity, so it must
    equal the plain single-GPU step bit for bit, for both step schedules; fp8 (BASELINE config 5)
    also compares the e4m3 weight shadows and the delayed scales.  B=256: the fc chain with the conv2
    dgrad inside it and its dW tiles writing gradients (the DP form) against the single-GPU step's
    fused-SGD epilogues."""
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    from dmlc.engine.fused import FusedCifarEngine
    steps = 11
    mp.spawn(_nccl1_rank, args=(1, free_port(), str(tmp_path), steps, dtype, B), nprocs=1, join=True)
    res = torch.load(tmp_path / "nccl1.pt", weights_only=True)
    x, y = _data()
    ref = FusedCifarEngine(B, x, y, device="cuda:0", seed=5, lr=1e-4, relu_logits=False, dtype=dtype)
    for _ in range(steps):
        ref.step()
    torch.cuda.synchronize()
    f8 = res.pop("fp8_state", None)
    if dtype == "fp8":
        assert torch.equal(f8["w2f8"], ref.w2f8.cpu()) and torch.equal(f8["scale_w"], ref.scale_w.cpu())
    for sched, r in res.items():
        assert r["step"] == steps, sched
        assert r["info"]["captured_comm"] and r["info"]["backend"] == "nccl", r["info"]
        assert torch.equal(r["flat"], ref.flat_params()), sched


@pytest.mark.parametrize("B,comm_dtype", [(32, "fp32"), (256, "fp32"), (64, "bf16")])
def test_xgmi_sgd_epilogue_is_bit_identical(B, comm_dtype):
    """r5 DP step without an SGD launch: the xGMI exchange kernel applies the SGD in its epilogue
    (k_xgmi_allreduce_sgd) to the float4s each thread owns in the exchange.  On a one-rank xGMI
    context (dp_force) the weights, every bf16 shadow, the next batch rows, the stats and the step
    counter after eager + chained graph replays equal the exchange + SGD-launch step bit for bit --
    and, for the fp32 wire (a one-rank sum is the identity), the single-GPU step."""
    from dmlc.engine.fused import FusedCifarEngine
    x, y = _data()
    kw = dict(device="cuda:0", seed=5, lr=1e-4, relu_logits=False, dp_force=True, allreduce="xgmi",
              dp_schedule="serial", comm_dtype=comm_dtype)
    fused = FusedCifarEngine(B, x, y, **kw, variant={"comm_sgd": True})
    ref = FusedCifarEngine(B, x, y, **kw)
    single = FusedCifarEngine(B, x, y, device="cuda:0", seed=5, lr=1e-4, relu_logits=False)
    assert fused.comm_sgd and not ref.comm_sgd and fused.comm_info["allreduce"] == "xgmi"
    for eng in (fused, ref, single):
        eng.step()
        eng.capture(steps_per_graph=4)
        eng.run(8)
        eng.set_step(eng.global_step() + 2)
        eng.run(3)
    torch.cuda.synchronize()
    assert fused.global_step() == ref.global_step() == 14
    assert torch.isfinite(ref.master).all()
    assert torch.equal(fused.master, ref.master)
    for name in ("w1f", "w2f", "w2d", "fc2t", "fc2n", "fc3t", "fc3d", "bidx"):
        assert torch.equal(getattr(fused, name), getattr(ref, name)), name
    assert torch.equal(fused.fc1n_current(), ref.fc1n_current())
    for s in (10, 11, 14):
        assert fused.read_stats(s) == ref.read_stats(s), s
    fused.check_comm()
    if comm_dtype == "fp32":
        assert torch.equal(fused.master, single.master)
        assert torch.equal(fused.fc1n_current(), single.fc1n_current())


def _grad16_rank(rank, world, port, out, steps, B):
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
        for g16 in (True, False):
            eng = FusedCifarEngine(B, x, y, device="cuda:0", seed=5, lr=1e-4, relu_logits=False, dp_force=True,
                                   dp_schedule=sched, allreduce="rccl", comm_dtype="bf16", variant={"grad16": g16})
            assert (eng.grad16 is not None) == g16, (sched, g16)
            eng.step()
            eng.capture(steps_per_graph=4)
            eng.run(steps - 1)
            torch.cuda.synchronize()
            res[(sched, g16)] = {"flat": eng.flat_params(), "step": eng.global_step(),
                                 "fc1n": eng.fc1n_current().cpu(), "w2f": eng.w2f.cpu()}
    torch.save({f"{k[0]}-{int(k[1])}": v for k, v in res.items()}, os.path.join(out, "g16.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("B", [256, 64])
def test_rccl_bf16_wire_grad16_equals_cast_path(tmp_path, B):
    """Round 6: on the RCCL bf16 wire the fc chain, the wgrad launch's slab reduction and the
    reduce-only SGD write the flat gradient as bf16 (grad16) and the apply-only SGD reads it -- no
    cast launches around the all-reduce.  On a 1-rank nccl group (captured RCCL, chained graphs) it
    must equal the fp32 gradient + t.to(bf16) + all-reduce + copy-back path bit for bit (the same
    single rounding of every gradient element), and the overlap schedule the serial one."""
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    steps = 9
    mp.spawn(_grad16_rank, args=(1, free_port(), str(tmp_path), steps, B), nprocs=1, join=True)
    r = torch.load(tmp_path / "g16.pt", weights_only=True)
    a, b = r["serial-1"], r["serial-0"]
    assert a["step"] == b["step"] == r["overlap-1"]["step"] == steps
    assert torch.isfinite(a["flat"]).all()
    for k in ("flat", "fc1n", "w2f"):
        assert torch.equal(a[k], b[k]), k
        # the overlap schedule's conv bucket crosses as bf16 too when grad16 holds it (without grad16
        # it goes fp32, fused.py _allreduce_bucket): the same weights as the serial step
        assert torch.equal(r["overlap-1"][k], a[k]), k


def _select_rank(rank, world, port, out):
    sys.path.insert(0, REPO)
    import datetime
    import torch.distributed as dist
    import dmlc  # noqa: F401
    from dmlc.parallel import xgmi as X
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60), device_id=torch.device("cuda", 0))
    real = X.XgmiAllReduce
    # select() at world 2 over a 1-rank nccl group, the IPC context built at world 1 (one GPU): the
    # captured-timing path (both collectives captured, agreed, replayed) runs for real
    X.XgmiAllReduce = lambda numel, r, w, group=None, wire="fp32": real(numel, 0, 1, None, wire=wire)
    res = {}
    for captured in (True, False):
        ar, info = X.select(1 << 20, 0, 2, torch.device("cuda", 0), [(0, 1 << 20)], mode="auto",
                            wire="bf16", captured=captured)
        res[str(captured)] = dict(info)
        if ar is not None:
            ar.close()
    torch.save(res, os.path.join(out, "select.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_select_times_captured_collectives_as_graph_replays(tmp_path):
    """The xGMI-vs-RCCL choice of a job whose step graph holds the collective times both as graph
    replays (a collective that adds cross-queue dependencies pays them only when captured), and
    falls back to eager timing otherwise; both choices report their timings."""
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    mp.spawn(_select_rank, args=(1, free_port(), str(tmp_path)), nprocs=1, join=True)
    res = torch.load(tmp_path / "select.pt", weights_only=True)
    print(json.dumps(res))
    assert res["True"]["timed"] == "graph", res
    assert res["False"]["timed"] == "eager", res
    for info in res.values():
        assert info["xgmi_us"] > 0 and info["rccl_us"] > 0, info
        assert info["allreduce"] in ("xgmi", "rccl") and "xgmi_unavailable" not in info, info
