"""xGMI peer-to-peer all-reduce (csrc/kernels/xgmi_allreduce.hip, parallel/xgmi.py).

Two ranks share the one GPU of the test box: each maps the other's buffer through HIP IPC exactly
as on an 8-GPU node (where the mapping crosses xGMI).  Checked: bit-exact sums against a PyTorch
fp32 reference (same summation order), offset buckets, HIP-graph replay of the captured launch,
and the sticky timeout error word when a peer never arrives.  SURVEY.md §5.8 (iii)."""
import datetime
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _init(rank, world, port):
    sys.path.insert(0, REPO)
    import torch.distributed as dist
    import dmlc  # noqa: F401
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    torch.cuda.set_device(0)
    return dist


def _data(rank, n, it):
    g = torch.Generator().manual_seed(1000 * it + rank)
    return torch.randn(n, generator=g)


def _rank_exact(rank, world, port, out):
    dist = _init(rank, world, port)
    from dmlc.parallel.xgmi import XgmiAllReduce
    n = 4096 * 37 + 64
    ar = XgmiAllReduce(n, rank, world)
    res = {"self_test": ar.self_test()}
    # eager: two buckets, random data
    ar.buf.copy_(_data(rank, ar.numel, 0).cuda())
    ar.all_reduce(0, 1024)
    ar.all_reduce(1024, ar.numel - 1024)
    torch.cuda.synchronize()
    res["eager"] = ar.buf.cpu().clone()
    # graph: capture once, replay with fresh data
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        ar.all_reduce(0, ar.numel, 8)
    torch.cuda.current_stream().wait_stream(s)
    reps = []
    for it in (1, 2, 3):
        ar.buf.copy_(_data(rank, ar.numel, it).cuda())
        torch.cuda.synchronize()
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        reps.append(ar.buf.cpu().clone())
    res["graph"] = reps
    res["err"] = ar.error()
    dist.barrier()
    ar.close()
    torch.save(res, os.path.join(out, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_xgmi_allreduce_two_ranks_exact(tmp_path):
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    world = 2
    mp.spawn(_rank_exact, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    rs = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    n = rs[0]["eager"].numel()
    for r in rs:
        assert r["self_test"] and r["err"] == 0
    want = _data(0, n, 0) + _data(1, n, 0)                 # kernel order: rank 0 + rank 1
    for r in rs:
        assert torch.equal(r["eager"], want)
    for k, it in enumerate((1, 2, 3)):
        want = _data(0, n, it) + _data(1, n, it)
        for r in rs:
            assert torch.equal(r["graph"][k], want), (k, float((r["graph"][k] - want).abs().max()))


def test_xgmi_single_rank_identity():
    """world = 1 (no peers): the launch is a barrier with itself and leaves the data unchanged."""
    import dmlc  # noqa: F401
    from dmlc.parallel.xgmi import XgmiAllReduce
    ar = XgmiAllReduce(1000, 0, 1)
    x = torch.randn(ar.numel, device="cuda")
    ar.buf.copy_(x)
    ar.all_reduce(0, ar.numel)
    ar.all_reduce(64, 128)
    torch.cuda.synchronize()
    assert torch.equal(ar.buf, x) and ar.error() == 0
    ar.close()


def _rank_timeout(rank, world, port, out):
    dist = _init(rank, world, port)
    from dmlc.parallel.xgmi import XgmiAllReduce
    ar = XgmiAllReduce(4096, rank, world)
    dist.barrier()
    err = 0
    if rank == 0:                      # rank 1 never launches: rank 0's barrier must time out, not hang
        ar.all_reduce(0, ar.numel, 4)
        torch.cuda.synchronize()
        err = ar.error()
    dist.barrier()
    ar.close()
    torch.save({"err": err}, os.path.join(out, f"t{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_xgmi_missing_peer_times_out(tmp_path):
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    mp.spawn(_rank_timeout, args=(2, free_port(), str(tmp_path)), nprocs=2, join=True)
    assert torch.load(tmp_path / "t0.pt", weights_only=True)["err"] & 1


def _rank_bf16(rank, world, port, out):
    dist = _init(rank, world, port)
    from dmlc.parallel.xgmi import XgmiAllReduce
    ar = XgmiAllReduce(4096 * 9 + 64, rank, world, wire="bf16")
    res = {"self_test": ar.self_test()}
    ar.buf.copy_(_data(rank, ar.numel, 5).cuda())
    dist.barrier()
    ar.all_reduce(0, 256)
    ar.all_reduce(256, ar.numel - 256)
    torch.cuda.synchronize()
    res["eager"] = ar.buf.cpu().clone()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        ar.all_reduce(0, ar.numel, 4)
    torch.cuda.current_stream().wait_stream(s)
    ar.buf.copy_(_data(rank, ar.numel, 6).cuda())
    torch.cuda.synchronize()
    dist.barrier()
    g.replay()
    torch.cuda.synchronize()
    res["graph"] = ar.buf.cpu().clone()
    res["err"] = ar.error()
    dist.barrier()
    ar.close()
    torch.save(res, os.path.join(out, f"b{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_xgmi_allreduce_bf16_wire(tmp_path):
    """--comm_dtype bf16 over the xGMI kernel: each rank's values cross as bf16, the owner sums in
    fp32 in rank order, and every replica receives the same bf16-rounded sums -- equal, bit for bit,
    to bf16(bf16(x0) + bf16(x1)) computed on the host, on both ranks, eager and graph-replayed."""
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    world = 2
    mp.spawn(_rank_bf16, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    rs = [torch.load(tmp_path / f"b{r}.pt", weights_only=True) for r in range(world)]
    n = rs[0]["eager"].numel()
    bf = lambda t: t.to(torch.bfloat16).float()
    for key, it in (("eager", 5), ("graph", 6)):
        want = bf(bf(_data(0, n, it)) + bf(_data(1, n, it)))
        for r in rs:
            assert r["self_test"] and r["err"] == 0
            assert torch.equal(r[key], want), (key, float((r[key] - want).abs().max()))


def _rank_exact_w(rank, world, port, out, wire):
    """One rank of the W-rank exact-sum check: two odd-sized buckets eager, then the whole buffer
    captured into a HIP graph and replayed on fresh data."""
    dist = _init(rank, world, port)
    from dmlc.parallel.xgmi import XgmiAllReduce
    ar = XgmiAllReduce(4 * 9973 + 4 * 3 * world, rank, world, wire=wire)
    res = {"self_test": ar.self_test(), "n": ar.numel}
    ar.buf.copy_(_data(rank, ar.numel, 10).cuda())
    dist.barrier()
    cut = 4 * 1237                     # neither bucket a multiple of W, of the block size or of 64
    ar.all_reduce(0, cut)
    ar.all_reduce(cut, ar.numel - cut)
    torch.cuda.synchronize()
    res["eager"] = ar.buf.cpu().clone()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        ar.all_reduce(0, ar.numel, 3)
    torch.cuda.current_stream().wait_stream(s)
    reps = []
    for it in (11, 12):
        ar.buf.copy_(_data(rank, ar.numel, it).cuda())
        torch.cuda.synchronize()
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        reps.append(ar.buf.cpu().clone())
    res["graph"] = reps
    res["err"] = ar.error()
    dist.barrier()
    ar.close()
    torch.save(res, os.path.join(out, f"w{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world,wire", [(3, "fp32"), (3, "bf16"), (4, "fp32"), (5, "bf16"), (6, "fp32"),
                                        (7, "bf16"), (8, "fp32"), (8, "bf16")])
def test_xgmi_allreduce_w_ranks_exact(tmp_path, world, wire):
    """W = 3..8 ranks (all on the test box's one GPU, each mapping every peer through HIP IPC as
    on an 8-GPU node): every replica holds, bit for bit, the rank-ordered fp32 sum (bf16 wire: of the
    bf16-rounded inputs, rounded to bf16) for two buckets whose sizes divide by nothing convenient,
    eager and graph-replayed; no timeout.  Every world size an 8-GPU node can run executes its kernel
    instance (W = 2 has its own test)."""
    import torch.multiprocessing as mp
    from dmlc.cli import free_port
    mp.spawn(_rank_exact_w, args=(world, free_port(), str(tmp_path), wire), nprocs=world, join=True)
    rs = [torch.load(tmp_path / f"w{r}.pt", weights_only=True) for r in range(world)]
    n = rs[0]["n"]
    bf = (lambda t: t.to(torch.bfloat16).float()) if wire == "bf16" else (lambda t: t)

    def want(it):
        s = bf(_data(0, n, it))
        for r in range(1, world):
            s = s + bf(_data(r, n, it))
        return bf(s)

    for r in rs:
        assert r["self_test"] and r["err"] == 0
    w10 = want(10)
    for r in rs:
        assert torch.equal(r["eager"], w10), float((r["eager"] - w10).abs().max())
    for k, it in enumerate((11, 12)):
        w = want(it)
        for r in rs:
            assert torch.equal(r["graph"][k], w), (k, float((r["graph"][k] - w).abs().max()))
