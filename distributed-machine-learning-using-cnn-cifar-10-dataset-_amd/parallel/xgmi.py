"""xGMI peer-to-peer gradient all-reduce (HIP IPC + a two-shot kernel), with RCCL as the fallback.

The reference moves every gradient worker -> parameter server and every variable back over gRPC
(/root/reference/cifar10cnn.py:188-196, :222, :230).  The framework's default
collective is RCCL (``torch.distributed`` "nccl").  An MI355X node, though, is 8 GPUs fully
connected by point-to-point xGMI links, and the gradient buckets of this model are small (3.84 MB +
0.43 MB per step) -- the latency-bound regime of a ring.  :class:`XgmiAllReduce` maps every peer's
gradient buffer into this process (``hipIpcOpenMemHandle``) and all-reduces with one kernel launch
per bucket (csrc/kernels/xgmi_allreduce.hip): each rank reduces 1/W of the bucket by reading it
from all W GPUs at once and pushes the sum back to all of them (wire format fp32, or bf16 for
``--comm_dtype bf16``: half the link bytes, sums in fp32).  The launch carries its barrier
epochs in device memory, so it is captured in the step's HIP graph together with the compute.

:func:`select` decides per job, by measurement: the xGMI path is used only when every rank could
map every peer, a self-test reproduces exact sums on every rank, and (mode "auto" over RCCL) it is
measured faster than RCCL on the real bucket sizes; otherwise every rank falls back to RCCL.  The
decision goes through MIN/MAX all-reduces, so it is identical on all ranks.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops import _ext

HANDLE_BYTES = 192                      # 3 IPC handles per rank: data, signals, bf16 wire


def _ops():
    _ext.hip()
    return torch.ops.dmlc


class XgmiError(RuntimeError):
    pass


class XgmiAllReduce:
    """In-place sum all-reduce of ranges of one IPC-shared fp32 buffer (``self.buf``).  wire="bf16":
    the values cross xGMI as bf16 and every replica ends with the bf16-rounded fp32 sums."""

    def __init__(self, numel: int, rank: int, world: int, group=None, wire: str = "fp32"):
        if wire not in ("fp32", "bf16"):
            raise XgmiError(f"unknown wire format {wire!r}")
        self.bf16 = wire == "bf16"
        if world > 8:
            raise XgmiError("xGMI all-reduce supports up to 8 ranks (one node)")
        ops = _ops()
        self.ops, self.rank, self.world, self.group = ops, rank, world, group
        self.numel = -(-int(numel) // 64) * 64
        self.ctx = int(ops.xgmi_create(rank, world, self.numel))
        self.closed = False
        self.buf = ops.xgmi_buffer(self.ctx)
        mine = ops.xgmi_handles(self.ctx)
        allh: List[Optional[bytes]] = [bytes(mine.numpy().tobytes())]
        if world > 1:
            allh = [None] * world
            dist.all_gather_object(allh, bytes(mine.numpy().tobytes()), group=group)
        table = torch.frombuffer(bytearray(b"".join(allh)), dtype=torch.uint8).view(world, HANDLE_BYTES).clone()
        ops.xgmi_open(self.ctx, table)

    def all_reduce(self, offset: int, numel: int, blocks: int = 0):
        """Sum-all-reduce ``buf[offset:offset+numel]`` on the current stream (capturable)."""
        self.ops.xgmi_allreduce(self.ctx, self.buf, int(offset), int(numel), int(blocks), self.bf16)

    def all_reduce_sgd(self, sgd_args: tuple, blocks: int = 0):
        """Sum-all-reduce the whole buffer (the flat gradient) and apply the SGD step in the same
        launch (xgmi_allreduce.hip k_xgmi_allreduce_sgd; ``sgd_args`` = the engine's mode-2 SGD
        arguments, its grad being this buffer).  Capturable."""
        self.ops.xgmi_allreduce_sgd(self.ctx, int(blocks), self.bf16, *sgd_args)

    def error(self) -> int:
        return int(self.ops.xgmi_error(self.ctx))

    def check(self):
        e = self.error()
        if e:
            raise XgmiError(f"xGMI all-reduce barrier timed out on rank {self.rank} (error word {e}): a peer "
                            "stopped participating")

    def self_test(self, iters: int = 3) -> bool:
        """Exact-sum check: rank r writes (r+1)*(i%97)/2 + it; every rank must read back the exact
        sum over ranks at every element (small multiples of 1/2: fp32 sums are exact; with the bf16
        wire the pattern is (r+1)*(i%5)/2 + it, exact in bf16 up to 8 ranks)."""
        n = self.numel
        pat = torch.remainder(torch.arange(n, device=self.buf.device, dtype=torch.float32), 5.0 if self.bf16 else 97.0) * 0.5
        ok = True
        for it in range(iters):
            self.buf.copy_(pat * (self.rank + 1) + it)
            split = 64 * it                               # exercise two buckets at an offset
            if split:
                self.all_reduce(0, split)
            self.all_reduce(split, n - split)
            torch.cuda.synchronize(self.buf.device)
            want = pat * (self.world * (self.world + 1) / 2) + self.world * it
            ok = ok and bool(torch.equal(self.buf, want)) and self.error() == 0
        self.buf.zero_()
        torch.cuda.synchronize(self.buf.device)
        return ok

    def close(self):
        if not self.closed:
            self.ops.xgmi_destroy(self.ctx)
            self.closed = True


def _reduce(v: float, op, device, group=None) -> float:
    t = torch.tensor([v], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=op, group=group)
    return float(t.item())


def _capture(fn, device, group=None) -> Optional["torch.cuda.CUDAGraph"]:
    """``fn``'s launches as a HIP graph, or None if the capture fails (nothing runs while capturing).
    thread_local: the process group's watchdog thread may poll events meanwhile (engine/fused.py)."""
    try:
        from .dist import quiesce_for_capture
        quiesce_for_capture(device, group)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                fn()
        torch.cuda.current_stream(device).wait_stream(s)
        torch.cuda.synchronize(device)
        return g
    except Exception:                            # noqa: BLE001 -- eager timing instead
        torch.cuda.synchronize(device)
        return None


def _time(fn, iters: int, device) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize(device)
    return (time.perf_counter() - t0) / iters


def select(numel: int, rank: int, world: int, device: torch.device, buckets: List[Tuple[int, int]],
           mode: str = "auto", group=None, log=None, wire: str = "fp32",
           captured: bool = False) -> Tuple[Optional[XgmiAllReduce], Dict]:
    """Collective choice of the gradient all-reduce.  Returns (XgmiAllReduce | None, info).

    mode "rccl": never xGMI.  "xgmi": xGMI unless it cannot work (then RCCL).  "auto": like "xgmi",
    and over RCCL additionally only if measured faster than RCCL on ``buckets`` ((offset, numel)),
    RCCL moving the same wire dtype.  ``captured``: the step graph will hold the collective, so both
    are timed as graph replays (eagerly if either capture fails on any rank)."""
    info: Dict = {"allreduce": "rccl"}
    if mode == "rccl" or world == 1 or device.type != "cuda":
        return None, info
    nccl = dist.get_backend(group) == "nccl"
    bdev = device if nccl else torch.device("cpu")
    ar, why = None, ""
    try:
        ar = XgmiAllReduce(numel, rank, world, group, wire=wire)
        ok = 1.0
    except Exception as e:                       # noqa: BLE001 -- any failure means: use RCCL
        ok, why = 0.0, f"{type(e).__name__}: {e}"
    if _reduce(ok, dist.ReduceOp.MIN, bdev, group) < 1.0:
        if ar is not None:
            ar.close()
        info["xgmi_unavailable"] = why or "a peer could not map the buffers"
        if log:
            log(f"xgmi all-reduce unavailable ({info['xgmi_unavailable']}); using RCCL")
        return None, info
    # (a first cross-GPU run is where a mapping problem would show: a raising self-test counts as a
    # failed one, so every rank still agrees on RCCL instead of one rank leaving the collective)
    try:
        ok, why = (1.0 if ar.self_test() else 0.0), "self-test mismatch"
    except Exception as e:                       # noqa: BLE001
        ok, why = 0.0, f"self-test raised {type(e).__name__}: {e}"
    if _reduce(ok, dist.ReduceOp.MIN, bdev, group) < 1.0:
        ar.close()
        info["xgmi_unavailable"] = why
        if log:
            log("xgmi all-reduce self-test failed; using RCCL")
        return None, info
    if mode == "auto" and nccl:
        scratch = torch.zeros(ar.numel, dtype=torch.bfloat16 if wire == "bf16" else torch.float32, device=device)

        def run_x():
            for off, n in buckets:
                ar.all_reduce(off, n)

        def run_r():
            for off, n in buckets:
                dist.all_reduce(scratch[off:off + n], group=group)

        # captured (the step graph holds the collective): time both as graph replays -- a collective
        # that brings cross-queue dependencies into a graph pays them there and not eagerly (one graph
        # branch node costs ~20 us per step here, profiles/r6s3_side_copy_probe.jsonl).  Capturing runs
        # no collective, so every rank first agrees that both captures worked, else all time eagerly.
        gx = gr = None
        if captured:
            gx, gr = _capture(run_x, device, group), _capture(run_r, device, group)
        both = _reduce(1.0 if gx is not None and gr is not None else 0.0, dist.ReduceOp.MIN, bdev, group) >= 1.0
        if both:
            fx, fr = gx.replay, gr.replay
        else:
            fx, fr = run_x, run_r
        tx = _reduce(_time(fx, 20, device), dist.ReduceOp.MAX, bdev, group)
        tr = _reduce(_time(fr, 20, device), dist.ReduceOp.MAX, bdev, group)
        del gx, gr
        ar.buf.zero_()
        torch.cuda.synchronize(device)
        info.update(xgmi_us=round(tx * 1e6, 1), rccl_us=round(tr * 1e6, 1), timed="graph" if both else "eager")
        if not tx < tr:
            ar.close()
            return None, info
    info["allreduce"] = "xgmi"
    info["wire"] = wire
    return ar, info
