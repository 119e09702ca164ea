"""Process-group bring-up: one process per GPU, RCCL (``nccl`` backend) on MI355X, gloo on CPU.

Replaces the reference's tf.train.ClusterSpec / tf.train.Server gRPC runtime
(/root/reference/cifar10cnn.py:185-196) with a c10d TCPStore rendezvous and
synchronous collectives.  Two entry styles are supported:
  * torchrun-style env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT);
  * the reference's CLI roles (``--ps_hosts/--worker_hosts/--job_name/--task_index``), mapped by
    :func:`dmlc.cli.resolve_role` onto the same fields.  With a ``ps`` task the TCPStore is served by
    the ps process (:func:`serve_ps`), which exits once every worker has reported completion.

Failure detection: every collective runs under the process-group timeout
(``pg_timeout_s``), so a dead rank makes the survivors fail fast instead of hanging; the local
launcher (:mod:`dmlc.launch`) then restarts the world from the latest checkpoint.
"""
from __future__ import annotations

import dataclasses
import datetime
import os
import time
from typing import Optional

import torch
import torch.distributed as dist

DONE_KEY = "dmlc/workers_done"


@dataclasses.dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    master_addr: str = "127.0.0.1"
    master_port: int = 29500
    backend: str = "gloo"
    device: torch.device = torch.device("cpu")
    initialized: bool = False
    store: Optional[object] = None
    store_is_ps: bool = False
    from_env: bool = False        # torchrun-style env: rendezvous via env:// (the agent's store)

    @property
    def is_chief(self) -> bool:
        return self.rank == 0


def env_info() -> DistInfo:
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    return DistInfo(rank=int(os.environ.get("RANK", "0")), world_size=ws,
                    local_rank=int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))),
                    master_addr=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                    master_port=int(os.environ.get("MASTER_PORT", "29500")), from_env="RANK" in os.environ)


def role_info(role) -> DistInfo:
    return DistInfo(rank=role.rank, world_size=role.world_size, local_rank=role.local_rank,
                    master_addr=role.master_addr, master_port=role.master_port, store_is_ps=role.store_is_ps,
                    from_env=role.from_env)


def pick_device(local_rank: int, want: str = "auto") -> torch.device:
    if want == "cpu" or (want == "auto" and not torch.cuda.is_available()):
        return torch.device("cpu")
    n = torch.cuda.device_count()
    if n == 0:
        raise RuntimeError("a GPU was requested but none is visible")
    d = torch.device("cuda", local_rank % n)
    torch.cuda.set_device(d)          # R3 fix: each rank owns exactly one GPU
    return d


RCCL_ENV_KEYS = ("NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_ALGO", "NCCL_PROTO", "RCCL_MSCCL_ENABLE",
                 "NCCL_P2P_LEVEL")


def rccl_env(channels: int = 0) -> dict:
    """RCCL channel layout for the 7 point-to-point xGMI links of an MI355X node.

    One ring drives one egress link per GPU, so an all-reduce over a single ring is bound by ONE of
    the seven ~153 GB/s links.  ``channels`` > 0 asks RCCL for at least that many channels (rings laid
    over different link permutations; 7 or a multiple of it covers every link) via NCCL_MIN_NCHANNELS,
    raising NCCL_MAX_NCHANNELS to match.  The variables are read when the communicator is created, so
    this runs before ``init_process_group``.  Values already in the environment win (per-job tuning
    from the shell); 0 leaves RCCL's own topology-based choice.  Returns the RCCL/NCCL variables in
    effect, which bench.py reports next to the measured all-reduce choice."""
    if channels > 0:
        os.environ.setdefault("NCCL_MIN_NCHANNELS", str(channels))
        mx = os.environ.get("NCCL_MAX_NCHANNELS")
        if mx is None or int(mx) < int(os.environ["NCCL_MIN_NCHANNELS"]):
            os.environ["NCCL_MAX_NCHANNELS"] = os.environ["NCCL_MIN_NCHANNELS"]
    return {k: os.environ[k] for k in RCCL_ENV_KEYS if k in os.environ}


def init(info: Optional[DistInfo] = None, device: str = "auto", timeout_s: float = 300.0,
         backend: Optional[str] = None, rccl_channels: int = 0) -> DistInfo:
    """Initialise the default process group (if world_size > 1) and bind this rank's device."""
    info = info or env_info()
    info.device = pick_device(info.local_rank, device)
    # DMLC_DIST_BACKEND=gloo: rehearse a multi-rank GPU job on one GPU (RCCL refuses two ranks per GPU)
    info.backend = backend or os.environ.get("DMLC_DIST_BACKEND") or ("nccl" if info.device.type == "cuda" else "gloo")
    if info.backend == "nccl":
        rccl_env(rccl_channels)
    if info.world_size > 1 and not dist.is_initialized():
        timeout = datetime.timedelta(seconds=timeout_s)
        kw = {}
        if info.backend == "nccl":
            kw["device_id"] = info.device
        if info.from_env:
            os.environ.setdefault("MASTER_ADDR", info.master_addr)
            os.environ.setdefault("MASTER_PORT", str(info.master_port))
            dist.init_process_group(info.backend, init_method="env://", rank=info.rank,
                                    world_size=info.world_size, timeout=timeout, **kw)
        else:
            # rank 0 hosts the store unless a ps task serves it (reference CLI with --ps_hosts)
            info.store = dist.TCPStore(info.master_addr, info.master_port, None,
                                       is_master=(info.rank == 0 and not info.store_is_ps), timeout=timeout,
                                       wait_for_workers=False)
            dist.init_process_group(info.backend, store=info.store, rank=info.rank, world_size=info.world_size,
                                    timeout=timeout, **kw)
        info.initialized = True
    return info


def serve_ps(role, timeout_s: float = 86400.0, poll_s: float = 0.2, log=print) -> int:
    """The ``--job_name=ps`` process: host the rendezvous store, wait until all workers are done."""
    store = dist.TCPStore(role.master_addr, role.master_port, None, is_master=True,
                          timeout=datetime.timedelta(seconds=timeout_s), wait_for_workers=False)
    log(f"ps: rendezvous store serving {role.master_addr}:{role.master_port} for {role.world_size} worker(s)")
    t0 = time.time()
    while True:
        done = store.add(DONE_KEY, 0)
        if done >= role.world_size:
            log(f"ps: all {role.world_size} worker(s) finished")
            return 0
        if time.time() - t0 > timeout_s:
            log("ps: timed out waiting for workers")
            return 1
        time.sleep(poll_s)


def report_done(info: DistInfo):
    if info.store is not None and info.store_is_ps:
        info.store.add(DONE_KEY, 1)


def barrier(info: DistInfo):
    if info.world_size > 1 and dist.is_initialized():
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def all_max(value: float, info: DistInfo) -> float:
    if info.world_size == 1 or not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=info.device if info.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def broadcast_(t: torch.Tensor, info: DistInfo, src: int = 0) -> torch.Tensor:
    """In-place broadcast from ``src`` (chief restores a checkpoint, every rank starts identical)."""
    if info.world_size > 1 and dist.is_initialized():
        dist.broadcast(t, src)
    return t


def shutdown(info: DistInfo):
    if info.initialized and dist.is_initialized():
        dist.destroy_process_group()
        info.initialized = False


# ProcessGroupNCCL's watchdog thread wakes every ~100 ms and queries the end event of every eager
# collective it still tracks.  Those events live on the group's internal stream, which a captured
# collective joins into the capture; a query landing while a HIP graph capture is open fails with
# hipErrorCapturedEvent and terminates the watchdog -- and the process (seen once on a 1-rank nccl
# group: tests/test_fused_dp_gpu.py, rccl bf16-wire test).  Completed work leaves the list on the
# watchdog's next pass, so a capture that follows eager collectives first lets it drain.
WATCHDOG_DRAIN_S = 0.35


def quiesce_for_capture(device, group=None) -> None:
    """Call before a graph capture that may follow eager RCCL collectives (a no-op sleep-free
    synchronise on any other backend / without a process group)."""
    if device is not None and torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
    if dist.is_available() and dist.is_initialized() and dist.get_backend(group) == "nccl":
        time.sleep(WATCHDOG_DRAIN_S)
