"""Process-group bring-up: one process per GPU, RCCL (``nccl`` backend) on MI355X, gloo on CPU.

Replaces the reference's tf.train.ClusterSpec / tf.train.Server gRPC runtime
(/root/reference/cifar10cnn.py:185-196) with a c10d TCPStore rendezvous and
synchronous collectives.  Two entry styles are supported:
  * torchrun-style env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT);
  * the reference's CLI roles (``--ps_hosts/--worker_hosts/--job_name/--task_index``), mapped by
    :mod:`dmlc.cli` onto the same fields.
"""
from __future__ import annotations

import dataclasses
import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


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

    @property
    def is_chief(self) -> bool:
        return self.rank == 0


def env_info() -> DistInfo:
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    return DistInfo(rank=int(os.environ.get("RANK", "0")), world_size=ws,
                    local_rank=int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))),
                    master_addr=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                    master_port=int(os.environ.get("MASTER_PORT", "29500")))


def pick_device(local_rank: int, want: str = "auto") -> torch.device:
    if want == "cpu" or (want == "auto" and not torch.cuda.is_available()):
        return torch.device("cpu")
    n = torch.cuda.device_count()
    if n == 0:
        raise RuntimeError("a GPU was requested but none is visible")
    d = torch.device("cuda", local_rank % n)
    torch.cuda.set_device(d)          # R3 fix: each rank owns exactly one GPU
    return d


def init(info: Optional[DistInfo] = None, device: str = "auto", timeout_s: float = 300.0,
         backend: Optional[str] = None) -> DistInfo:
    """Initialise the default process group (if world_size > 1) and bind this rank's device."""
    info = info or env_info()
    info.device = pick_device(info.local_rank, device)
    info.backend = backend or ("nccl" if info.device.type == "cuda" else "gloo")
    if info.world_size > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", info.master_addr)
        os.environ.setdefault("MASTER_PORT", str(info.master_port))
        kw = {}
        if info.backend == "nccl":
            kw["device_id"] = info.device
        dist.init_process_group(info.backend, init_method=f"tcp://{info.master_addr}:{info.master_port}",
                                rank=info.rank, world_size=info.world_size,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
        info.initialized = True
    return info


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


def shutdown(info: DistInfo):
    if info.initialized and dist.is_initialized():
        dist.destroy_process_group()
