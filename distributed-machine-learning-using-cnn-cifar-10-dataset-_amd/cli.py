"""Command line of the framework — flag-compatible with the reference script.

The six reference flags (/root/reference/cifar10cnn.py:249-272) keep their names, types and
defaults; unknown arguments are tolerated like ``parse_known_args`` + ``tf.app.run`` (:273-274).
The reference's hard-coded constants (:9-27) become extension flags with the same defaults
(SURVEY.md §5.6).

Roles:
  --job_name=worker --task_index=k   -> DP rank k of W = len(--worker_hosts) ranks, one GPU each;
                                        rendezvous (c10d TCPStore) at ps_hosts[0] if given, else
                                        at worker_hosts[0]
  --job_name=ps                      -> the rendezvous host: serves the TCPStore, waits until every
                                        worker has finished, then exits (the reference PS blocked
                                        forever in server.join(), :191-192)
  no --job_name and torchrun env     -> RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT
  neither                            -> single process (world_size 1)
Any other --job_name does nothing, like the reference (:191-196).
"""
from __future__ import annotations

import argparse
import dataclasses
import os
import socket
from typing import List, Optional, Tuple

from . import config as C


def _bool(v: str) -> bool:
    # the reference registered a "bool" type (:247); here it is actually usable
    if isinstance(v, bool):
        return v
    s = v.strip().lower()
    if s in ("1", "true", "t", "yes", "y"):
        return True
    if s in ("0", "false", "f", "no", "n"):
        return False
    raise argparse.ArgumentTypeError(f"not a boolean: {v!r}")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X-native distributed CIFAR-10 CNN training "
                                            "(flag-compatible with cifar10cnn.py)")
    p.register("type", "bool", _bool)
    d = C.TrainConfig()
    # --- reference flags (cifar10cnn.py:249-272) ---
    p.add_argument("--ps_hosts", type=str, default=d.ps_hosts, help="Comma-separated list of hostname:port pairs")
    p.add_argument("--worker_hosts", type=str, default=d.worker_hosts,
                   help="Comma-separated list of hostname:port pairs")
    p.add_argument("--job_name", type=str, default=d.job_name, help="One of 'ps', 'worker'")
    p.add_argument("--task_index", type=int, default=d.task_index, help="Index of task within the job")
    p.add_argument("--data_dir", type=str, default=d.data_dir, help="Directory for storing input data")
    p.add_argument("--log_dir", type=str, default=d.log_dir, help="Directory for train logs / checkpoints")
    # --- extension flags (reference constants made overridable; defaults == reference) ---
    p.add_argument("--batch_size", type=int, default=d.batch_size)
    p.add_argument("--generations", type=int, default=d.generations)
    p.add_argument("--learning_rate", type=float, default=d.learning_rate)
    p.add_argument("--lr_decay", type=float, default=d.lr_decay)
    p.add_argument("--num_gens_to_wait", type=float, default=d.num_gens_to_wait)
    p.add_argument("--lr_schedule", choices=["staircase", "constant"], default=d.lr_schedule)
    p.add_argument("--lr_scaling", choices=["none", "linear"], default=d.lr_scaling,
                   help="linear: learning_rate * global_batch / lr_base_batch (large-batch recipe)")
    p.add_argument("--lr_base_batch", type=int, default=d.lr_base_batch)
    p.add_argument("--warmup_steps", type=int, default=d.warmup_steps, help="linear LR warm-up steps")
    p.add_argument("--output_every", type=int, default=d.output_every)
    p.add_argument("--eval_every", type=int, default=d.eval_every)
    p.add_argument("--eval_batches", type=int, default=d.eval_batches)
    p.add_argument("--crop", type=int, default=None,
                   help="center crop (default 24 = the reference for cifar_cnn, 32 = full images for resnet20)")
    p.add_argument("--relu_logits", type="bool", default=d.relu_logits)
    p.add_argument("--augment", type="bool", default=d.augment)
    p.add_argument("--synthetic", type="bool", nargs="?", const=True, default=d.synthetic)
    p.add_argument("--synthetic_size", type=int, default=d.synthetic_size)
    p.add_argument("--download", type="bool", nargs="?", const=True, default=False)
    p.add_argument("--model", choices=["cifar_cnn", "resnet20"], default=d.model)
    p.add_argument("--dtype", choices=["fp32", "bf16", "fp8"], default=d.dtype)
    p.add_argument("--impl", choices=["auto", "fused", "eager", "hipf32"], default=d.impl)
    p.add_argument("--device", choices=["auto", "cpu", "cuda"], default=d.device)
    p.add_argument("--seed", type=int, default=d.seed)
    p.add_argument("--checkpoint_secs", type=float, default=d.checkpoint_secs)
    p.add_argument("--max_to_keep", type=int, default=d.max_to_keep)
    p.add_argument("--save_checkpoints", type="bool", default=d.save_checkpoints)
    p.add_argument("--metrics_file", type=str, default=d.metrics_file)
    p.add_argument("--comm_dtype", choices=["fp32", "bf16"], default=d.comm_dtype)
    p.add_argument("--allreduce", choices=["auto", "rccl", "xgmi"], default=d.allreduce,
                   help="gradient all-reduce: xGMI peer-to-peer kernel (auto: when it self-tests and "
                        "measures faster than RCCL) or RCCL")
    p.add_argument("--dp_schedule", choices=["auto", "serial", "overlap"], default=d.dp_schedule,
                   help="N>1 fused CNN step: one stream + one all-reduce (serial), or the fc bucket's "
                        "all-reduce + SGD on a comm stream under the conv backward (overlap); auto times "
                        "both at start-up (max over ranks) and keeps the faster")
    p.add_argument("--steps_per_graph", type=int, default=d.steps_per_graph,
                   help="longest chain of training steps captured into one HIP graph")
    p.add_argument("--pg_timeout_s", type=float, default=d.pg_timeout_s)
    p.add_argument("--heartbeat_s", type=float, default=d.heartbeat_s)
    p.add_argument("--heartbeat_timeout_s", type=float, default=d.heartbeat_timeout_s,
                   help="a peer silent this long makes the survivors exit 75 (0: off)")
    p.add_argument("--check_replicas", type="bool", default=d.check_replicas,
                   help="compare a parameter checksum across ranks at every output point")
    p.add_argument("--rccl_channels", type=int, default=d.rccl_channels,
                   help="RCCL channels (rings over different xGMI link permutations); 0 = RCCL's choice")
    p.add_argument("--graph", type="bool", default=d.graph)
    p.add_argument("--trace", choices=["", "roctx", "torch"], default=d.trace)
    p.add_argument("--trace_steps", type=int, default=d.trace_steps)
    return p


def parse(argv: Optional[List[str]] = None) -> Tuple[C.TrainConfig, List[str]]:
    """Parse flags -> (TrainConfig, unparsed args).  Unknown flags are returned, not rejected."""
    ns, unparsed = build_parser().parse_known_args(argv)
    fields = {f.name for f in dataclasses.fields(C.TrainConfig)}
    if ns.crop is None:
        ns.crop = 32 if ns.model == "resnet20" else C.CROP_HEIGHT
    cfg = C.TrainConfig(**{k: v for k, v in vars(ns).items() if k in fields})
    return cfg, unparsed


# --- role -> (rank, world, local rank, rendezvous) ---------------------------------------------------
@dataclasses.dataclass
class Role:
    kind: str                 # 'worker' | 'ps' | 'none'
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    master_addr: str = "127.0.0.1"
    master_port: int = 29500
    store_is_ps: bool = False  # the TCPStore is served by the ps process
    from_env: bool = False     # torchrun env rendezvous


def split_hosts(s: str) -> List[str]:
    return [h.strip() for h in s.split(",") if h.strip()] if s else []


def parse_hostport(hp: str) -> Tuple[str, int]:
    host, _, port = hp.rpartition(":")
    if not host or not port.isdigit():
        raise ValueError(f"expected host:port, got {hp!r}")
    return host, int(port)


def _norm_host(h: str) -> str:
    return "127.0.0.1" if h in ("localhost", "") else h


def resolve_role(cfg: C.TrainConfig, env=None) -> Role:
    env = os.environ if env is None else env
    ps, workers = split_hosts(cfg.ps_hosts), split_hosts(cfg.worker_hosts)
    if cfg.job_name in ("ps", "worker"):
        if not workers:
            raise ValueError("--worker_hosts is required for --job_name=ps/worker")
        anchor = ps[0] if ps else workers[0]
        host, port = parse_hostport(anchor)
        if cfg.job_name == "ps":
            if cfg.task_index != 0:
                return Role("none")   # extra PS tasks have nothing to do (no sharded variables)
            return Role("ps", rank=-1, world_size=len(workers), master_addr=_norm_host(host), master_port=port,
                        store_is_ps=True)
        k = cfg.task_index
        if not 0 <= k < len(workers):
            raise ValueError(f"--task_index={k} out of range for {len(workers)} workers")
        my_host = _norm_host(parse_hostport(workers[k])[0])
        local = sum(1 for w in workers[:k] if _norm_host(parse_hostport(w)[0]) == my_host)
        return Role("worker", rank=k, world_size=len(workers), local_rank=local, master_addr=_norm_host(host),
                    master_port=port, store_is_ps=bool(ps))
    if cfg.job_name:
        return Role("none")
    if "RANK" in env and "WORLD_SIZE" in env:
        return Role("worker", rank=int(env["RANK"]), world_size=int(env["WORLD_SIZE"]),
                    local_rank=int(env.get("LOCAL_RANK", env["RANK"])),
                    master_addr=env.get("MASTER_ADDR", "127.0.0.1"), master_port=int(env.get("MASTER_PORT", 29500)),
                    from_env=True)
    return Role("worker")


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
