"""Hyper-parameters and run configuration.

The module constants mirror the reference's hard-coded block (``/root/reference/cifar10cnn.py:9-27``)
with the same names and values.  Unlike the reference, every one of them is overridable through
:class:`TrainConfig` (and the CLI extension flags in :mod:`dmlc.cli`); the defaults reproduce the
reference exactly.
"""
from __future__ import annotations

import dataclasses
from typing import Optional

# --- reference constants (cifar10cnn.py:9-27) -------------------------------------------------
OUTPUT_EVERY = 200
EVAL_EVERY = 500
BATCH_SIZE = 128
GENERATIONS = 20000
IMAGE_HEIGHT = 32
IMAGE_WIDTH = 32
CROP_HEIGHT = 24
CROP_WIDTH = 24
NUM_CHANNELS = 3
NUM_TARGETS = 10
LEARNING_RATE = 0.1
LR_DECAY = 0.9
NUM_GENS_TO_WAIT = 250.0
IMAGE_VECTOR_LENGTH = IMAGE_HEIGHT * IMAGE_WIDTH * NUM_CHANNELS
RECORD_LENGTH = IMAGE_VECTOR_LENGTH + 1
DATA_DIR = "cifar10data"
EXTRACT_FOLDER = "cifar-10-batches-bin"
CIFAR10_URL = "http://www.cs.toronto.edu/~kriz/cifar-10-binary.tar.gz"  # cifar10cnn.py:39

# Checkpoint cadence of TF1's default CheckpointSaverHook (MonitoredTrainingSession, cifar10cnn.py:222)
CHECKPOINT_SECS = 600
MAX_TO_KEEP = 5
STEP_COUNTER_EVERY = 100


@dataclasses.dataclass
class TrainConfig:
    """Everything a training run needs.  Defaults == reference behaviour."""

    # reference flags (cifar10cnn.py:249-272)
    ps_hosts: str = ""
    worker_hosts: str = ""
    job_name: str = ""
    task_index: int = 0
    data_dir: str = "/tmp/mnist_data"   # reference default (a copy-paste leftover); see data.resolve_data_dir
    log_dir: str = "/tmp/train_logs"

    # extension flags (reference constants made overridable)
    batch_size: int = BATCH_SIZE          # per worker
    generations: int = GENERATIONS        # StopAtStepHook(last_step)
    learning_rate: float = LEARNING_RATE
    lr_decay: float = LR_DECAY
    num_gens_to_wait: float = NUM_GENS_TO_WAIT
    lr_schedule: str = "staircase"        # 'staircase' (D3 fixed) | 'constant' (reference as run)
    # large-batch recipe (BASELINE config 5): lr = learning_rate * global_batch / lr_base_batch with
    # 'linear' scaling, ramped linearly from lr / warmup_steps over the first warmup_steps steps
    lr_scaling: str = "none"              # 'none' (reference) | 'linear'
    lr_base_batch: int = BATCH_SIZE       # the batch learning_rate was tuned for (the reference's 128)
    warmup_steps: int = 0
    output_every: int = OUTPUT_EVERY
    eval_every: int = EVAL_EVERY
    eval_batches: int = 0                 # 0 = full test set; 1 = reference fidelity (one batch)
    crop: int = CROP_HEIGHT
    relu_logits: bool = True              # D4: the reference applies ReLU to the logits
    augment: bool = False                 # D5: reference uses a deterministic center crop
    synthetic: bool = False
    synthetic_size: int = 50000
    download: bool = False                # fetch the CIFAR-10 archive if absent (offline by default)
    model: str = "cifar_cnn"              # cifar_cnn | resnet20
    dtype: str = "bf16"                   # fp32 | bf16 | fp8
    impl: str = "auto"                    # auto | fused (HIP kernels + hipGraph) | eager (torch ops) | hipf32 (fp32 HIP)
    device: str = "auto"                  # auto | cpu | cuda
    seed: int = 0
    checkpoint_secs: float = CHECKPOINT_SECS
    max_to_keep: int = MAX_TO_KEEP
    save_checkpoints: bool = True
    metrics_file: Optional[str] = None    # JSONL metrics (default: <log_dir>/metrics.jsonl on the chief)
    comm_dtype: str = "fp32"              # gradient all-reduce dtype: fp32 | bf16
    allreduce: str = "auto"               # gradient all-reduce: auto | rccl | xgmi (parallel/xgmi.py)
    dp_schedule: str = "auto"             # N>1 fused step: auto (measured at start) | serial | overlap
    steps_per_graph: int = 32             # longest chain of training steps per HIP graph replay (= bench.py)
    rccl_channels: int = 0                # >0: NCCL_MIN_NCHANNELS for RCCL over the 7 xGMI links (§5.8)
    pg_timeout_s: float = 300.0           # process-group timeout (fail-fast on a dead rank)
    heartbeat_s: float = 1.0              # liveness beat interval (parallel/health.py); N>1 only
    heartbeat_timeout_s: float = 20.0     # a peer silent this long -> exit 75 (0 disables the heartbeat)
    check_replicas: bool = True           # compare a parameter checksum across ranks every output_every
    graph: bool = True                    # capture the fused step into a HIP graph
    trace: str = ""                       # '' | 'roctx' (phase ranges for rocprofv3 --marker-trace)
                                          #    | 'torch' (torch.profiler chrome trace in log_dir)
    trace_steps: int = 20                 # steps covered by a torch.profiler trace

    def replace(self, **kw) -> "TrainConfig":
        return dataclasses.replace(self, **kw)


def effective_lr(cfg: "TrainConfig", world_size: int) -> float:
    """The base learning rate the engines run with: the reference's, or linearly scaled with the
    global batch (cfg.lr_scaling == 'linear'; Goyal et al.'s large-minibatch rule, used together
    with cfg.warmup_steps)."""
    if cfg.lr_scaling == "linear":
        return cfg.learning_rate * cfg.batch_size * max(1, world_size) / cfg.lr_base_batch
    return cfg.learning_rate
