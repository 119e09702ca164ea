"""TF1-compatible checkpoints in ``--log_dir`` (TensorBundle V2 + the ``checkpoint`` state file).

The reference never saves explicitly: ``tf.train.MonitoredTrainingSession(checkpoint_dir=log_dir,
is_chief=task_index == 0)`` (/root/reference/cifar10cnn.py:222) adds a chief-only
CheckpointSaverHook (every 600 s + at the end, ``Saver(sharded=True, max_to_keep=5)``) and restores
the latest checkpoint on start-up.  This module reproduces that on-disk contract:

  <log_dir>/checkpoint                       text proto: model_checkpoint_path / all_model_checkpoint_paths
  <log_dir>/model.ckpt-N.index               SSTable of BundleEntryProto      (native: csrc/runtime)
  <log_dir>/model.ckpt-N.data-00000-of-00001 raw tensor bytes

Keys: the 10 ``model_definition/...`` variables in TF layouts (HWIO conv kernels, [in,out] fc
weights, ``full_weight_1`` rows in NHWC flatten order), ``global_step`` (int64 scalar) and
``Variable`` (int32 scalar = the reference's ``generation_num``, :216).

With ``graph_info`` the manager also writes what the TF1 hooks write beside the checkpoints:
``<log_dir>/graph.pbtxt`` (once) and ``model.ckpt-N.meta`` (a MetaGraphDef per checkpoint, removed
with it): the reference model as a TF1 graph with a V2 saver (utils/metagraph.py).
"""
from __future__ import annotations

import os
import re
import time
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .ops import _ext

# TF DataType enum <-> torch dtype
_TF2TORCH = {1: torch.float32, 2: torch.float64, 3: torch.int32, 4: torch.uint8, 5: torch.int16, 6: torch.int8,
             9: torch.int64, 10: torch.bool, 14: torch.bfloat16, 19: torch.float16}
_TORCH2TF = {v: k for k, v in _TF2TORCH.items()}

STATE_FILE = "checkpoint"
PREFIX = "model.ckpt"


def _tensor_bytes(t: torch.Tensor) -> bytes:
    t = t.detach().to("cpu").contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().tobytes()
    return t.numpy().tobytes()


def write_bundle(prefix: str, tensors: Dict[str, torch.Tensor]) -> None:
    """Write ``<prefix>.index`` + ``<prefix>.data-00000-of-00001`` (native writer)."""
    names = list(tensors)
    dtypes, shapes, blobs = [], [], []
    for n in names:
        t = torch.as_tensor(tensors[n])
        if t.dtype not in _TORCH2TF:
            raise TypeError(f"{n}: dtype {t.dtype} has no TF DataType")
        dtypes.append(_TORCH2TF[t.dtype])
        shapes.append(list(t.shape))
        blobs.append(_tensor_bytes(t))
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    _ext.rt().write_bundle(prefix, names, dtypes, shapes, blobs)


def read_bundle(prefix: str) -> Dict[str, torch.Tensor]:
    """Read every tensor of a TensorBundle (crc32c-verified) as CPU torch tensors."""
    out = {}
    for name, dtype, shape, data in _ext.rt().read_bundle(prefix):
        if dtype not in _TF2TORCH:
            raise TypeError(f"{name}: unsupported TF dtype {dtype}")
        td = _TF2TORCH[dtype]
        if td == torch.bfloat16:
            arr = torch.from_numpy(np.frombuffer(data, dtype=np.int16).copy()).view(torch.bfloat16)
        else:
            np_dt = torch.empty(0, dtype=td).numpy().dtype
            arr = torch.from_numpy(np.frombuffer(data, dtype=np_dt).copy())
        out[name] = arr.reshape(shape)
    return out


# --- the `checkpoint` state file (CheckpointState text proto) ------------------------------------
def _quote(s: str) -> str:
    return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'


def write_state(log_dir: str, latest: str, all_paths: List[str]) -> None:
    lines = [f"model_checkpoint_path: {_quote(latest)}"]
    lines += [f"all_model_checkpoint_paths: {_quote(p)}" for p in all_paths]
    tmp = os.path.join(log_dir, STATE_FILE + ".tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(log_dir, STATE_FILE))


def read_state(log_dir: str) -> Tuple[Optional[str], List[str]]:
    path = os.path.join(log_dir, STATE_FILE)
    if not os.path.exists(path):
        return None, []
    latest, all_paths = None, []
    pat = re.compile(r'^\s*(model_checkpoint_path|all_model_checkpoint_paths)\s*:\s*"((?:[^"\\]|\\.)*)"\s*$')
    with open(path) as f:
        for line in f:
            m = pat.match(line)
            if not m:
                continue
            val = m.group(2).replace('\\"', '"').replace("\\\\", "\\")
            if m.group(1) == "model_checkpoint_path":
                latest = val
            else:
                all_paths.append(val)
    return latest, all_paths


def _abs(log_dir: str, p: str) -> str:
    return p if os.path.isabs(p) else os.path.join(log_dir, p)


def latest_checkpoint(log_dir: str) -> Optional[str]:
    """tf.train.latest_checkpoint: the prefix named by the state file, if its index exists."""
    latest, _ = read_state(log_dir)
    if latest is None:
        return None
    p = _abs(log_dir, latest)
    return p if os.path.exists(p + ".index") else None


class CheckpointManager:
    """Chief-side saver: TF1 CheckpointSaverHook semantics (save at start, every ``secs`` seconds and
    at the end; keep the newest ``max_to_keep``)."""

    def __init__(self, log_dir: str, max_to_keep: int = 5, secs: float = 600.0, graph_info: Optional[dict] = None):
        self.log_dir = os.path.abspath(log_dir)
        self.graph_info = graph_info       # model / batch / crop / relu_logits for graph.pbtxt + .meta
        self._meta = None
        self.max_to_keep = max_to_keep
        self.secs = secs
        self.last_save = None
        os.makedirs(self.log_dir, exist_ok=True)
        latest, kept = read_state(self.log_dir)
        if not kept and latest:
            kept = [latest]
        self.kept = [_abs(self.log_dir, p) for p in kept]

    def save(self, step: int, tensors: Dict[str, torch.Tensor]) -> str:
        prefix = os.path.join(self.log_dir, f"{PREFIX}-{int(step)}")
        write_bundle(prefix, tensors)
        if self.graph_info is not None:
            # metagraph imports google.protobuf lazily (inside its builders), so a missing protobuf
            # runtime surfaces from build/write, not from the module import: all of it is guarded,
            # and the bundle + state file written around it keep the checkpoint usable
            try:
                from .utils import metagraph as MG
                if self._meta is None:        # the variables never change: build once
                    self._meta = MG.build_meta_graph(tensors, max_to_keep=self.max_to_keep, **self.graph_info)
                    MG.write_graph_pbtxt(self.log_dir, self._meta)
                MG.write_meta(prefix, self._meta)
            except ImportError as e:          # protobuf runtime missing
                print(f"[dmlc] graph.pbtxt / .meta not written ({e})", flush=True)
                self.graph_info, self._meta = None, None
        self.kept = [p for p in self.kept if p != prefix] + [prefix]
        while self.max_to_keep and len(self.kept) > self.max_to_keep:
            old = self.kept.pop(0)
            for suffix in (".index", ".data-00000-of-00001", ".meta"):
                try:
                    os.remove(old + suffix)
                except FileNotFoundError:
                    pass
        write_state(self.log_dir, prefix, self.kept)
        self.last_save = time.time()
        return prefix

    def due(self, now: Optional[float] = None) -> bool:
        if self.last_save is None:
            return True
        return (now or time.time()) - self.last_save >= self.secs


def model_tensors(flat: torch.Tensor, global_step: int, generation_num: int = 0, specs=None) -> Dict[str, torch.Tensor]:
    """Checkpoint dict of the reference CNN from the flat fp32 parameter buffer (TF layouts)."""
    from .models import cifar_cnn as M
    specs = specs or M.PARAM_SPECS
    flat = flat.detach().float().cpu()
    d = {s.name: flat[s.offset:s.offset + s.numel].view(s.shape).clone() for s in specs}
    d["global_step"] = torch.tensor(int(global_step), dtype=torch.int64)
    d["Variable"] = torch.tensor(int(generation_num), dtype=torch.int32)
    return d


def load_model_tensors(tensors: Dict[str, torch.Tensor], flat_size: Optional[int] = None, specs=None):
    """Inverse of :func:`model_tensors`: (flat fp32 buffer, global_step, generation_num)."""
    from .models import cifar_cnn as M
    specs = specs or M.PARAM_SPECS
    flat = torch.zeros(flat_size or M.FLAT_SIZE, dtype=torch.float32)
    for s in specs:
        if s.name not in tensors:
            raise KeyError(f"checkpoint is missing {s.name}")
        t = tensors[s.name]
        if tuple(t.shape) != tuple(s.shape):
            raise ValueError(f"{s.name}: checkpoint shape {tuple(t.shape)} != model shape {s.shape}")
        flat[s.offset:s.offset + s.numel] = t.float().reshape(-1)
    step = int(tensors["global_step"]) if "global_step" in tensors else 0
    gen = int(tensors["Variable"]) if "Variable" in tensors else 0
    return flat, step, gen


def module_tensors(model, global_step: int, generation_num: int = 0) -> Dict[str, torch.Tensor]:
    """Checkpoint dict of an eager model with flat buffers (``flat`` + optional ``state``)."""
    d = {s.name: model.flat.detach().cpu()[s.offset:s.offset + s.numel].view(s.shape).clone() for s in model.specs}
    for s in getattr(model, "state_specs", []):
        d[s.name] = model.state.detach().cpu()[s.offset:s.offset + s.numel].view(s.shape).clone()
    d["global_step"] = torch.tensor(int(global_step), dtype=torch.int64)
    d["Variable"] = torch.tensor(int(generation_num), dtype=torch.int32)
    return d


@torch.no_grad()
def load_module_tensors(model, tensors: Dict[str, torch.Tensor]) -> int:
    """Inverse of :func:`module_tensors`; returns global_step."""
    for specs, buf in ((model.specs, model.flat), (getattr(model, "state_specs", []), getattr(model, "state", None))):
        for s in specs:
            if s.name not in tensors:
                raise KeyError(f"checkpoint is missing {s.name}")
            t = tensors[s.name]
            if tuple(t.shape) != tuple(s.shape):
                raise ValueError(f"{s.name}: checkpoint shape {tuple(t.shape)} != model shape {s.shape}")
            buf[s.offset:s.offset + s.numel] = t.reshape(-1).to(buf.device, buf.dtype)
    return int(tensors["global_step"]) if "global_step" in tensors else 0
