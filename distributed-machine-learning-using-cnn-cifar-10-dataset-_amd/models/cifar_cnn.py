"""The reference CIFAR-10 CNN (``create_cnn``, /root/reference/cifar10cnn.py:94-147).

conv5x5(3→64)+bias+ReLU → maxpool 3×3/2 TF-SAME → conv5x5(64→64)+bias+ReLU → maxpool 3×3/2 TF-SAME
→ flatten (NHWC order) → fc 2304→384 ReLU → fc 384→192 ReLU → fc 192→10 ReLU (ReLU on the logits, D4).

This module holds
  * ``PARAM_SPECS`` — the checkpoint contract: TF variable names, TF layouts (HWIO / [in,out]) and
    the offsets of each tensor inside the framework's flat fp32 parameter buffer;
  * :class:`CifarCNN` — a plain-PyTorch implementation with TF semantics.  It is the numerics oracle
    for the HIP kernels, the CPU "plumbing" path (BASELINE config 1) and the framework-default eager
    comparison line of the benchmark.

Layout decisions:
  * parameters keep the TF layout, so the checkpoint is a slice of the flat buffer (no permutation);
  * the flat buffer orders the conv tensors first and the fc tensors last, so that the fc gradients —
    90 % of the bytes, ready first in backward — form one contiguous all-reduce bucket;
  * every tensor starts on a 64-element (256 B) boundary so kernels can use 16-byte vector access.
"""
from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import config as C

SCOPE = "model_definition"
ALIGN = 64


@dataclasses.dataclass(frozen=True)
class ParamSpec:
    name: str                 # TF variable name (checkpoint key)
    shape: Tuple[int, ...]    # TF layout
    init: str                 # 'trunc_normal' (σ=0.05) | 'const' (0.1)
    offset: int               # element offset in the flat fp32 buffer
    bucket: int               # all-reduce bucket (0 = fc, ready first in backward; 1 = conv)

    @property
    def numel(self) -> int:
        return int(math.prod(self.shape))


def _build_specs(crop: int = C.CROP_HEIGHT) -> Tuple[List[ParamSpec], int]:
    flat = (crop // 4) * (crop // 4) * 64  # two stride-2 pools: 24 → 12 → 6 ; 6*6*64 = 2304
    raw = [
        ("conv1/conv1_kernel", (5, 5, C.NUM_CHANNELS, 64), "trunc_normal", 1),   # :106-107
        ("conv1/conv1_bias", (64,), "const", 1),                                # :108-109
        ("conv2/conv2_kernel", (5, 5, 64, 64), "trunc_normal", 1),              # :117-118
        ("conv2/conv2_bias", (64,), "const", 1),                                # :119-120
        ("full1/full_weight_1", (flat, 384), "trunc_normal", 0),                # :130-131
        ("full1/full_bias_1", (384,), "const", 0),                              # :132
        ("full2/full_weight_2", (384, 192), "trunc_normal", 0),                 # :136-137
        ("full2/full_bias_2", (192,), "const", 0),                              # :138
        ("full3/full_weight_3", (192, C.NUM_TARGETS), "trunc_normal", 0),       # :142-143
        ("full3/full_bias_3", (C.NUM_TARGETS,), "const", 0),                    # :144
    ]
    specs, off = [], 0
    for name, shape, init, bucket in raw:
        specs.append(ParamSpec(f"{SCOPE}/{name}", shape, init, off, bucket))
        off += -(-int(math.prod(shape)) // ALIGN) * ALIGN
    return specs, off


PARAM_SPECS, FLAT_SIZE = _build_specs()
NUM_PARAMS = sum(s.numel for s in PARAM_SPECS)          # 1,068,298
FC_BUCKET_OFFSET = next(s.offset for s in PARAM_SPECS if s.bucket == 0)
SPEC_BY_NAME: Dict[str, ParamSpec] = {s.name: s for s in PARAM_SPECS}


def short(name: str) -> str:
    """'model_definition/conv1/conv1_kernel' -> 'conv1_kernel'."""
    return name.rsplit("/", 1)[-1]


def init_flat_params(generator: torch.Generator | None = None, specs=PARAM_SPECS,
                     size: int = FLAT_SIZE) -> torch.Tensor:
    """Reference initialisers (cifar10cnn.py:96-101): truncated normal σ=0.05 (re-drawn beyond 2σ,
    TF semantics), biases 0.1.  Returns the flat fp32 buffer (CPU)."""
    flat = torch.zeros(size, dtype=torch.float32)
    for s in specs:
        if s.init == "const":
            v = torch.full((s.numel,), 0.1)
        else:
            v = torch.empty(s.numel)
            _trunc_normal_(v, 0.05, generator)
        flat[s.offset:s.offset + s.numel] = v
    return flat


def _trunc_normal_(t: torch.Tensor, std: float, generator) -> torch.Tensor:
    # TF truncated_normal: samples outside ±2σ are re-drawn.
    t.normal_(0.0, std, generator=generator)
    while True:
        bad = t.abs() > 2 * std
        n = int(bad.sum())
        if n == 0:
            return t
        t[bad] = torch.empty(n).normal_(0.0, std, generator=generator)


def views(flat: torch.Tensor, specs=PARAM_SPECS) -> Dict[str, torch.Tensor]:
    """TF-layout views into a flat buffer keyed by short name ('conv1_kernel', ...)."""
    return {short(s.name): flat[s.offset:s.offset + s.numel].view(s.shape) for s in specs}


def tf_same_maxpool_3x3s2(x_nchw: torch.Tensor) -> torch.Tensor:
    """tf.nn.max_pool(ksize=3, strides=2, padding='SAME') (cifar10cnn.py:113, :123).

    For even input sizes TF-SAME pads 0 before and 1 after (D12) — *not* PyTorch's symmetric
    padding=1.  Padded cells never win the max (-inf)."""
    return F.max_pool2d(F.pad(x_nchw, (0, 1, 0, 1), value=float("-inf")), 3, 2)


def cnn_forward(images_nhwc: torch.Tensor, p: Dict[str, torch.Tensor], relu_logits: bool = True) -> torch.Tensor:
    """Pure-functional forward with TF semantics.  ``images_nhwc``: [B,H,W,3] float (raw 0..255).
    ``p``: TF-layout tensors keyed by short name.  Returns logits [B,10]."""
    x = images_nhwc.permute(0, 3, 1, 2)
    x = F.conv2d(x, p["conv1_kernel"].permute(3, 2, 0, 1), p["conv1_bias"], padding=2)   # SAME 5x5
    x = tf_same_maxpool_3x3s2(F.relu(x))
    x = F.conv2d(x, p["conv2_kernel"].permute(3, 2, 0, 1), p["conv2_bias"], padding=2)
    x = tf_same_maxpool_3x3s2(F.relu(x))
    x = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)          # NHWC flatten order (cifar10cnn.py:126)
    x = F.relu(x @ p["full_weight_1"] + p["full_bias_1"])
    x = F.relu(x @ p["full_weight_2"] + p["full_bias_2"])
    x = x @ p["full_weight_3"] + p["full_bias_3"]
    return F.relu(x) if relu_logits else x


def cifar_loss(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """sparse softmax cross-entropy, mean over the batch (cifar10cnn.py:150-157)."""
    return F.cross_entropy(logits.float(), labels.long().view(-1))


def batch_accuracy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """mean(argmax(logits) == label) (cifar10cnn.py:166-176).  Ties → first index (tf.argmax)."""
    return (logits.argmax(dim=1) == labels.long().view(-1)).float().mean()


class CifarCNN(nn.Module):
    """nn.Module wrapper around :func:`cnn_forward`.  Parameters live in ONE flat fp32 tensor
    (``self.flat``) laid out by ``PARAM_SPECS``; the per-variable tensors are views of it, so a
    gradient all-reduce or an optimizer step is a single flat operation."""

    specs = PARAM_SPECS

    def __init__(self, flat: torch.Tensor | None = None, relu_logits: bool = True, seed: int = 0,
                 backend: str = "torch"):
        super().__init__()
        if backend not in ("torch", "hip_f32"):
            raise ValueError(f"unknown CNN backend {backend!r}")
        # 'hip_f32': every matmul/conv on the fp32 HIP kernels (ops/f32.py) -- reference precision
        self.backend = backend
        if flat is None:
            g = torch.Generator().manual_seed(seed)
            flat = init_flat_params(g)
        self.flat = nn.Parameter(flat.clone().float())
        self.relu_logits = relu_logits

    def params(self) -> Dict[str, torch.Tensor]:
        return views(self.flat)

    def forward(self, images_nhwc: torch.Tensor) -> torch.Tensor:
        if self.backend == "hip_f32":
            from ..ops.f32 import cnn_forward_f32, flat_views
            return cnn_forward_f32(images_nhwc, flat_views(self.flat, self.specs), self.relu_logits)
        return cnn_forward(images_nhwc, self.params(), self.relu_logits)

    def named_tf_variables(self) -> Dict[str, torch.Tensor]:
        return {s.name: self.flat.detach()[s.offset:s.offset + s.numel].view(s.shape) for s in self.specs}

    def grad_buckets(self):
        """All-reduce buckets over the flat gradient, in backward-readiness order (fc, then conv)."""
        return [(FC_BUCKET_OFFSET, FLAT_SIZE), (0, FC_BUCKET_OFFSET)]
