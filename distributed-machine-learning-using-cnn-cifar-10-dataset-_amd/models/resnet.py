"""ResNet-20 for CIFAR-10 (He et al. 2016, §4.2) — the deeper conv stack of BASELINE.json config 4.

Not part of the reference (which only has the 2-conv CNN of /root/reference/cifar10cnn.py:94-147);
it exists to stress the implicit-GEMM weight-gradient path at DP=8 ("Extra kernels
not in the reference").  Layout and conventions match the reference CNN so the same trainer,
checkpoint and DP machinery apply:
  * NHWC input (uint8 crops cast to float), the same center-crop pipeline (``--crop 32`` for full
    images);
  * trainable parameters live in ONE flat fp32 buffer (``flat``) in TF layouts (HWIO kernels,
    [in, out] dense), with TF-style variable names; BatchNorm moving statistics live in a second flat
    buffer (``state``) and are checkpointed too;
  * 3x3 convs SAME-padded, 3 stages x 3 basic blocks (16/32/64 channels), option-A shortcuts
    (identity; stride-2 subsampling + zero channel padding), global average pool, fc 64 -> 10.
  * train-mode BN uses batch statistics (per-rank in DP, like the reference's per-worker graphs),
    eval uses the moving averages (momentum 0.1, eps 1e-3).
"""
from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .cifar_cnn import ParamSpec, _trunc_normal_

SCOPE = "resnet20"
ALIGN = 64
WIDTHS = (16, 32, 64)
BLOCKS = 3
BN_EPS = 1e-3
BN_MOMENTUM = 0.1


def _specs() -> Tuple[List[ParamSpec], int, List[ParamSpec], int]:
    params, state = [], []
    poff = soff = 0

    def add_p(name, shape, init):
        nonlocal poff
        params.append(ParamSpec(f"{SCOPE}/{name}", shape, init, poff, 0))
        poff += -(-int(math.prod(shape)) // ALIGN) * ALIGN

    def add_s(name, shape, init):
        nonlocal soff
        state.append(ParamSpec(f"{SCOPE}/{name}", shape, init, soff, 0))
        soff += -(-int(math.prod(shape)) // ALIGN) * ALIGN

    def conv_bn(prefix, cin, cout):
        add_p(f"{prefix}/conv/kernel", (3, 3, cin, cout), "he")
        add_p(f"{prefix}/bn/gamma", (cout,), "one")
        add_p(f"{prefix}/bn/beta", (cout,), "zero")
        add_s(f"{prefix}/bn/moving_mean", (cout,), "zero")
        add_s(f"{prefix}/bn/moving_variance", (cout,), "one")

    conv_bn("stem", 3, WIDTHS[0])
    cin = WIDTHS[0]
    for s, wdt in enumerate(WIDTHS):
        for b in range(BLOCKS):
            conv_bn(f"stage{s}/block{b}/a", cin, wdt)
            conv_bn(f"stage{s}/block{b}/b", wdt, wdt)
            cin = wdt
    add_p("fc/weights", (WIDTHS[-1], 10), "fc")
    add_p("fc/biases", (10,), "zero")
    return params, poff, state, soff


PARAM_SPECS, FLAT_SIZE, STATE_SPECS, STATE_SIZE = _specs()
NUM_PARAMS = sum(s.numel for s in PARAM_SPECS)      # 269,722 trainable (+ 1,376 BN moving stats)


def init_flat_params(generator=None) -> Tuple[torch.Tensor, torch.Tensor]:
    flat = torch.zeros(FLAT_SIZE)
    for s in PARAM_SPECS:
        if s.init == "he":
            fan_in = s.shape[0] * s.shape[1] * s.shape[2]
            v = torch.empty(s.numel)
            _trunc_normal_(v, math.sqrt(2.0 / fan_in), generator)
        elif s.init == "fc":
            v = torch.empty(s.numel)
            _trunc_normal_(v, 1.0 / math.sqrt(s.shape[0]), generator)
        elif s.init == "one":
            v = torch.ones(s.numel)
        else:
            v = torch.zeros(s.numel)
        flat[s.offset:s.offset + s.numel] = v
    state = torch.zeros(STATE_SIZE)
    for s in STATE_SPECS:
        if s.init == "one":
            state[s.offset:s.offset + s.numel] = 1.0
    return flat, state


def _views(buf: torch.Tensor, specs) -> Dict[str, torch.Tensor]:
    return {s.name[len(SCOPE) + 1:]: buf[s.offset:s.offset + s.numel].view(s.shape) for s in specs}


def _conv3x3(x, k, stride):
    # x NCHW, k HWIO; SAME padding for 3x3 at stride 1/2 on even sizes: pad (1,1) at s1, (0,1) at s2
    w = k.permute(3, 2, 0, 1)
    if stride == 1:
        return F.conv2d(x, w, padding=1)
    return F.conv2d(F.pad(x, (0, 1, 0, 1)), w, stride=2)


def _bn(x, p, st, prefix, training):
    gamma, beta = p[f"{prefix}/bn/gamma"], p[f"{prefix}/bn/beta"]
    rm, rv = st[f"{prefix}/bn/moving_mean"], st[f"{prefix}/bn/moving_variance"]
    return F.batch_norm(x, rm, rv, gamma, beta, training=training, momentum=BN_MOMENTUM, eps=BN_EPS)


def resnet20_forward(images_nhwc: torch.Tensor, p: Dict[str, torch.Tensor], st: Dict[str, torch.Tensor],
                     training: bool = True) -> torch.Tensor:
    x = images_nhwc.permute(0, 3, 1, 2)
    x = F.relu(_bn(_conv3x3(x, p["stem/conv/kernel"], 1), p, st, "stem", training))
    cin = WIDTHS[0]
    for s, wdt in enumerate(WIDTHS):
        for b in range(BLOCKS):
            stride = 2 if (s > 0 and b == 0) else 1
            pre = f"stage{s}/block{b}"
            y = F.relu(_bn(_conv3x3(x, p[f"{pre}/a/conv/kernel"], stride), p, st, f"{pre}/a", training))
            y = _bn(_conv3x3(y, p[f"{pre}/b/conv/kernel"], 1), p, st, f"{pre}/b", training)
            sc = x
            if stride == 2 or cin != wdt:      # option A: subsample + zero-pad channels
                sc = x[:, :, ::2, ::2] if stride == 2 else x
                sc = F.pad(sc, (0, 0, 0, 0, 0, wdt - cin))
            x = F.relu(y + sc)
            cin = wdt
    x = x.mean(dim=(2, 3))
    return x @ p["fc/weights"] + p["fc/biases"]


class ResNet20(nn.Module):
    specs = PARAM_SPECS
    state_specs = STATE_SPECS

    def __init__(self, flat: torch.Tensor | None = None, seed: int = 0, relu_logits: bool = False):
        super().__init__()
        f0, s0 = init_flat_params(torch.Generator().manual_seed(seed))
        if flat is not None:
            f0 = flat.clone().float()
        self.flat = nn.Parameter(f0)
        self.register_buffer("state", s0)
        self.relu_logits = relu_logits

    def forward(self, images_nhwc: torch.Tensor) -> torch.Tensor:
        logits = resnet20_forward(images_nhwc, _views(self.flat, PARAM_SPECS), _views(self.state, STATE_SPECS),
                                  self.training)
        return F.relu(logits) if self.relu_logits else logits

    def grad_buckets(self):
        return [(0, FLAT_SIZE)]

    def named_tf_variables(self) -> Dict[str, torch.Tensor]:
        d = {s.name: self.flat.detach()[s.offset:s.offset + s.numel].view(s.shape) for s in PARAM_SPECS}
        d.update({s.name: self.state[s.offset:s.offset + s.numel].view(s.shape) for s in STATE_SPECS})
        return d
