"""fp32-accurate CNN path on hand-written HIP kernels (``--dtype fp32`` on the GPU).

The reference keeps every variable and op in ``tf.float32`` (/root/reference/cifar10cnn.py:97-145,
loss/SGD :150-164).  The fused engine trains in bf16 (fp32 accumulation and fp32 master weights);
this module is the reference-precision alternative on the same kind of native code: every
matrix product of the step -- conv forward, conv weight/data gradients, the three fc layers and
their gradients -- runs on ``torch.ops.dmlc.f32_gemm`` (fp32 MFMA ``v_mfma_f32_16x16x4_f32``, true
fp32 operands, deterministic split-K), convolutions as ``f32_im2col`` + GEMM with a gather-form
``f32_col2im`` adjoint, bias gradients on ``f32_colsum``.  ReLU, the TF-SAME max-pool and the loss
are fp32 PyTorch ops (exact in fp32; no rounding choice to make).

Activations are NHWC and weights keep the TF layouts (HWIO / [in, out]), so the weights are
views of the model's flat parameter buffer and the im2col column order (kh, kw, ci) is the row
order of the HWIO weight viewed as [kh*kw*ci, co] -- no transposes anywhere.
"""
from __future__ import annotations

from typing import Dict

import torch

from . import _ext


def _ops():
    _ext.hip()          # loud failure when the native library is missing on a GPU box
    return torch.ops.dmlc


class _Linear(torch.autograd.Function):
    """y = x W + b (W stored [in, out])."""

    @staticmethod
    def forward(ctx, x, w, b):
        x, w = x.contiguous(), w.contiguous()
        ctx.save_for_backward(x, w)
        return _ops().f32_gemm(x, w, b.contiguous(), False, False, False)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        ops = _ops()
        gy = gy.contiguous()
        gx = ops.f32_gemm(gy, w, None, False, True, False) if ctx.needs_input_grad[0] else None   # dY W^T
        gw = ops.f32_gemm(x, gy, None, True, False, False)                                        # X^T dY
        return gx, gw, ops.f32_colsum(gy)


class _ConvSame(torch.autograd.Function):
    """Stride-1 TF-'SAME' KxK convolution, x NHWC [B,H,W,C], w HWIO [K,K,C,CO] -> NHWC."""

    @staticmethod
    def forward(ctx, x, w, b):
        ops = _ops()
        B, H, W, C = x.shape
        k, co = w.shape[0], w.shape[3]
        cols = ops.f32_im2col(x.contiguous(), k, k, k // 2)                   # [B*H*W, K*K*C]
        wm = w.contiguous().view(k * k * C, co)
        y = ops.f32_gemm(cols, wm, b.contiguous(), False, False, False)
        ctx.save_for_backward(cols, wm)
        ctx.geom = (B, H, W, C, k)
        return y.view(B, H, W, co)

    @staticmethod
    def backward(ctx, gy):
        cols, wm = ctx.saved_tensors
        B, H, W, C, k = ctx.geom
        ops = _ops()
        g2 = gy.contiguous().view(B * H * W, wm.shape[1])
        gw = ops.f32_gemm(cols, g2, None, True, False, False).view(k, k, C, wm.shape[1])
        gb = ops.f32_colsum(g2)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = ops.f32_col2im(ops.f32_gemm(g2, wm, None, False, True, False), B, H, W, C, k, k, k // 2)
        return gx, gw, gb


def linear(x, w, b):
    return _Linear.apply(x, w, b)


def conv_same(x, w, b):
    return _ConvSame.apply(x, w, b)


def _pool_nhwc(x: torch.Tensor) -> torch.Tensor:
    from ..models.cifar_cnn import tf_same_maxpool_3x3s2
    return tf_same_maxpool_3x3s2(x.permute(0, 3, 1, 2)).permute(0, 2, 3, 1).contiguous()


def cnn_forward_f32(images_nhwc: torch.Tensor, p: Dict[str, torch.Tensor], relu_logits: bool = True) -> torch.Tensor:
    """The reference CNN (models/cifar_cnn.py:cnn_forward semantics) on the fp32 HIP kernels."""
    x = images_nhwc.float().contiguous()
    x = _pool_nhwc(torch.relu(conv_same(x, p["conv1_kernel"], p["conv1_bias"])))
    x = _pool_nhwc(torch.relu(conv_same(x, p["conv2_kernel"], p["conv2_bias"])))
    x = x.reshape(x.shape[0], -1)                                  # NHWC flatten (cifar10cnn.py:126)
    x = torch.relu(linear(x, p["full_weight_1"], p["full_bias_1"]))
    x = torch.relu(linear(x, p["full_weight_2"], p["full_bias_2"]))
    x = linear(x, p["full_weight_3"], p["full_bias_3"])
    return torch.relu(x) if relu_logits else x
