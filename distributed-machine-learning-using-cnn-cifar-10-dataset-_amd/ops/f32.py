"""fp32-accurate CNN path on hand-written HIP kernels (``--dtype fp32`` on the GPU).

The reference keeps every variable and op in ``tf.float32`` (/root/reference/cifar10cnn.py:97-145,
loss/SGD :150-164).  The fused engine trains in bf16 (fp32 accumulation and fp32 master weights);
this module is the reference-precision alternative on the same kind of native code: every
matrix product of the step -- conv forward, conv weight/data gradients, the three fc layers and
their gradients -- runs on ``torch.ops.dmlc.f32_gemm`` (fp32 MFMA ``v_mfma_f32_16x16x4_f32``, true
fp32 operands, deterministic split-K).  The two convolutions are implicit GEMMs
(``f32_conv_gemm``: the tile loader gathers the im2col matrix straight from the NHWC activation):
forward = im2col(x) W, weight + bias gradient = im2col(x)^T dY with a ones column (its output row
is the bias gradient), data gradient = im2col(dY) against the flipped, transposed weight -- no
column matrix is ever written.  Other geometries (e.g. another crop) use ``f32_im2col`` + GEMM with
the gather-form ``f32_col2im`` adjoint.  fc bias gradients: ``f32_colsum``.  ReLU, the TF-SAME max-pool and the loss
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


_IMPLICIT = {(24, 3), (12, 64)}          # (H, C) geometries of f32_conv_gemm (5x5, pad 2)


class _ConvImplicit(torch.autograd.Function):
    """Stride-1 TF-'SAME' 5x5 convolution as implicit GEMMs (no column matrix in memory)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ops = _ops()
        B, H, W, C = x.shape
        co = w.shape[3]
        x = x.contiguous()
        wm = w.contiguous().view(25 * C, co)
        y = ops.f32_conv_gemm(x, wm, b.contiguous(), False, False)
        ctx.save_for_backward(x, w)
        return y.view(B, H, W, co)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        ops = _ops()
        B, H, W, C = x.shape
        co = w.shape[3]
        gy = gy.contiguous()
        gwb = ops.f32_conv_gemm(x, gy.view(B * H * W, co), None, True, True)   # [25*C + 1, co]
        gw, gb = gwb[:25 * C].view(5, 5, C, co), gwb[25 * C]
        gx = None
        if ctx.needs_input_grad[0] and (H, co) in _IMPLICIT:
            # dx = im2col(dY) . W'  with  W'[(kh, kw, co), ci] = W[4-kh, 4-kw, ci, co]
            wt = w.flip(0, 1).permute(0, 1, 3, 2).contiguous().view(25 * co, C)
            gx = ops.f32_conv_gemm(gy, wt, None, False, False).view(B, H, W, C)
        elif ctx.needs_input_grad[0]:          # dY geometry without an implicit kernel: explicit adjoint
            dcols = ops.f32_gemm(gy.view(B * H * W, co), w.contiguous().view(25 * C, co), None, False, True, False)
            gx = ops.f32_col2im(dcols, B, H, W, C, 5, 5, 2)
        return gx, gw, gb


class _ConvSame(torch.autograd.Function):
    """Stride-1 TF-'SAME' KxK convolution, x NHWC [B,H,W,C], w HWIO [K,K,C,CO] -> NHWC (explicit
    im2col; geometries without an implicit kernel)."""

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


def conv_same(x, w, b, implicit: bool = True):
    if implicit and w.shape[0] == 5 and w.shape[1] == 5 and (x.shape[1], x.shape[3]) in _IMPLICIT \
            and x.shape[1] == x.shape[2]:
        return _ConvImplicit.apply(x, w, b)
    return _ConvSame.apply(x, w, b)


def _pool_nhwc(x: torch.Tensor) -> torch.Tensor:
    """TF-SAME 3x3/2 max-pool of an NHWC tensor with no layout copies: for an even input, TF-SAME pads
    one -inf row/column at the bottom/right only, i.e. exactly ceil_mode windows starting at 2i; the
    NCHW view of NHWC memory is channels_last, so the pool runs in place of layout and its output
    permutes back to a contiguous NHWC tensor."""
    y = torch.nn.functional.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, ceil_mode=True).permute(0, 2, 3, 1)
    return y if y.is_contiguous() else y.contiguous()


class _FlatViews(torch.autograd.Function):
    """The per-variable tensors of a flat parameter buffer whose backward builds the flat gradient
    in ONE concatenation (autograd through plain views of a leaf would zero-fill a full-size
    gradient and add into it once per variable: 10 fills + 10 adds of 4.3 MB per step)."""

    @staticmethod
    def forward(ctx, flat, specs):
        ctx.specs, ctx.n = specs, flat.numel()
        return tuple(flat[s.offset:s.offset + s.numel].view(s.shape) for s in specs)

    @staticmethod
    def backward(ctx, *grads):
        parts, pos = [], 0
        ref = next((g for g in grads if g is not None), None)
        if ref is None:
            return None, None
        for s, g in zip(ctx.specs, grads):
            if s.offset > pos:
                parts.append(ref.new_zeros(s.offset - pos))
            parts.append(g.reshape(-1) if g is not None else ref.new_zeros(s.numel))
            pos = s.offset + s.numel
        if ctx.n > pos:
            parts.append(ref.new_zeros(ctx.n - pos))
        return torch.cat(parts), None


def flat_views(flat: torch.Tensor, specs) -> Dict[str, torch.Tensor]:
    from ..models.cifar_cnn import short
    return {short(s.name): v for s, v in zip(specs, _FlatViews.apply(flat, tuple(specs)))}


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
