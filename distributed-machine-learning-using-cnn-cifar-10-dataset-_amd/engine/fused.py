"""Fused MI355X training engine for the reference CNN (hand-written HIP kernels + HIP graphs + RCCL).

One training step (= one ``mon_sess.run([train_op, loss])`` of /root/reference/cifar10cnn.py:230,
SURVEY.md §3.3) is THREE kernel launches on the single-GPU bf16 path at 128 < B <= 256, all reading
their inputs from device memory:

  1 conv12_fwd   uint8 gather + center crop + conv1 + bias + ReLU + pool1 (+argmax), handed through
                 LDS to conv2 + bias + ReLU + pool2 (+argmax) -- one workgroup per image
  2 fc_chain     one persistent launch (cnn_fc.hip): fc1 forward (split-K tiles) -> MLP head (fc1
                 reduce / bias / ReLU, fc2, fc3, ReLU logits, softmax xent, accuracy, dlogits -> dh2 ->
                 dh1) -> dp2 = dh1 W1^T tiles + the fc weight-gradient tiles with the fc1 SGD in their
                 epilogue -> the conv2 input gradient of each workgroup's image (pool2/ReLU backward
                 gather + conv2 dgrad, conv2_core.h) once its dp2 row tile is published
  3 wgrad        pool1/ReLU backward + conv1 weight/bias gradients and conv2 weight/bias gradients
                 (split-K slabs), then -- on one GPU -- the whole rest of the SGD in the same launch
                 (sub-grid barrier per slab family, every block reduces its share in the SGD kernel's
                 order and applies the update + bf16 shadows; the stats, global_step and the next
                 step's batch rows too)

At B <= 128 launch 1 is k_conv12_fwd_split (cnn_split.hip: conv1 -> pool1 -> conv2 -> pool2 in ONE
launch with two workgroups per image that swap their pool1 channel halves through write-through
stores + a flag, so a small batch fills the 256 CUs) and the fc chain's 256 workgroups run the conv2
input gradient two per image (cnn_split.hip's channel halves): three launches as well.  B > 256 (and
ranks sharing one GPU) use the three-launch fc path (grouped fc1 GEMM, head, grouped backward GEMM).
The fp8 path (BASELINE config 5) runs conv1 and the fp8 conv2 forward as two launches, the fp8 conv2
dgrad as its own launch and the SGD as its own launch.

Data parallel (N > 1): the wgrad launch reduces the conv slabs into the flat gradient instead of
applying them, then the gradient is exchanged and applied -- serial schedule: one all-reduce of the
whole flat gradient (xGMI peer-to-peer kernel or RCCL) and one SGD launch; overlap schedule: the fc
bucket's all-reduce on a comm stream beside the wgrad launch, the conv bucket after it on the same
stream, the conv SGD on the main stream and the fc SGD on the comm stream beside the NEXT step's
forward (_dp_step).  bench.py times both before the timed region and keeps the
faster (tune_schedule).

Every data-consuming kernel computes its batch rows from the device-resident global_step and the
generated epoch order (data/order.py: a keyed Feistel permutation per epoch, no index buffer), so
the whole step is a static HIP graph and ``k`` consecutive steps -- across epoch boundaries -- are
one graph replay.  Any batch size works: the kernels run on the batch padded to the 16-row tile and
the head gives padding rows zero loss weight (their gradients are exactly zero).

Variants: every default below is the measured-fastest path of its configuration; the alternatives
that stay are the bitwise references the tests compare against, selected with the ``variant``
dict of the constructor (VARIANT_DEFAULTS).  Three environment switches turn a persistent,
co-residency-dependent launch off without code changes (a training run builds the engine without a
``variant``): DMLC_FC_FUSED=0 (the fc chain), DMLC_WGRAD_SGD=0 (the in-launch SGD / slab reduction of
the wgrad launch) and DMLC_FWD12_SPLIT=0 (the B <= 128 forward whose two workgroups per image wait on
each other).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional

import torch

from .. import config as C
from ..parallel.dist import quiesce_for_capture
from ..data.order import OrderSpec
from ..models import cifar_cnn as M
from ..ops import _ext

OPS = None


def _ops():
    global OPS
    if OPS is None:
        _ext.hip()
        OPS = torch.ops.dmlc
    return OPS


SEG_OFF = [s.offset for s in M.PARAM_SPECS]


def head_rows(B: int) -> int:
    """Batch rows per workgroup of the three-launch path's head kernel: 2 up to B=256 (more
    workgroups on the otherwise idle chip, profiles/r2_v26_head_rows_groups_sweep.txt), 4 above
    (each workgroup streams all of fc2)."""
    return 2 if B <= 256 else 4


# The engine's path choices (constructor ``variant=``).  None = chosen per configuration.
VARIANT_DEFAULTS = {
    "split_fwd": False,        # conv1 and conv2 forward as two launches (bitwise reference of conv12_fwd)
    "fc_fused": None,          # the persistent fc chain (B <= 256, one rank per GPU); env DMLC_FC_FUSED=0 off
    "fc_dgrad": None,          # conv2 dgrad inside the fc chain (default: on; two workgroups per image at B <= 128)
    "fc_dw_in_wgrad": None,    # fc dW tiles in the wgrad launch (default: only when the dgrad is not in the chain)
    "fc1_epilogue": True,      # single GPU: the fc1 update in the dW1 epilogue
    "wgrad_sgd": True,         # in-launch SGD / slab reduction of the wgrad launch; env DMLC_WGRAD_SGD=0 off
    "wgrad_sgd_fp8": False,    # the same for --dtype fp8 (bit-identical, measured 1.4 % slower at B=1024)
    "fp8_dgrad": True,         # fp8: the conv2 input gradient on e4m3 too
    "fp8_wgrad": True,         # fp8 (with fp8_dgrad): the conv2 weight gradient on e4m3 MFMA (per-batch scales)
    "comm_sgd": False,         # data parallel over xGMI: the SGD in the exchange kernel's epilogue
    "xraw_prefetch": True,     # the step's raw images gathered by the previous step's finalizer
    "fwd12_split": True,       # B <= 128: conv1 + conv2 forward in one launch, two workgroups per image;
                               # env DMLC_FWD12_SPLIT=0 off
    "fc_sgd_in_chain": None,   # single GPU, dW tiles in the fc chain: every fc SGD in their epilogues (default B < 256)
    "grad16": True,            # data parallel, RCCL, bf16 wire, fc chain: the producers write a bf16 flat gradient
                               # (no cast launches around the all-reduce; bitwise the cast path)
}
# int32 words of the SGD arrival ticket (DMLC_TICKET_WORDS in csrc/kernels/api.h)
TICKET_WORDS = 9 * 32
# int32 words of the wgrad apply-mode barriers (DMLC_WBAR_WORDS); the last line is the error word
WBAR_WORDS = 20 * 32
SEG = {M.short(s.name): s for s in M.PARAM_SPECS}


def _gemm_params(M_, N_, K_, lda, a_kmajor, ldb, b_kmajor, ldc, c_mode, ksplit=1, relu=0, nvalid=None, b_par=0,
                 s_par=0):
    return [M_, N_, K_, lda, a_kmajor, ldb, b_kmajor, ldc, c_mode, ksplit, relu, N_ if nvalid is None else nvalid,
            b_par, s_par]


FC1_NUMEL = 2304 * 384


class FusedCifarEngine:
    """Owns every device buffer of the fused step.  Not an nn.Module: parameters live in one flat
    fp32 buffer (``self.master``) in the TF checkpoint layout; see models/cifar_cnn.py."""

    def __init__(self, batch_size: int, data: torch.Tensor, labels: torch.Tensor, *, device=None,
                 flat_params: Optional[torch.Tensor] = None, lr: float = C.LEARNING_RATE,
                 lr_decay: float = C.LR_DECAY, decay_steps: float = C.NUM_GENS_TO_WAIT, staircase: bool = True,
                 relu_logits: bool = True, crop_offset=(4, 4), world_size: int = 1, rank: int = 0,
                 process_group=None, seed: int = 0, fc1_split: Optional[int] = None, g1: Optional[int] = None,
                 g2: Optional[int] = None, stats_len: int = 4096, comm_dtype: str = "fp32",
                 capture_comm: Optional[bool] = None, dtype: str = "bf16", allreduce: str = "auto",
                 dp_schedule: str = "serial", dp_force: bool = False, warmup_steps: int = 0,
                 conv_split: Optional[int] = None, conv1_split: Optional[int] = None,
                 dgrad_split: Optional[int] = None, variant: Optional[dict] = None):
        unknown = set(variant or {}) - set(VARIANT_DEFAULTS)
        if unknown:
            raise ValueError(f"unknown engine variant keys {sorted(unknown)}")
        V = dict(VARIANT_DEFAULTS, **(variant or {}))
        self.variant = V
        ops = _ops()
        self.ops = ops
        self.device = torch.device(device or "cuda")
        dev = self.device
        Bv = int(batch_size)
        if Bv < 1:
            raise ValueError("batch size must be >= 1")
        B = -(-Bv // 16) * 16              # kernel batch: padded to the 16-row MFMA tile
        self.B, self.Bv = B, Bv
        self.world_size, self.rank, self.pg = world_size, rank, process_group
        # dp_force: run the data-parallel step (all-reduce + apply) even at world_size 1 -- exercises
        # the collective path (e.g. a captured RCCL all-reduce) on a single GPU
        self.dp = world_size > 1 or dp_force
        self.lr0, self.decay, self.decay_steps, self.staircase = lr, lr_decay, decay_steps, staircase
        self.warmup = float(warmup_steps)      # linear LR warm-up (large-batch recipe), in the SGD kernel
        self.relu_logits = relu_logits
        self.cy, self.cx = crop_offset
        self.comm_dtype = comm_dtype
        if capture_comm is None:     # RCCL collectives go into the step graph unless told otherwise
            capture_comm = self.dp and self._pg_backend() == "nccl"
        self.capture_comm = bool(capture_comm)
        self.seed = seed
        if dtype not in ("bf16", "fp8"):
            raise ValueError("fused engine dtype must be bf16 or fp8")
        self.dtype = dtype

        # --- data (device resident) ---------------------------------------------------------
        assert data.dtype == torch.uint8 and tuple(data.shape[1:]) == (32, 32, 3)
        self.data = data.to(dev).contiguous()
        self.labels = labels.to(dev, torch.int32).contiguous()
        self.n_data = self.data.shape[0]
        self.order = OrderSpec(self.n_data, Bv, world_size, rank, seed)
        self.period = self.order.period          # steps per epoch
        self.order_desc = self.order.descriptor()   # host int64 [6]: the generated order
        # this step's batch rows (int32 [B], rows >= Bv repeat the last): written for step s+1 by the
        # finalizing SGD launch of step s (cnn_sgd.hip), so each data kernel reads one index per row;
        # set from the host whenever the step counter is set from the host
        self.bidx = torch.zeros(B, dtype=torch.int32, device=dev)
        # raw uint8 images of the step's rows, written by the forward for the conv1 weight gradient
        self.xraw = torch.zeros(B, 3072, dtype=torch.uint8, device=dev)

        # --- parameters + shadows -------------------------------------------------------------
        if flat_params is None:
            flat_params = M.init_flat_params(torch.Generator().manual_seed(seed))
        self.master = flat_params.to(dev, torch.float32).contiguous().clone()
        # gradient all-reduce: xGMI peer-to-peer kernel over an IPC-shared grad buffer when every
        # rank can map every peer and it measures faster than RCCL (parallel/xgmi.py), else RCCL
        self.xgmi, self.comm_info = None, {"allreduce": "rccl" if self.dp else "none"}
        self._buckets = {True: (M.FC_BUCKET_OFFSET, self.master.numel() - M.FC_BUCKET_OFFSET),
                         False: (0, M.FC_BUCKET_OFFSET)}
        if world_size > 1 and dev.type == "cuda" and comm_dtype in ("fp32", "bf16") and allreduce != "rccl":
            from ..parallel import xgmi as X
            # timed on the call pattern the step will issue: one whole-buffer all-reduce (serial) or
            # the fc bucket then the conv bucket (overlap)
            pattern = ([(0, self.master.numel())] if dp_schedule == "serial"
                       else [self._buckets[True], self._buckets[False]])
            self.xgmi, self.comm_info = X.select(self.master.numel(), rank, world_size, dev, pattern,
                                                 mode=allreduce, group=process_group, wire=comm_dtype,
                                                 captured=self.capture_comm)
        elif dp_force and world_size == 1 and allreduce == "xgmi" and dev.type == "cuda":
            # a one-rank xGMI context (no peers): the DP step's exchange kernel on a single GPU
            from ..parallel import xgmi as X
            self.xgmi = X.XgmiAllReduce(self.master.numel(), 0, 1, None, wire=comm_dtype)
            self.comm_info = {"allreduce": "xgmi", "wire": comm_dtype}
        if self.xgmi is not None:
            self.grad = self.xgmi.buf[:self.master.numel()]
            self.grad.zero_()
        else:
            self.grad = torch.zeros_like(self.master)
        bf = torch.bfloat16
        z = lambda *s, dt=bf: torch.zeros(*s, dtype=dt, device=dev)
        self.w1f, self.w2f, self.w2d = z(64, 96), z(64, 1600), z(64, 1600)
        # fc1's bf16 shadow is double-buffered by step parity ([2][2304][384]): the kernels of step s
        # read fc1n[s & 1] and the update writes fc1n[(s + 1) & 1], so at N=1 the dW1 GEMM can apply
        # the fc1 update in its epilogue while the dp2 problem of the same launch still reads the
        # current weights (fc1_epilogue below)
        self.fc1n, self.fc2t, self.fc2n = z(2, 2304, 384), z(192, 384), z(384, 192)
        self.fc3t, self.fc3d = z(16, 192), z(192, 32)
        # fp8 conv2 forward + input gradient (BASELINE config 5): e4m3 weight shadows [0] forward
        # (co-major) and [1] the dgrad's flipped ci-major copy, delayed per-tensor weight scale;
        # variant fp8_dgrad=False keeps the conv2 input gradient in bf16
        self.fp8 = dtype == "fp8"
        self.fp8_dgrad = self.fp8 and bool(V["fp8_dgrad"])
        if self.fp8:
            self.w2f8 = z(2, 64, 1600, dt=torch.uint8)
            self.amax_x = z(B, dt=torch.float32)      # per-image activation maxima (conv1 -> conv2)
            self.amax_w = z(2, 400, dt=torch.float32)  # [slot][SGD conv2-row block] weight maxima
            self.scale_w = z(2, dt=torch.float32)
        # fp8 conv2 weight gradient (cnn_wgrad.hip w2_fp8_main): the e4m3 X the fp8 forward quantised
        # (per-batch scale sx) and the e4m3 dY2 the fp8 dgrad quantised (a power-of-two scale per
        # image, the MFMA's E8M0 block scale), written by those kernels next to their bf16 outputs
        self.fp8_wgrad = self.fp8_dgrad and bool(V["fp8_wgrad"])
        if self.fp8_wgrad:
            self.p1f8, self.dy2f8 = z(B, 144, 64, dt=torch.uint8), z(B, 144, 64, dt=torch.uint8)
            self.sx8, self.sy_img = z(1, dt=torch.float32), torch.ones(B, dtype=torch.float32, device=dev)
        self._w8 = dict(fp8=[self.p1f8, self.dy2f8, self.sx8, self.sy_img]) if self.fp8_wgrad else {}

        # --- activations / workspaces -------------------------------------------------------
        self.fc1_split = fc1_split or self._pick_fc1_split(B)
        # conv1 and conv2 forward in one launch (bf16 path; variant split_fwd: two launches)
        self.fused_fwd = not V["split_fwd"]
        # channel-split convolutions (cnn_split.hip): conv_split = 2 runs conv1 forward (conv1_split =
        # 2 or 4 workgroups per image), conv2 forward and the conv2 input gradient as 2 workgroups per
        # image, so a small batch fills the 256 CUs; 1 = one workgroup per image (cnn_conv.hip).
        # same-session A/B (r3): B=128 73.5 us (split, conv1 2-way) vs 74.6 (conv1 4-way) vs 79.0 (one
        # workgroup per image); B=256 85.1 vs 82.9 -- the split pays only while the chip is not full
        self.conv_split = 1 if self.fp8 else (conv_split or (2 if B <= 128 else 1))
        self.conv1_split = conv1_split or 2
        # the conv2 input gradient's split, independently of the forward's
        self.dgrad_split = 1 if self.fp8 else (dgrad_split or self.conv_split)
        if self.conv_split not in (1, 2) or self.conv1_split not in (2, 4) or self.dgrad_split not in (1, 2):
            raise ValueError(f"conv_split / dgrad_split must be 1 or 2 and conv1_split 2 or 4 "
                             f"({self.conv_split}, {self.dgrad_split}, {self.conv1_split})")
        self.keep_dp1 = False          # tests: also write the pool1 gradient to global memory
        # Both weight gradients run in ONE launch (ops.wgrad) of g1 + 4 * g2 <= 256 blocks (one wave
        # of workgroups): conv2 one block per (input-channel quarter, image group), one fp32 slab per
        # group (g2 = slabs the reduction sums); conv1 one block per image group on the CUs the conv2
        # blocks leave.  Multiples of 8 keep every group's images on one XCD (cnn_wgrad.hip).
        # B=128: 32 groups of 4 images -> 69.2 us per step vs 16 groups of 8 -> 73.7 (r3 sweep);
        # B=256: 32 -> 81.7 vs 24 -> 85.1, 40 -> 83.1, 48 -> 86.8.  Past B=256 every conv1 block takes
        # several images instead of the grid growing beyond the chip.
        g2_ = max(1, min(B, 32, B // 4))
        self.g2 = g2 or (g2_ // 8 * 8 if g2_ >= 8 else g2_)
        self.g1 = g1 or max(1, min(B, 256 - 4 * self.g2))
        self.groups2 = self.g2
        self.p1, self.am1 = z(B, 12, 12, 64), z(B, 12, 12, 64, dt=torch.uint8)
        self.p2, self.am2 = z(B, 6, 6, 64), z(B, 6, 6, 64, dt=torch.uint8)
        self.h1part = z(self.fc1_split, B, 384, dt=torch.float32)
        self.h1, self.h2, self.dl = z(B, 384), z(B, 192), z(B, 16)
        self.dh1, self.dh2 = z(B, 384), z(B, 192)
        self.dp2 = z(B, 6, 6, 64)
        self.dp1, self.dy2 = z(B, 12, 12, 64), z(B, 144, 64)
        # conv weight-gradient slabs: fp32 partial sums over 1/g of the batch each, summed in fixed
        # order.  (bf16 conv2 slabs measured 1.3 us/step faster in r3 but added a 4e-4 relative error
        # to the conv2 weight gradient and a 7 % drift in the loss-curve parity test: not kept.)
        self.part2, self.partb2 = z(self.g2, 1600, 64, dt=torch.float32), z(self.g2, 64, dt=torch.float32)
        self.part1, self.partb1 = z(self.g1, 80, 64, dt=torch.float32), z(self.g1, 64, dt=torch.float32)
        # the whole fc chain of a training step (fc1 forward, head, fc backward) as ONE persistent
        # launch (cnn_fc.hip) instead of three: B <= 256, 256 co-resident workgroups (one per CU, so
        # not when several ranks share a GPU).  DMLC_FC_FUSED=0 turns it off.
        local_ = int(os.environ.get("LOCAL_WORLD_SIZE", world_size))
        ndev_ = torch.cuda.device_count() if dev.type == "cuda" else 0
        cus = torch.cuda.get_device_properties(dev).multi_processor_count if dev.type == "cuda" else 0
        fc_ok = B <= 256 and cus >= 256 and local_ <= max(1, ndev_)
        self.fc_fused = (fc_ok if V["fc_fused"] is None else bool(V["fc_fused"]) and fc_ok) \
            and os.environ.get("DMLC_FC_FUSED", "1") != "0"
        self.h1part8 = z(8, B, 384, dt=torch.float32) if self.fc_fused else None
        self.fc_sync = torch.zeros(212 * 32, dtype=torch.int32, device=dev)   # fc_common.h SY_END
        self._fc_src = None
        # head: head_rows(B) batch rows per workgroup (B / rows workgroups share the fc2 weight reads);
        # the fused fc chain's head takes 4 rows per workgroup
        hr = 4 if self.fc_fused else head_rows(B)
        self.loss_part = z(B // hr, dt=torch.float32)
        self.correct_part = z(B // hr, dt=torch.int32)
        self.step_t = torch.zeros(1, dtype=torch.int64, device=dev)
        # the head kernel copies the step counter here; the SGD (launch or in-launch) reads the copy,
        # so one of its workgroups can bump step_t without an arrival ticket (cnn_sgd.hip)
        self.step_sgd = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ticket = torch.zeros(TICKET_WORDS, dtype=torch.int32, device=dev)   # two-level arrival counters
        self.stats = torch.zeros(stats_len, 4, dtype=torch.float32, device=dev)
        self.logits_buf = z(B, 10, dt=torch.float32)

        p = {k: self.master[s.offset:s.offset + s.numel] for k, s in SEG.items()}
        self.pv = p
        gv = {k: self.grad[s.offset:s.offset + s.numel] for k, s in SEG.items()}
        self.gv = gv
        # data parallel over RCCL with the bf16 wire: the fc chain (its dW tiles), the wgrad launch's
        # conv-slab reduction / the reduce-only SGD launch write the gradient as bf16 into grad16, the
        # all-reduce runs on it in place and the apply-only SGD reads it (DmlcSgdArgs::grad16) -- the
        # fp32 gradient + t.to(bf16) + all-reduce + copy back, bit for bit, minus two cast launches of
        # 4.27 / 2.1 MB (world-1 A/B: +13.1 us over the single-GPU step with the casts vs +5.7 fp32,
        # profiles/r6s2_dp1_ab_grad16_bf16.jsonl).  The three-launch fc path writes fp32 only: fc chain
        # engines (B <= 256, a GPU per rank) only.
        self.grad16 = None
        if (self.dp and comm_dtype == "bf16" and self.xgmi is None and self.fc_fused and bool(V["grad16"])):
            self.grad16 = torch.zeros(self.master.numel(), dtype=torch.bfloat16, device=dev)
        self.gv_chain = ({k: self.grad16[s.offset:s.offset + s.numel] for k, s in SEG.items()}
                         if self.grad16 is not None else gv)

        # grouped GEMM problem lists (the three-launch fc path)
        self._fc1_fwd = dict(A=[self.p2.view(B, 2304)], B=[self.fc1n], C=[self.h1part], bias=[None],
                             params=_gemm_params(B, 384, 2304, 2304, 1, 384, 0, 384, 2, self.fc1_split,
                                                 b_par=FC1_NUMEL))
        self._fc_bwd = dict(
            A=[self.dh1, self.p2.view(B, 2304), self.h1, self.h2, self.dh1, self.dh2, self.dl],
            B=[self.fc1n, self.dh1, self.dh2, self.dl, self.dh1, self.dh2, self.dl],
            C=[self.dp2.view(B, 2304), gv["full_weight_1"], gv["full_weight_2"], gv["full_weight_3"],
               gv["full_bias_1"], gv["full_bias_2"], gv["full_bias_3"]],
            bias=[None] * 7,
            params=(_gemm_params(B, 2304, 384, 384, 1, 384, 1, 2304, 1, b_par=FC1_NUMEL)  # dp2 = dh1 W1^T
                    + _gemm_params(2304, 384, B, 2304, 0, 384, 0, 384, 0)          # dW1 = p2^T dh1
                    + _gemm_params(384, 192, B, 384, 0, 192, 0, 192, 0)            # dW2 = h1^T dh2
                    + _gemm_params(192, 16, B, 192, 0, 16, 0, 10, 0, nvalid=10)    # dW3 = h2^T dl
                    + _gemm_params(384, 8, B, 384, 0, 8, 0, 1, 3, nvalid=384)      # db1
                    + _gemm_params(192, 8, B, 192, 0, 8, 0, 1, 3, nvalid=192)      # db2
                    + _gemm_params(16, 8, B, 16, 0, 8, 0, 1, 3, nvalid=10)))       # db3
        fb = self._fc_bwd
        # single GPU: the same launch with dW1 as a fused SGD epilogue (c_mode 4) -- the fc1 weights
        # (83 % of the parameters) are updated where their gradient is produced instead of the fp32
        # gradient going through HBM to the SGD kernel (which then updates the fc1 bias only).
        # Bitwise the same update (same lr expression, same fp32 arithmetic); variant fc1_epilogue off
        self.fc1_epilogue = not self.dp and bool(V["fc1_epilogue"])
        # single GPU + fc1 epilogue: the merged weight-gradient launch also runs the rest of the SGD
        # (cnn_wgrad.hip apply mode: sub-grid barriers per slab family, the SGD kernel's reduction
        # order -> bit-identical weights) and the step has no SGD launch.  DMLC_WGRAD_SGD=0 off.
        in_launch = (1 <= self.g1 <= cus and 4 * self.g2 <= cus and bool(V["wgrad_sgd"])
                     and os.environ.get("DMLC_WGRAD_SGD", "1") != "0")
        # fp8: bit-identical too (the e4m3 shadows + amax slots in-launch), but measured slower at
        # B=1024 (207.5 vs 204.7 us, profiles/r3_fp8_wgrad_sgd_ab.txt): variant wgrad_sgd_fp8 opts in
        self.wgrad_apply = in_launch and self.fc1_epilogue and (not self.fp8 or bool(V["wgrad_sgd_fp8"]))
        # data parallel: the same launch reduces the conv slabs into the flat gradient (the reduce-only
        # SGD launch before the all-reduce goes away).  Needs the launch's blocks co-resident, so not
        # when several ranks share one GPU (rehearsals / tests: another rank's kernels hold CUs).
        local = int(os.environ.get("LOCAL_WORLD_SIZE", world_size))
        ndev = torch.cuda.device_count() if dev.type == "cuda" else 0
        reduce_ok = in_launch and self.dp and local <= max(1, ndev)
        # reduce-only also serves compute_gradients() on one GPU (fp8 included: bit for bit the
        # two-launch path, tests/test_fp8_gpu.py)
        self._grad_in_launch = in_launch and (self.wgrad_apply or reduce_ok)
        # the data-parallel step takes the in-launch reduction exactly when compute_gradients() does
        # (one predicate: the DP step and _conv_backward can never disagree)
        self.wgrad_reduce = self.dp and self._grad_in_launch
        # data parallel over xGMI, serial schedule, variant comm_sgd: the exchange kernel applies the
        # SGD in its epilogue (k_xgmi_allreduce_sgd: no SGD launch; bit-identical weights; bf16 shadows
        # only).  Off by default: measured on one GPU (tools/dp1_ab.py, world-1 xGMI context, B=256)
        # the DP step took 103.0 us with the epilogue on the exchange's 128 workgroups and 142.2 us on
        # 512 (every workgroup pays the barriers' system-scope release fences) vs 96.2 us for exchange
        # + the 800-workgroup SGD launch (profiles/r5_dp1_ab_128blocks.jsonl, r5_dp1_ab_512blocks.jsonl).
        self.comm_sgd = self.xgmi is not None and not self.fp8 and bool(V["comm_sgd"])
        # workgroups of the exchange + SGD kernel: 2 per CU on a GPU of its own (the epilogue streams
        # the whole flat buffer); ranks sharing one GPU (rehearsals) split the workgroups, since every
        # workgroup waits at the barriers for the same-index workgroup of every peer
        share = max(1, -(-int(os.environ.get("LOCAL_WORLD_SIZE", world_size)) // max(1, ndev)))
        self._comm_blocks = 512 if share == 1 else max(32, 128 // share)
        # the training forward (conv12_fwd) reads its raw images from xraw, which the previous step's
        # finalizer (wgrad apply mode, the SGD launch or the xGMI+SGD kernel) filled with the next
        # step's rows -- one image load instead of index load -> image load at the head of the step;
        # the host fills it whenever it sets the step (_sync_bidx)
        self.xraw_prefetch = self.fused_fwd and not self.fp8 and self.conv_split == 1 and bool(V["xraw_prefetch"])
        # B <= 128 (channel-split convs, conv1 in halves): conv1 -> conv2 in ONE launch whose two
        # workgroups per image swap their pool1 halves through sc1 stores + a flag (cnn_split.hip
        # k_conv12_fwd_split) -- one launch boundary and the conv2 input's global round trip less
        self.fwd12_split = (self.conv_split == 2 and self.conv1_split == 2 and not self.fp8
                            and B * 2 <= cus and local_ <= max(1, ndev_) and bool(V["fwd12_split"])
                            and os.environ.get("DMLC_FWD12_SPLIT", "1") != "0")
        self.c12_flags = torch.zeros(32 * 2 * B if self.fwd12_split else 1, dtype=torch.int32, device=dev)
        self.wbar = torch.zeros(WBAR_WORDS, dtype=torch.int32, device=dev)   # barrier words + error word
        # pinned host copy of the barrier error word, refreshed by queue_error_copy() behind each
        # chunk of steps (the trainer checks it at every progress point without a device sync)
        self._err_host = (torch.zeros(1, dtype=torch.int32).pin_memory() if dev.type == "cuda"
                          else torch.zeros(1, dtype=torch.int32))
        # the plain bf16 conv2 dgrad (one image per workgroup) runs in the fc chain's workgroups, each
        # once its dp2 row tile is published: one launch boundary less, but the hand-off (publish ->
        # poll -> sc1 dp2 loads) costs ~2 us of it back.  With the fc dW tiles kept in the chain (below)
        # it measured 1.8-2.5 us/step faster at B = 144 / 160 / 192 / 224 / 256 (profiles/
        # r4_v8_fc_dgrad_b144_256_ab.txt); at B <= 128 the chain's 256 workgroups run the split dgrad
        # (two per image, cnn_split.hip's halves) instead of its own launch (r5, profiles/
        # r5_fc_split_dgrad_b128_ab.txt).  Variant fc_dgrad forces it on / off.
        fdg = V["fc_dgrad"]
        self.fc_dgrad = self.fc_fused and not self.fp8_dgrad and (bool(fdg) if fdg is not None else True)
        self._dgrad_done = False
        # single GPU, fused fc chain + apply mode: the fc weight-gradient tiles and every fc SGD can run
        # in the wgrad launch's conv1 blocks (between their barrier arrival and the conv1 reduction),
        # so the fc chain launch ends with its dp2 tiles.  Same-box A/B at B=256 (profiles/
        # r4_v7_fc_dgrad_dw_ab.txt, us/step): chain dgrad off: dW in chain 81.8, in wgrad 80.4; chain
        # dgrad on: dW in chain 79.8, in wgrad 80.2 -- so by default the dW tiles move to the wgrad
        # launch only when the dgrad is not in the chain.  Variant fc_dw_in_wgrad forces it.
        # At B <= 128 (the chain's split dgrad) the dW tiles once measured better in the wgrad launch
        # (64.2-64.4 vs 65.6-65.9 us at B = 128, profiles/r5_fc_split_dgrad_b128_ab.txt) -- with the
        # conv1 blocks then too busy to help reduce the conv2 slabs.  With the tiles in the chain the
        # conv1 blocks help again (torch_ops.cpp: helpers whenever they carry no fc tiles): B = 32 71.6
        # -> 64.0, 64 65.3 -> 62.7, 96 65.8 -> 64.7, 112 67.5 -> 65.5, 128 63.6 -> 63.6 us
        # (profiles/r5_dw_placement_helpers_ab.txt).
        fdw = V["fc_dw_in_wgrad"]
        self.fc_dw_in_wgrad = (self.fc_fused and self.wgrad_apply
                               and (bool(fdw) if fdw is not None else not self.fc_dgrad))
        # ... and with the tiles in the chain, the chain can apply every fc SGD in their epilogues (fc2 /
        # fc3 / fc biases too, as the wgrad launch does when it runs them): the wgrad launch's conv1
        # blocks then have no fc SGD roles before their conv1 reduction and conv2 help, while the
        # chain's dW2 / dW3 tiles (whose images' dgrads end the chain) carry the transposed-shadow
        # epilogues.  Same-box A/B (profiles/r5_fc_sgd_in_chain_ab.txt): B = 64 / 128 / 160 / 192 / 224
        # -0.9 / -0.3 / -0.5 / -0.9 / -0.7 us, B = 256 +0.9 us -- on below B = 256.
        fsc = V["fc_sgd_in_chain"]
        self.fc_sgd_in_chain = (self.fc_fused and self.wgrad_apply and not self.fc_dw_in_wgrad
                                and (bool(fsc) if fsc is not None else B < 256))
        self._fc_bwd_sgd = dict(fb, C=[fb["C"][0], p["full_weight_1"]] + fb["C"][2:],
                                params=fb["params"][:14] + _gemm_params(2304, 384, B, 2304, 0, 384, 0, 384, 4,
                                                                        s_par=FC1_NUMEL)
                                + fb["params"][28:])

        self.graphs: List[torch.cuda.CUDAGraph] = []
        self.chains: Dict[int, Optional[torch.cuda.CUDAGraph]] = {}   # k -> graph of k chained steps
        self.comm_stream = torch.cuda.Stream(device=dev) if self.dp else None
        # N>1 step schedule: "overlap" = two buckets, fc all-reduce + fc SGD on the comm stream under
        # the conv backward; "serial" = one stream, one all-reduce of the whole flat gradient, one SGD
        # launch (no fork/join, no co-resident comm/SGD blocks slowing the conv kernels).
        # tune_schedule() measures both and keeps the faster.
        assert dp_schedule in ("overlap", "serial"), dp_schedule
        self.dp_schedule = dp_schedule
        self._captured_schedule = None
        if self.dp:
            self.comm_info.update(schedule=dp_schedule, backend=self._backend(),
                                  captured_comm=bool(self.capture_comm or self.xgmi is not None),
                                  grad_dtype="bf16" if self.grad16 is not None else "fp32")
        self.host_step = 0
        self._sync_bidx()
        self.refresh_shadows()

    # ------------------------------------------------------------------------------------------
    @staticmethod
    def _pick_fc1_split(B: int) -> int:
        # the largest power-of-two split in (8, 4, 2) whose (B/64) * 6 tiles * split workgroups stay
        # <= 450: with the XCD-aware GEMM order (cnn_gemm.hip) every XCD gets its own K slice of p2
        # and W1 (split 8: one slice per XCD).  Whole-step sweeps: tools/sweep_fc.py,
        # profiles/r2_v26_fc1_split_sweep.jsonl.
        tiles = max(1, math.ceil(B / 64)) * 6
        for s in (8, 4, 2):
            if tiles * s <= 450:
                return s
        return 1

    def refresh_shadows(self):
        if self.fp8:    # exact amax of the current W2 for the shadow quantisation at this step
            s = self.host_step & 1
            w2 = self.master[SEG["conv2_kernel"].offset:SEG["conv2_kernel"].offset + SEG["conv2_kernel"].numel]
            self.amax_w[s] = w2.abs().max()
            self.amax_w[s ^ 1] = 0.0
        self._sgd(mode=3)

    def set_step(self, step: int):
        old = int(self.step_t.item())
        if (old ^ int(step)) & 1:      # the current fc1 shadow moves to the new step's parity slot
            self.fc1n[int(step) & 1].copy_(self.fc1n[old & 1])
        self.step_t.fill_(int(step))
        self.step_sgd.fill_(int(step))
        self.host_step = int(step)
        self._sync_bidx()

    def _sync_bidx(self):
        self.bidx.copy_(self._padded(self.batch_indices(self.host_step)))
        self._sync_xraw()

    def _sync_xraw(self):
        """The current step's raw images into xraw (the prefetching forward reads them there)."""
        if getattr(self, "xraw_prefetch", False):
            self.xraw.copy_(self.data.index_select(0, self.bidx.long()).view(self.B, 3072))

    # --- data order ---------------------------------------------------------------------------
    def epoch_permutation(self, epoch: int) -> torch.Tensor:
        """This rank's dataset rows for ``epoch`` (int32 [period * Bv], batch after batch): the
        generated order the kernels evaluate in place (data/order.py; D6: disjoint rank shards)."""
        return self.order.epoch_shard(epoch).to(torch.int32)

    def batch_indices(self, step: int) -> torch.Tensor:
        """Dataset rows (int32 [Bv]) this rank trains on at global step ``step``."""
        return self.order.batch(step).to(torch.int32)

    def _padded(self, idx: torch.Tensor) -> torch.Tensor:
        """An explicit index list of Bv rows padded to the kernel batch (last row repeated)."""
        idx = idx.to(self.device, torch.int32).reshape(-1)
        if idx.numel() == self.B:
            return idx.contiguous()
        assert 1 <= idx.numel() <= self.B, idx.numel()
        return torch.cat([idx, idx[-1:].expand(self.B - idx.numel())]).contiguous()

    # --- kernels ------------------------------------------------------------------------------
    def _forward(self, idx, counter, period, train=True, logits_out=None):
        o, p = self.ops, self.pv
        if self.fwd12_split:                       # one launch, two workgroups per image (cnn_split.hip)
            o.conv12_fwd(self.data, idx, counter, period, self.cy, self.cx, self.w1f, p["conv1_bias"], self.p1,
                         self.am1, self.w2f, p["conv2_bias"], self.p2, self.am2, self.xraw if train else None, False,
                         self.c12_flags, self.wbar[10 * 32:10 * 32 + 1])
        elif self.conv_split == 2 and not self.fp8:  # channel-split: B * nsplit workgroups per conv
            o.conv1_fwd_split(self.data, idx, counter, period, self.cy, self.cx, self.w1f, p["conv1_bias"], self.p1,
                              self.am1, self.xraw if train else None, self.conv1_split)
            o.conv2_fwd_split(self.p1, self.w2f, p["conv2_bias"], self.p2, self.am2)
        elif self.fused_fwd and not self.fp8:      # conv1 + pool1 + conv2 + pool2 in one launch
            pre = train and self.xraw_prefetch and idx is self.bidx   # the step's own (prefetched) batch
            o.conv12_fwd(self.data, idx, counter, period, self.cy, self.cx, self.w1f, p["conv1_bias"], self.p1,
                         self.am1, self.w2f, p["conv2_bias"], self.p2, self.am2, self.xraw if train else None, pre)
        else:
            o.conv1_fwd(self.data, idx, counter, period, self.cy, self.cx, self.w1f, p["conv1_bias"], self.p1,
                        self.am1, self.amax_x if self.fp8 else None, self.xraw if train else None)
        if self.fp8:
            o.conv2_fwd_fp8(self.p1, self.w2f8[0], p["conv2_bias"], self.amax_x, self.scale_w, counter, self.p2, self.am2,
                            *((self.p1f8, self.sx8) if train and self.fp8_wgrad else (None, None)))
        elif not self.fused_fwd and self.conv_split == 1:
            o.conv2_fwd(self.p1, self.w2f, p["conv2_bias"], self.p2, self.am2)
        if train and self.fc_fused:
            self._fc_src = (idx, counter, period)    # fc forward + head run in _fc_backward's launch
            return
        self._gemm(self._fc1_fwd)
        o.head(self.h1part, p["full_bias_1"], self.fc2t, p["full_bias_2"], self.fc3t, p["full_bias_3"], self.fc3d,
               self.fc2n, self.labels, idx, counter, period, 1.0 / (self.Bv * self.world_size), self.relu_logits,
               train, self.h1, self.h2, self.dl, self.dh1, self.dh2, self.loss_part, self.correct_part, logits_out,
               self.Bv, self.step_t, self.step_sgd)

    def _gemm(self, f, sgd: bool = False):
        if sgd:
            sched = [self.lr0, self.decay, self.decay_steps, 1.0 if self.staircase else 0.0, self.warmup, 1.0]
            self.ops.gemm_grouped(f["A"], f["B"], f["C"], f["bias"], f["params"], self.step_t, self.fc1n, sched)
        else:
            self.ops.gemm_grouped(f["A"], f["B"], f["C"], f["bias"], f["params"], self.step_t)

    def _fc_backward(self, fused_sgd: bool = False):
        if self.fc_fused:
            self._fc_chain(fused_sgd)
            return
        self._gemm(self._fc_bwd_sgd if fused_sgd else self._fc_bwd, sgd=fused_sgd)

    def _fc_chain(self, fused_sgd: bool):
        """fc1 forward + head + fc backward in one persistent launch (cnn_fc.hip), for the batch of
        the preceding _forward(train=True).  fused_sgd: the fc1 weights are updated in the dW1
        epilogue (single GPU), else the fc1 weight gradient goes to the flat gradient."""
        if self._fc_src is None:
            raise RuntimeError("_fc_chain must follow a training _forward")
        if self._dgrad_done:
            raise RuntimeError("the previous fc chain's conv backward never ran")
        idx, counter, period = self._fc_src
        self._fc_src = None
        p, gv = self.pv, self.gv
        sched = [self.lr0, self.decay, self.decay_steps, 1.0 if self.staircase else 0.0, self.warmup, 1.0]
        all_sgd = fused_sgd and self.fc_sgd_in_chain
        if not fused_sgd:
            gv = self.gv_chain                   # (bf16 views on the RCCL bf16 wire)
        g = p if all_sgd else gv                 # every fc SGD here: the master views, else the gradients
        self.ops.fc_chain(self.p2.view(self.B, 2304), self.fc1n, self.h1part8, p["full_bias_1"], self.fc2t,
                          p["full_bias_2"], self.fc3t, p["full_bias_3"], self.fc3d, self.labels, idx, counter, period,
                          1.0 / (self.Bv * self.world_size), self.relu_logits, self.h1, self.h2, self.dl, self.dh1,
                          self.dh2, self.loss_part, self.correct_part, self.dp2.view(self.B, 2304),
                          p["full_weight_1"] if fused_sgd else gv["full_weight_1"], g["full_weight_2"],
                          g["full_weight_3"], g["full_bias_1"], g["full_bias_2"], g["full_bias_3"], fused_sgd,
                          sched, self.Bv, self.step_t, self.step_sgd, self.fc_sync, self.wbar[10 * 32:10 * 32 + 1],
                          not (fused_sgd and self.fc_dw_in_wgrad),
                          *((self.am2, self.w2d, self.dp1, self.dy2) if self.fc_dgrad else (None, None, None, None)),
                          self.fc2n if all_sgd else None)
        self._dgrad_done = self.fc_dgrad

    def _conv_backward(self, src=None, apply: bool = False, reduce: bool = False):
        """apply: + the whole SGD in the wgrad launch (single GPU); reduce: + the conv slab reduction
        into the flat gradient (SGD mode 1) in the wgrad launch."""
        o = self.ops
        idx, counter, period = src or (self.bidx, None, 1)
        assert not apply or (self.wgrad_apply and src is None), "apply mode: the training step only"
        assert not reduce or self._grad_in_launch
        if self._dgrad_done:
            self._dgrad_done = False                 # the fc chain launch did it (fc_dgrad)
        elif self.fp8_dgrad:
            o.conv2_dgrad_fp8(self.dp2, self.am2, self.w2f8[1], self.scale_w, self.dp1, self.dy2,
                              *((self.dy2f8, self.sy_img) if self.fp8_wgrad else (None, None)))
        elif self.dgrad_split == 2:
            o.conv2_dgrad_split(self.dp2, self.am2, self.w2d, self.dp1, self.dy2)
        else:
            o.conv2_dgrad(self.dp2, self.am2, self.w2d, self.dp1, self.dy2)
        if apply or reduce:
            fc_acts = None
            if apply and self.fc_dw_in_wgrad:
                fc_acts = [self.p2.view(self.B, 2304), self.h1, self.h2, self.dl, self.dh1, self.dh2]
            o.wgrad_sgd(self.data, idx, counter, period, self.cy, self.cx, self.dp1, self.am1, self.p1, self.dy2,
                        self.groups2, self.xraw, self.wbar,
                        *(self._sgd_args(mode=0, fc1_fused=True) if apply else self._sgd_args(mode=1)),
                        fc_acts=fc_acts, fc_sgd_done=bool(apply and self.fc_sgd_in_chain), **self._w8)
            return
        o.wgrad(self.data, idx, counter, period, self.cy, self.cx, self.dp1, self.am1,
                self.part1, self.partb1, self.p1, self.dy2, self.part2, self.partb2, self.groups2, self.xraw,
                **self._w8)

    def _sgd_args(self, mode: int, scale: float = 1.0, roles: int = 0, finalize: bool = True,
                  fc1_fused: bool = False) -> tuple:
        gflat = self.grad16 if (self.grad16 is not None and mode in (1, 2)) else self.grad
        return (self.master, gflat, mode, scale, SEG_OFF, self.part1, self.partb1, self.part2, self.partb2,
                self.w1f, self.w2f, self.w2d, self.fc1n, self.fc2t, self.fc2n, self.fc3t, self.fc3d,
                self.step_t, self.lr0, self.decay, self.decay_steps, self.staircase, self.ticket,
                self.loss_part, self.correct_part, self.stats,
                *((self.w2f8, self.amax_w, self.scale_w) if self.fp8 else (None, None, None)),
                roles, finalize, self.Bv, self.bidx, self.order_desc, self.warmup, fc1_fused,
                None if mode == 3 else self.step_sgd,
                *((self.xraw, self.data) if self.xraw_prefetch and mode in (0, 2) and finalize else (None, None)))

    def _sgd(self, mode: int, scale: float = 1.0, roles: int = 0, finalize: bool = True, fc1_fused: bool = False):
        self.ops.sgd(*self._sgd_args(mode, scale, roles, finalize, fc1_fused))

    @property
    def barriers_in_use(self) -> bool:
        """The wgrad launch meets at sub-grid barriers: apply mode (single-GPU SGD) or the in-launch
        conv-slab reduction (data parallel / compute_gradients)."""
        return bool(self.wgrad_apply or self._grad_in_launch or self.fc_fused or self.fwd12_split)

    def queue_error_copy(self):
        """Enqueue a copy of the barrier error word into pinned host memory (stream-ordered: valid once
        an event recorded after this call has completed)."""
        if self.barriers_in_use:
            self._err_host.copy_(self.wbar[10 * 32:10 * 32 + 1], non_blocking=True)

    def check_barriers(self, cached: bool = False):
        """Raise if a sub-grid barrier of the wgrad launch timed out (sticky device error word): apply
        mode would have updated the weights, the reduce mode would have reduced (and all-reduced)
        partial conv gradients -- every replica would agree on them, so the replica check cannot see
        it.  ``cached``: read the pinned copy of :meth:`queue_error_copy` (no device sync)."""
        if not self.barriers_in_use:
            return
        e = int(self._err_host[0]) if cached else int(self.wbar[10 * 32].item())
        if e != 0:
            # error word: value 1 = a wgrad sub-grid barrier, value 2 = an fc chain hand-off timed out
            mode = "apply" if self.wgrad_apply else "reduce"
            parts = []
            if e & 1:
                parts.append(f"k_wgrad ({mode} mode): a sub-grid barrier timed out; rerun with DMLC_WGRAD_SGD=0")
            if e & 2:
                parts.append("k_fc_chain / k_conv12_fwd_split: a hand-off wait timed out; rerun with "
                             "DMLC_FC_FUSED=0 / DMLC_FWD12_SPLIT=0")
            if self.fwd12_split:
                self.c12_flags.zero_()     # a timed-out hand-off can leave a partner's flag raised
            raise RuntimeError("; ".join(parts) + f" (blocks not co-resident, error word {e})")

    def _allreduce(self, t: torch.Tensor):
        import torch.distributed as dist
        if t.dtype == torch.bfloat16:            # grad16: already on the wire's dtype
            dist.all_reduce(t, group=self.pg)
        elif self.comm_dtype == "bf16":
            tb = t.to(torch.bfloat16)
            dist.all_reduce(tb, group=self.pg)
            t.copy_(tb)
        else:
            dist.all_reduce(t, group=self.pg)

    def _allreduce_bucket(self, fc: bool):
        off, n = self._buckets[fc]
        if self.xgmi is not None:
            self.xgmi.all_reduce(off, n)
        elif fc or self.grad16 is not None:
            self._allreduce(self._wire_grad()[off:off + n])
        else:
            # the 0.43 MB conv bucket sits on the step's critical path: fp32 on any wire (latency-bound
            # at this size; the bf16 wire's two cast kernels would cost more than the bytes it saves)
            import torch.distributed as dist
            dist.all_reduce(self.grad[off:off + n], group=self.pg)

    def _wire_grad(self) -> torch.Tensor:
        """The flat gradient the collectives run on (grad16 on the RCCL bf16 wire)."""
        return self.grad16 if self.grad16 is not None else self.grad

    def check_comm(self):
        """Raise if the xGMI all-reduce saw a peer stop participating (sticky device error word) or a
        wgrad sub-grid barrier timed out (device read: callers that must not sync use
        ``check_barriers(cached=True)``)."""
        self.check_barriers()
        if self.xgmi is not None:
            self.xgmi.check()

    def _pg_backend(self) -> str:
        import torch.distributed as dist
        return dist.get_backend(self.pg) if dist.is_available() and dist.is_initialized() else "none"

    def _backend(self) -> str:
        if self.xgmi is not None:
            return "xgmi"
        if not self.dp:
            return "none"
        return self._pg_backend()

    # segments of one step: each is a capturable list of launches on the current stream
    def _seg_compute_a(self):
        self._forward(self.bidx, None, 1, train=True)
        self._fc_backward()

    def _seg_forward(self):
        self._forward(self.bidx, None, 1, train=True)

    def _seg_fc(self):
        self._fc_backward()

    def _seg_compute_b(self):
        if self.wgrad_reduce:                   # conv slabs reduced inside the wgrad launch
            self._conv_backward(reduce=True)
            return
        self._seg_compute_b_launch()

    def _seg_compute_b_launch(self):
        """conv backward + the slab reduction as its own SGD launch.  The overlap schedule always uses
        it: its wgrad launch runs beside the comm stream's collective, and sub-grid barriers there
        could close a cycle across GPUs -- a collective partly resident on each of two GPUs, each
        GPU's missing collective blocks waiting for CUs held by wgrad blocks that spin for their own
        missing blocks, which wait for the CUs of the resident collective blocks, which wait on the
        other GPU.  The bounded spin would turn that into a timeout (a wrong step), so no in-launch
        barrier ever runs beside a collective."""
        self._conv_backward()
        self._sgd(mode=1 if self.dp else 0)

    def _seg_apply(self):
        self._sgd(mode=2, scale=1.0)

    def _seg_apply_fc(self):
        # fc parameters: SGD from the all-reduced fc bucket; runs on the comm stream while the conv
        # backward still runs on the main stream (it touches no conv weights / conv gradients)
        self._sgd(mode=2, scale=1.0, roles=2, finalize=False)

    def _seg_apply_conv(self):
        self._sgd(mode=2, scale=1.0, roles=1, finalize=True)

    def compute_gradients(self, idx: Optional[torch.Tensor] = None, check: bool = True):
        """Forward + backward only (no update); the full gradient lands in ``self.grad``.
        ``idx``: explicit dataset rows (int32 [Bv]) instead of this step's generated batch.
        ``check`` (default True): SYNCHRONISES the device (one read of the error word) and raises if a
        persistent launch's hand-off timed out (the gradient would be partial); loops that call this
        repeatedly should pass False -- the call is then asynchronous -- and call check_barriers() at
        their own sync point."""
        g = self._compute_gradients(idx)
        if check:
            self.check_barriers()
        return g if self.grad16 is None else self.grad16.float()   # (grad16: a converted copy)

    def _compute_gradients(self, idx: Optional[torch.Tensor] = None):
        if idx is None:
            self._seg_compute_a()
            if self._grad_in_launch:
                self._conv_backward(reduce=True)
                return self.grad
            self._conv_backward()
        else:
            ids = self._padded(idx)
            self._forward(ids, None, 1, train=True)
            self._fc_backward()
            if self._grad_in_launch:
                self._conv_backward(src=(ids, None, 1), reduce=True)
                self._sync_xraw()                    # the explicit rows went through xraw
                return self.grad
            self._conv_backward(src=(ids, None, 1))
            self._sync_xraw()
        self._sgd(mode=1)
        return self.grad

    def _reset_step_state(self):
        """Forget a half-issued step (an exception between the fc chain and the conv backward, an
        interrupted capture): the next step starts clean instead of failing the pairing checks."""
        self._fc_src = None
        self._dgrad_done = False
        self._pending_comm = None          # callers synchronise the device first (capture())
        if self.fwd12_split and not torch.cuda.is_current_stream_capturing():
            self.c12_flags.zero_()         # stream-ordered: no half-finished hand-off carries over

    def _eager_step(self):
        try:
            self._eager_step_body()
        except BaseException:
            self._reset_step_state()
            raise
        if not torch.cuda.is_current_stream_capturing():
            self._join_comm()             # an eager step ends joined (captures join at the chain's end)

    def _eager_step_body(self):
        if not self.dp:
            if self.fc1_epilogue:
                self._forward(self.bidx, None, 1, train=True)
                self._fc_backward(fused_sgd=True)
                if self.wgrad_apply:                # the SGD runs inside the wgrad launch
                    self._conv_backward(apply=True)
                    return
                self._conv_backward()
                self._sgd(mode=0, fc1_fused=True)
                return
            self._seg_compute_a()
            self._seg_compute_b()
            return
        if self.dp_schedule == "serial":
            self._serial_dp_step([self._seg_compute_ab, self._seg_apply])
            return
        self._dp_step([self._seg_forward, self._seg_fc, self._seg_compute_b_launch, self._seg_apply_fc,
                       self._seg_apply_conv])

    def _seg_compute_ab(self):
        self._seg_compute_a()
        self._seg_compute_b()

    def _serial_dp_step(self, seg):
        """Single-stream data-parallel step: fwd + bwd + conv-grad reduction | ONE all-reduce of the
        whole flat gradient (4.27 MB fp32; the two buckets are contiguous) | one SGD launch -- or, over
        xGMI (comm_sgd), the exchange kernel that applies the SGD itself."""
        seg[0]()
        n = self.master.numel()
        if self.comm_sgd:           # (xGMI: the whole step is one graph, seg is never a replay list)
            self.xgmi.all_reduce_sgd(self._sgd_args(mode=2), blocks=self._comm_blocks)
            return
        if self.xgmi is not None:
            self.xgmi.all_reduce(0, n)
        else:
            self._allreduce(self._wire_grad()[:n])
        seg[1]()

    def _dp_step(self, seg):
        """Data-parallel step around two all-reduce buckets, two streams:
            main: fwd | [join s-1] fc chain | wgrad, slab-reduction launch |     [wait] conv SGD (+ finalize)
            comm:                  [wait] all-reduce fc | [wait] all-reduce conv -> fc SGD
        Both collectives go through ONE stream in one order (one communicator, the same issue order on
        every rank).  The fc bucket (90 % of the bytes) crosses the links while the wgrad launch runs;
        only the 0.43 MB conv bucket and the conv SGD stay on the step's critical path.  The fc SGD
        (fc weights + shadows) is NOT joined at the end of the step: the next step's forward does not
        read an fc parameter, so the join sits before the next fc chain (the fc SGD runs beside the
        next conv12 forward) -- :meth:`_join_comm` closes a sequence (end of a captured chain, an eager
        step, before a graph replay).
        seg: [forward, fc chain, conv backward, fc apply, conv apply] (eager launchers or, with eager
        collectives, replays of the segment graphs)."""
        main = torch.cuda.current_stream(self.device)
        seg[0]()
        self._join_comm()                       # step s-1's fc SGD wrote the shadows the chain reads
        seg[1]()
        ev_fc = torch.cuda.Event()
        ev_fc.record(main)
        self.comm_stream.wait_event(ev_fc)
        with torch.cuda.stream(self.comm_stream):
            self._allreduce_bucket(fc=True)
        seg[2]()
        ev_wg = torch.cuda.Event()
        ev_wg.record(main)
        self.comm_stream.wait_event(ev_wg)
        ev_conv, ev_done = torch.cuda.Event(), torch.cuda.Event()
        with torch.cuda.stream(self.comm_stream):
            self._allreduce_bucket(fc=False)
            ev_conv.record(self.comm_stream)
            seg[3]()
            ev_done.record(self.comm_stream)
        main.wait_event(ev_conv)
        seg[4]()
        self._pending_comm = ev_done

    def _join_comm(self):
        """The current stream waits for the last step's comm-stream work (the fc SGD)."""
        ev = getattr(self, "_pending_comm", None)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
            self._pending_comm = None

    # --- graph capture --------------------------------------------------------------------------
    @property
    def single_graph(self) -> bool:
        """The whole step (collectives included) is one capturable launch sequence."""
        return not self.dp or self.capture_comm or self.xgmi is not None

    def capture(self, steps_per_graph: int = 8):
        """Capture the step into HIP graph(s).  N=1, N>1 over xGMI and N>1 over RCCL with
        ``capture_comm`` (the default): the whole step -- compute, all-reduce, SGD, on one or two
        streams -- is one graph, and further graphs chain 2, 4, ... ``steps_per_graph`` complete
        steps (every step reads its batch and LR through the device step counter, so consecutive
        steps need no host work, across epoch boundaries too).  :meth:`run` replays any step count
        as a sum of chains -- no single-step tails, no host gap between the chained steps.
        RCCL without ``capture_comm``: compute graphs around eager collectives (no chains)."""
        quiesce_for_capture(self.device, self.pg if self.dp else None)
        self._reset_step_state()
        self.graphs, self.chains = [], {}
        pool = torch.cuda.graph_pool_handle()
        if self.single_graph:
            segs = [lambda: self._steps_joined(1)]
        elif self.dp_schedule == "serial":
            segs = [self._seg_compute_ab, self._seg_apply]
        else:
            segs = [self._seg_forward, self._seg_fc, self._seg_compute_b_launch, self._seg_apply_fc,
                    self._seg_apply_conv]
        self._captured_schedule = self.dp_schedule
        # a capture records launches without running them: the step counter and weights are
        # identical before and after
        for fn in segs:
            self.graphs.append(self._capture_one(fn, pool))
        if self.single_graph:
            k = 2
            while k <= int(steps_per_graph):
                self.chains[k] = self._capture_one(lambda k=k: self._steps_joined(k), pool)
                k *= 2
        self.chains[1] = self.graphs[0] if self.single_graph else None
        self._pool = pool
        torch.cuda.synchronize(self.device)

    def add_chain(self, k: int) -> bool:
        """Also capture a chain of exactly ``k`` steps, so :meth:`run` (k) is ONE graph replay (a
        short timed region otherwise pays one graph-launch boundary per power-of-two piece)."""
        k = int(k)
        if not self.single_graph or not self.graphs or k < 2 or self.chains.get(k) is not None:
            return False
        quiesce_for_capture(self.device, self.pg if self.dp else None)
        self.chains[k] = self._capture_one(lambda: self._steps_joined(k), self._pool)
        torch.cuda.synchronize(self.device)
        return True

    def _steps_joined(self, k: int):
        """``k`` steps, then the comm stream joined (a captured graph must end on its origin stream;
        inside it, step s's fc SGD overlaps step s+1's forward)."""
        for _ in range(k):
            self._eager_step()
        self._join_comm()

    def _capture_one(self, fn, pool):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            # thread_local: the capture forbids unsafe calls on THIS thread only -- the process group's
            # watchdog thread polls the events of earlier (eager) collectives, and under the default
            # global mode one such poll invalidates the capture (seen on a 1-rank nccl group)
            with torch.cuda.graph(g, pool=pool, stream=s, capture_error_mode="thread_local"):
                fn()
        torch.cuda.current_stream(self.device).wait_stream(s)
        return g

    @property
    def multi(self):
        """(k, graph) of the longest captured chain, or None."""
        ks = [k for k, g in getattr(self, "chains", {}).items() if g is not None and k > 1]
        return (max(ks), self.chains[max(ks)]) if ks else None

    def run(self, n: int):
        """``n`` complete training steps (asynchronous): the longest captured chains first, then the
        binary decomposition of the remainder (e.g. 21 = 8 + 8 + 4 + 1 replays)."""
        n = int(n)
        chains = {k: g for k, g in getattr(self, "chains", {}).items() if g is not None}
        if not self.graphs or not chains:
            for _ in range(n):
                self.step()
            return
        self._join_comm()
        for k in sorted(chains, reverse=True):
            while n >= k:
                chains[k].replay()
                self.host_step += k
                n -= k

    def step(self):
        """One training step (asynchronous: returns once launched)."""
        if not self.graphs:
            self._eager_step()
        elif len(self.graphs) == 1:
            self._join_comm()
            self.graphs[0].replay()
        elif self._captured_schedule == "serial":
            self._serial_dp_step([g.replay for g in self.graphs])
        else:
            self._dp_step([g.replay for g in self.graphs])
            self._join_comm()
        self.host_step += 1

    def tune_schedule(self, iters: int = 30, steps_per_graph: int = 8, rounds: int = 2, log=None) -> str:
        """Data-parallel step: capture each schedule (overlap / serial), time ``iters`` real
        training steps of each (max over ranks, so every rank takes the same decision) over
        ``rounds`` alternating rounds (overlap, serial, serial, overlap, ...), keep the minimum per
        schedule and the faster schedule captured.  Both windows replay the same chain
        decomposition and cross no host work (the data order is generated in-kernel), so neither
        pays for anything the other does not.  The timed steps are ordinary training steps."""
        if not self.dp:
            return self.dp_schedule
        import time
        import torch.distributed as dist
        nccl = self._backend() == "nccl" or (self.xgmi is not None and dist.get_backend(self.pg) == "nccl")
        bdev = self.device if nccl else torch.device("cpu")
        times = {"overlap": [], "serial": []}
        order = []
        for r in range(max(1, rounds)):
            order += ["overlap", "serial"] if r % 2 == 0 else ["serial", "overlap"]
        for sched in order:
            self.dp_schedule = sched
            self.capture(steps_per_graph)
            self.run(steps_per_graph)
            torch.cuda.synchronize(self.device)
            dist.barrier(group=self.pg)
            t0 = time.perf_counter()
            self.run(iters)
            torch.cuda.synchronize(self.device)
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=bdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.pg)
            # a persistent launch's bounded wait timed out on some rank: that schedule is out (the
            # sticky word is cleared for the run that follows; every rank sees the same MAX)
            e = torch.tensor([int(self.wbar[10 * 32].item()) if self.barriers_in_use else 0],
                             dtype=torch.float64, device=bdev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX, group=self.pg)
            if self.xgmi is not None:
                self.xgmi.check()      # a timed-out exchange leaves no consistent epoch to resume from
            if float(e.item()) != 0.0:
                if log:
                    log(f"dp schedule {sched}: a persistent launch's wait timed out -- not eligible")
                self.wbar[10 * 32].zero_()
                times[sched].append(math.inf)
                continue
            times[sched].append(float(t.item()) / iters)
        best_t = {k: min(v) for k, v in times.items()}
        best = min(best_t, key=best_t.get)
        self.comm_info.update(schedule=best, schedule_us={k: round(v * 1e6, 1) for k, v in best_t.items()
                                                          if v != math.inf})
        if log:
            log(f"dp schedule: {best} ({self.comm_info['schedule_us']})")
        if best != self.dp_schedule:
            self.dp_schedule = best
            self.capture(steps_per_graph)
        return best

    # --- evaluation -----------------------------------------------------------------------------
    @torch.no_grad()
    def evaluate(self, data: torch.Tensor, labels: torch.Tensor, max_batches: int = 0) -> float:
        """Test accuracy over ``data`` (uint8 [N,32,32,3]) with the fused forward kernels."""
        data = data.to(self.device).contiguous()
        labels = labels.to(self.device, torch.int32).contiguous()
        saved = (self.data, self.labels)
        self.data, self.labels = data, labels
        if self.fp8:    # eval launches carry no step counter: they read scale slot 0 (see cnn_fp8.hip)
            self.scale_w[0] = self.scale_w[self.host_step & 1]
        n = data.shape[0]
        nb = math.ceil(n / self.Bv)
        if max_batches:
            nb = min(nb, max_batches)
        correct, total = 0, 0
        try:
            for i in range(nb):
                ids = torch.arange(i * self.Bv, i * self.Bv + self.B, device=self.device, dtype=torch.int32)
                valid = int(min(self.Bv, n - i * self.Bv))
                ids = torch.clamp(ids, max=n - 1)
                self._forward(ids, None, 1, train=False, logits_out=self.logits_buf)
                pred = self.logits_buf[:valid].argmax(dim=1)
                correct += int((pred == labels[i * self.Bv:i * self.Bv + valid].long()).sum())
                total += valid
        finally:
            self.data, self.labels = saved
        return correct / max(1, total)

    @torch.no_grad()
    def forward_logits(self, idx: torch.Tensor) -> torch.Tensor:
        """Logits (fp32 [n,10]) of dataset rows ``idx`` (int32 [n], n <= B) — for tests."""
        if self.fp8:
            self.scale_w[0] = self.scale_w[self.host_step & 1]
        n = idx.numel()
        self._forward(self._padded(idx), None, 1, train=False, logits_out=self.logits_buf)
        return self.logits_buf[:n].clone()

    # --- state ----------------------------------------------------------------------------------
    def read_stats(self, step: int) -> Dict[str, float]:
        """Stats published by the SGD kernel for the step that produced global_step == ``step``."""
        row = self.stats[(step - 1) % self.stats.shape[0]].tolist()
        return {"global_step": int(row[0]), "loss": row[1], "accuracy": row[2], "lr": row[3]}

    def global_step(self) -> int:
        return int(self.step_t.item())

    def fc1n_current(self) -> torch.Tensor:
        """The bf16 fc1 weight shadow the kernels of the current step read ([2304][384])."""
        return self.fc1n[self.global_step() & 1]

    def flat_params(self) -> torch.Tensor:
        return self.master.detach().cpu()

    def load_flat_params(self, flat: torch.Tensor, step: Optional[int] = None):
        self.master.copy_(flat.to(self.device, torch.float32))
        if step is not None:
            self.set_step(step)
        self.refresh_shadows()
