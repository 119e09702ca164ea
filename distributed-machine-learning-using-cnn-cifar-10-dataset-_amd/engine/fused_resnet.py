"""Fused MI355X training engine for ResNet-20 (BASELINE.json config 4; model: models/resnet.py).

Not in the reference (/root/reference/cifar10cnn.py only has the 2-conv CNN); SURVEY.md §2.C lists
ResNet-20 as the "extra kernels" configuration: conv3x3 stride 1/2, train-mode BatchNorm, residual
add, global average pool.  One step is 19 forward convs + 1 head + 18 dgrads + 19 wgrads + 1 SGD,
all HIP kernels of csrc/kernels/resnet.hip, captured as one HIP graph:

  fwd  l=0..18   z_l = conv_l(a_{l-1}); the prologue of conv_l applies BN_{l-1} (+ReLU, + option-A
                 shortcut) from the fp64 batch statistics conv_{l-1}'s epilogue accumulated, and
                 materialises a_{l-1} for the backward.  Conv_0 gathers the uint8 batch itself.
  head           BN_18 + residual + ReLU + global average pool + fc + softmax-xent + its backward
  bwd  l=18..1   dgrad_l: g_z_l (BN backward, prologue) -> g_a_{l-1} (+ shortcut grad) -> ReLU mask
                 -> g_y_{l-1} and the BN_{l-1} reductions (epilogue)
       l=18..0   wgrad_l, split-K fp32 slabs: in the same launch as dgrad_l (block roles), or on a
                 side stream (a second graph branch, wgrad_branch=True)
  sgd            slab reduction + SGD (conv, BN gamma/beta, fc) + BN running statistics (momentum 0.1)
                 + bf16 weight shadows + global_step++ + stats ring

Batch statistics are per rank (as in the eager model under DP).  With data parallelism the SGD runs
in two halves around ONE all-reduce of the 1.1 MB flat gradient (mode 1 -> RCCL -> mode 2).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch

from .. import config as C
from ..parallel.dist import quiesce_for_capture
from ..data.order import OrderSpec
from ..models import resnet as R
from ..ops import _ext
from .fused import TICKET_WORDS

OPS = None


def _ops():
    global OPS
    if OPS is None:
        _ext.hip()
        OPS = torch.ops.dmlc
    return OPS


def layer_table():
    """[(name prefix, cin, cout, hin, stride, shortcut mode used when this layer's output is applied)]
    in execution order (l = 0..18)."""
    layers = [("stem", 3, 16, 32, 1)]
    cin, hin = 16, 32
    for s, w in enumerate(R.WIDTHS):
        for b in range(R.BLOCKS):
            stride = 2 if (s > 0 and b == 0) else 1
            layers.append((f"stage{s}/block{b}/a", cin, w, hin, stride))
            hin //= stride
            layers.append((f"stage{s}/block{b}/b", w, w, hin, 1))
            cin = w
    return layers


NSLOT = 8            # BN statistics slots per layer (resnet.hip)
LAYERS = layer_table()
NL = len(LAYERS)
assert NL == 19


def _kp(cin):
    return (9 * max(cin, 8) + 31) // 32 * 32


def _kpd(cout):
    return (9 * cout + 31) // 32 * 32


FX_ONE = float(2 ** 48)   # fraction unit of the fixed-point BN statistics (resnet.hip fx_add)


def fx_encode(x: torch.Tensor):
    """Host mirror of resnet.hip fx_add for finite |x| < 2^50: (integer part, 48-bit fraction)."""
    x = x.double()
    f = torch.floor(x)
    return f.long(), torch.round((x - f) * FX_ONE).long()


def fx_decode(slots: torch.Tensor) -> torch.Tensor:
    """Totals of fixed-point statistic slots [..., NSLOT, 256] int64 -> fp64 [..., 128] (resnet.hip
    fx_total; a slot at or beyond the poison bound 2^55 decodes to NaN)."""
    hi, lo = slots[..., :128], slots[..., 128:]
    bad = (hi.abs() >= 2 ** 55).any(-2)
    tot = hi.sum(-2).double() + lo.sum(-2).double() / FX_ONE
    return torch.where(bad, torch.full_like(tot, float("nan")), tot)


def _block_sc_mode(b_layer: int) -> int:
    """Shortcut mode of the block whose second conv is ``b_layer`` (1 identity, 2 subsample+pad)."""
    a_layer = b_layer - 1
    return 2 if LAYERS[a_layer][4] == 2 else 1


class FusedResNetEngine:
    """Owns every device buffer of the fused ResNet-20 step.  Parameters: one flat fp32 buffer in the
    TF layout of models/resnet.py (HWIO kernels), BN moving statistics in a second flat buffer."""

    def __init__(self, batch_size: int, data: torch.Tensor, labels: torch.Tensor, *, device=None,
                 flat_params: Optional[torch.Tensor] = None, state: Optional[torch.Tensor] = None,
                 lr: float = C.LEARNING_RATE, lr_decay: float = C.LR_DECAY,
                 decay_steps: float = C.NUM_GENS_TO_WAIT, staircase: bool = True, world_size: int = 1,
                 rank: int = 0, process_group=None, seed: int = 0, groups: Optional[List[int]] = None,
                 stats_len: int = 4096, comm_dtype: str = "fp32", wgrad_branch: Optional[bool] = None,
                 allreduce: str = "auto", capture_comm: Optional[bool] = None, dp_force: bool = False,
                 warmup_steps: int = 0,
                 merged_bwd: Optional[bool] = None, bwd_img_level: int = 1, sgd_split: bool = False):
        ops = _ops()
        self.ops = ops
        self.device = torch.device(device or "cuda")
        dev = self.device
        Bv = int(batch_size)
        if Bv < 1:
            raise ValueError("batch size must be >= 1")
        # any batch size: the kernels run on the batch padded to the 16-image tile; the padding images
        # are excluded from every BatchNorm statistic and get zero loss weight / gradient (nvalid)
        B = -(-Bv // 16) * 16
        self.B, self.Bv = B, Bv
        self.world_size, self.rank, self.pg = world_size, rank, process_group
        self.lr0, self.decay, self.decay_steps, self.staircase = lr, lr_decay, decay_steps, staircase
        self.warmup = float(warmup_steps)      # linear LR warm-up, in the SGD kernel
        self.seed, self.comm_dtype = seed, comm_dtype
        self.dp = world_size > 1 or dp_force     # dp_force: the all-reduce path at world_size 1 (tests)
        if capture_comm is None:                 # RCCL collectives inside the step graph (nccl only)
            import torch.distributed as dist
            nccl = dist.is_initialized() and dist.get_backend(process_group) == "nccl"
            capture_comm = self.dp and nccl
        self.capture_comm = bool(capture_comm)

        assert data.dtype == torch.uint8 and tuple(data.shape[1:]) == (32, 32, 3)
        self.data = data.to(dev).contiguous()
        self.labels = labels.to(dev, torch.int32).contiguous()
        self.n_data = self.data.shape[0]
        self.order = OrderSpec(self.n_data, Bv, world_size, rank, seed)   # generated order (data/order.py)
        self.period = self.order.period
        self.order_desc = self.order.descriptor()

        f0, s0 = R.init_flat_params(torch.Generator().manual_seed(seed))
        if flat_params is not None:
            f0 = flat_params
        if state is not None:
            s0 = state
        self.master = f0.to(dev, torch.float32).contiguous().clone()
        self.state = s0.to(dev, torch.float32).contiguous().clone()
        # gradient all-reduce (N>1): xGMI peer-to-peer kernel over an IPC-shared buffer when it
        # self-tests and measures faster than RCCL (parallel/xgmi.py), else RCCL
        self.xgmi, self.comm_info = None, {"allreduce": "rccl" if self.dp else "none"}
        if world_size > 1 and dev.type == "cuda" and comm_dtype in ("fp32", "bf16") and allreduce != "rccl":
            from ..parallel import xgmi as X
            self.xgmi, self.comm_info = X.select(self.master.numel(), rank, world_size, dev,
                                                 [(0, self.master.numel())], mode=allreduce, group=process_group,
                                                 wire=comm_dtype, captured=self.capture_comm)
        if self.xgmi is not None:
            self.grad = self.xgmi.buf[:self.master.numel()]
            self.grad.zero_()
        else:
            self.grad = torch.zeros_like(self.master) if self.dp else None
        P = {s.name[len(R.SCOPE) + 1:]: s for s in R.PARAM_SPECS}
        S = {s.name[len(R.SCOPE) + 1:]: s for s in R.STATE_SPECS}
        view = lambda buf, s: buf[s.offset:s.offset + s.numel]
        self.conv_off = [P[f"{n}/conv/kernel"].offset for n, *_ in LAYERS]
        self.gamma_off = [P[f"{n}/bn/gamma"].offset for n, *_ in LAYERS]
        self.beta_off = [P[f"{n}/bn/beta"].offset for n, *_ in LAYERS]
        self.mm_off = [S[f"{n}/bn/moving_mean"].offset for n, *_ in LAYERS]
        self.mv_off = [S[f"{n}/bn/moving_variance"].offset for n, *_ in LAYERS]
        self.gamma = [view(self.master, P[f"{n}/bn/gamma"]) for n, *_ in LAYERS]
        self.beta = [view(self.master, P[f"{n}/bn/beta"]) for n, *_ in LAYERS]
        self.fcw_off, self.fcb_off = P["fc/weights"].offset, P["fc/biases"].offset
        self.fcw, self.fcb = view(self.master, P["fc/weights"]), view(self.master, P["fc/biases"])

        bf = torch.bfloat16
        z = lambda *s, dt=bf: torch.zeros(*s, dtype=dt, device=dev)
        self.wf = [z(co, _kp(ci)) for _, ci, co, _, _ in LAYERS]
        self.wd = [z(co, _kp(ci)) if l == 0 else z(ci, _kpd(co)) for l, (_, ci, co, _, _) in enumerate(LAYERS)]
        hout = [h // s for _, _, _, h, s in LAYERS]
        self.z = [z(B, ho, ho, co) for ho, (_, _, co, _, _) in zip(hout, LAYERS)]
        self.gy = [z(B, ho, ho, co) for ho, (_, _, co, _, _) in zip(hout, LAYERS)]
        self.a = [z(B, ho, ho, co) for ho, (_, _, co, _, _) in zip(hout[:-1], LAYERS[:-1])]   # a_0 .. a_17
        # [stat | red] BatchNorm sums, NSLOT fixed-point copies per layer (resnet.hip fx_add): per statistic
        # an int64 integer part [0, 128) and a 48-bit fraction [128, 256), added with 64-bit integer
        # atomics -- order independent, so every step is bitwise reproducible (graph replay == eager);
        # zeroed at the start of each forward
        self.acc = torch.zeros(2, NL, NSLOT, 256, dtype=torch.int64, device=dev)
        self.stat, self.red = self.acc[0], self.acc[1]
        # per-image backward (k_rn_bwd_img, merged backward only): bwd_img_level 0 off, 1 the 16->16
        # layers (their wgrad keeps one slab per image anyway), 2 also the 32->32 stride-1 layers (one
        # slab per image instead of B/2 groups: more slab bytes for the SGD, fewer re-reads)
        self.bwd_img_level = int(bwd_img_level)
        self.groups = groups or [B if (self.bwd_img_level >= 2 and B <= 256 and (ci, co, h, s) == (32, 32, 16, 1))
                                 else self._pick_groups(B, ci, co) for _, ci, co, h, s in LAYERS]
        self.part = [z(g, _kp(ci), co, dt=torch.float32) for g, (_, ci, co, _, _) in zip(self.groups, LAYERS)]
        self.fc_part = z(B, 656, dt=torch.float32)
        self.loss_img = z(B, dt=torch.float32)
        self.correct_img = z(B, dt=torch.int32)
        self.logits_buf = z(B, 10, dt=torch.float32)
        self.step_t = torch.zeros(1, dtype=torch.int64, device=dev)
        # The SGD finds the last arriver with a ticket (the CNN engine's ticketless form -- the head
        # copies the step counter for the SGD -- measured no better here in r3: 0.679 / 0.682 ms vs
        # 0.675 / 0.678 with the ticket); step_sgd is the kernel argument that form would use
        self.step_sgd = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ticket = torch.zeros(TICKET_WORDS, dtype=torch.int32, device=dev)   # two-level arrival counters
        self.stats = torch.zeros(stats_len, 4, dtype=torch.float32, device=dev)

        self.graphs: List[torch.cuda.CUDAGraph] = []
        self.chains: Dict[int, torch.cuda.CUDAGraph] = {}
        if self.dp:
            self.comm_info.update(captured_comm=bool(self.capture_comm or self.xgmi is not None))
        self.side_stream = torch.cuda.Stream(device=dev)
        # Backward schedule, measured per batch size (graph replay, img/s on 1 MI355X):
        #                          B=256   B=1024
        #   merged dgrad+wgrad     376 k   508 k   one launch per layer, no fork/join edges
        #   two launches, 1 stream 363 k   590 k
        #   wgrads on a branch     336 k   620 k   19 fork/join edges in the graph
        # The merged kernel runs at the occupancy of the larger (wgrad) body, which costs more than the
        # saved launches once each layer has >= ~4 dgrad workgroups per CU; wgrad_branch / merged_bwd
        # override the choice.
        self.wgrad_branch = (B > 256) if wgrad_branch is None else bool(wgrad_branch)
        self.merged_bwd = (B <= 256) if merged_bwd is None else bool(merged_bwd)
        # sgd_split=True (single GPU, merged backward): the SGD of stage 3 (layers 13-18) and of
        # stage 2 (7-12) runs on a graph branch as soon as their weight gradients are complete, beside
        # the stage-2 / stage-1 backward; the main-stream SGD does the rest and publishes the step.
        # Measured at B=256: 341 k vs 371 k img/s with one SGD launch -- the co-resident SGD blocks
        # slow the one-image-per-workgroup backward more than the hidden slab reads save: off.
        self.sgd_split = bool(sgd_split) and not self.dp and self.merged_bwd and not self.wgrad_branch
        self._sgd_points = {13: (13, NL), 7: (7, 13)}    # after bwd launch of layer l: SGD of [lo, hi)
        self.host_step = 0
        self._stem_src = None          # explicit (idx, counter, period) of the stem wgrad, else generated
        self.refresh_shadows()

    # ------------------------------------------------------------------------------------------
    @staticmethod
    def _pick_groups(B: int, cin: int, cout: int) -> int:
        """Split-K image groups of one wgrad (grid = groups x m-chunks): enough blocks to fill the chip
        (256) while the fp32 slabs the SGD kernel reads back stay under 16 MB per layer (64 groups for
        the 64-channel layers, 677 -> 667 us/step at B=256, profiles/r1_v17_rn_slab_cap_ab.txt).  A
        power of two in [8, B]."""
        blocks = 256
        cap = 16.0 * 2 ** 20
        mt = _kp(cin) // 16
        mc = 1 if mt <= 12 else (2 if mt <= 24 else 3)      # Wg<>::MC in resnet.hip
        lim = min(blocks / mc, cap / (_kp(cin) * cout * 4))
        g = 1 << max(0, int(math.floor(math.log2(max(1.0, lim)))))
        return int(max(1, min(B, max(8, g))))

    def refresh_shadows(self):
        self._sgd(mode=3)

    def set_step(self, step: int):
        self.step_t.fill_(int(step))
        self.step_sgd.fill_(int(step))
        self.host_step = int(step)

    def epoch_permutation(self, epoch: int) -> torch.Tensor:
        """This rank's rows of ``epoch`` (int32 [period * B]), the order the kernels generate."""
        return self.order.epoch_shard(epoch).to(torch.int32)

    def bn_sums(self) -> torch.Tensor:
        """Decoded BatchNorm sums of the last step, fp64 [2, NL, 128]: [0] sum z / sum z^2, [1] R1 / R2
        (channels at [0, cout) and [64, 64 + cout))."""
        return fx_decode(self.acc)

    def batch_indices(self, step: int) -> torch.Tensor:
        return self.order.batch(step).to(torch.int32)

    # --- kernels ------------------------------------------------------------------------------
    def _forward(self, idx, counter, period, logits_out=None):
        o = self.ops
        self.acc.zero_()
        for l, (_, ci, co, h, s) in enumerate(LAYERS):
            if l == 0:
                o.rn_fwd(ci, co, h, s, self.data, idx, counter, period, 0, 0, None, None, None, None, None, 0, None,
                         self.wf[0], self.z[0], self.stat[0], self.Bv)
                continue
            p = l - 1
            sc_mode, sc_src = 0, None
            if p >= 2 and p % 2 == 0:                  # layer p closes a residual block
                sc_mode = _block_sc_mode(p)
                sc_src = self.a[p - 2]
            o.rn_fwd(ci, co, h, s, None, None, None, 1, 0, 0, self.z[p], self.stat[p], self.gamma[p], self.beta[p],
                     sc_src, sc_mode, self.a[p], self.wf[l], self.z[l], self.stat[l], self.Bv)
        o.rn_head(self.z[18], self.stat[18], self.gamma[18], self.beta[18], self.a[16], self.fcw, self.fcb,
                  self.labels, idx, counter, period, 1.0 / (self.Bv * self.world_size), self.gy[18], self.red[18],
                  self.fc_part, self.loss_img, self.correct_img, logits_out, self.Bv,
                  self.step_t, self.step_sgd)

    def _per_image(self, l) -> bool:
        """Layer l's dgrad and wgrad from one workgroup per image (k_rn_bwd_img): the 16->16 stride-1
        layers whose weight gradient already keeps one split-K slab per image (G == B, B <= 256).
        bwd_img_level=0: the merged launch with separate wgrad blocks."""
        _, ci, co, h, s = LAYERS[l]
        lvl = {(16, 16, 32, 1): 1, (32, 32, 16, 1): 2}.get((ci, co, h, s))
        return bool(lvl and self.bwd_img_level >= lvl and self.part[l].shape[0] == self.B)

    def _wgrad(self, l):
        _, ci, co, h, s = LAYERS[l]
        if l == 0:
            idx, counter, period = self._stem_src or (self.order_desc, self.step_t, self.period)
            self.ops.rn_wgrad(ci, co, h, s, self.data, idx, counter, period, 0, 0, None, self.gy[0],
                              self.z[0], self.stat[0], self.red[0], self.gamma[0], self.part[0], self.Bv)
        else:
            self.ops.rn_wgrad(ci, co, h, s, None, None, None, 1, 0, 0, self.a[l - 1], self.gy[l], self.z[l],
                              self.stat[l], self.red[l], self.gamma[l], self.part[l], self.Bv)

    def _backward(self):
        o = self.ops
        main = torch.cuda.current_stream(self.device)
        side = self.side_stream if self.wgrad_branch else main
        if side is main and self.merged_bwd:
            # one launch per layer: dgrad_l and wgrad_l both only read what dgrad_{l+1} produced
            for l in range(NL - 1, 0, -1):
                _, ci, co, h, s = LAYERS[l]
                sc_mode, gy_sc = 0, None
                if l % 2 == 1:
                    sc_mode = _block_sc_mode(l + 1)
                    gy_sc = self.gy[l + 1]
                o.rn_bwd(ci, co, h, s, self.gy[l], self.z[l], self.stat[l], self.red[l], self.gamma[l], self.wd[l],
                         self.a[l - 1], self.z[l - 1], self.stat[l - 1], gy_sc, sc_mode, self.gy[l - 1],
                         self.red[l - 1], self.part[l], self.Bv, self._per_image(l))
                if self.sgd_split and l in self._sgd_points:
                    # layers >= l: slabs complete, weights no longer read this step
                    self.side_stream.wait_stream(main)
                    with torch.cuda.stream(self.side_stream):
                        self._sgd(mode=0, layers=self._sgd_points[l], tail=False)
            self._wgrad(0)
            return
        for l in range(NL - 1, -1, -1):
            # gy_l and red_l are complete here (head or dgrad_{l+1}): fork wgrad_l onto the side branch
            if side is not main:
                ev = torch.cuda.Event()
                ev.record(main)
                side.wait_event(ev)
            with torch.cuda.stream(side):
                self._wgrad(l)
            if l == 0:
                break
            _, ci, co, h, s = LAYERS[l]
            p = l - 1
            sc_mode, gy_sc = 0, None
            if l % 2 == 1:                             # a-conv: its input also feeds the block shortcut
                sc_mode = _block_sc_mode(l + 1)
                gy_sc = self.gy[l + 1]
            o.rn_dgrad(ci, co, h, s, self.gy[l], self.z[l], self.stat[l], self.red[l], self.gamma[l], self.wd[l],
                       self.a[p], self.z[p], self.stat[p], gy_sc, sc_mode, self.gy[p], self.red[p],
                       self.Bv)
        if side is not main:
            main.wait_stream(side)

    def _sgd(self, mode: int, scale: float = 1.0, layers=(0, NL), tail: bool = True):
        self.ops.rn_sgd(self.master, self.grad, scale, self.state, self.conv_off, self.gamma_off, self.beta_off,
                        self.mm_off, self.mv_off, self.fcw_off, self.fcb_off, self.part, self.wf, self.wd, self.stat,
                        self.red, self.fc_part, self.loss_img, self.correct_img, self.step_t, self.ticket, self.stats,
                        mode, self.lr0, self.decay, self.decay_steps, self.staircase, R.BN_MOMENTUM, self.warmup,
                        layers[0], layers[1], tail, self.Bv,
                        None)

    def _allreduce(self, t: torch.Tensor):
        import torch.distributed as dist
        if self.xgmi is not None:
            self.xgmi.all_reduce(0, t.numel())
            return
        if self.comm_dtype == "bf16":
            tb = t.to(torch.bfloat16)
            dist.all_reduce(tb, group=self.pg)
            t.copy_(tb)
        else:
            dist.all_reduce(t, group=self.pg)

    def check_comm(self):
        """Raise if the xGMI all-reduce saw a peer stop participating (sticky device error word)."""
        if self.xgmi is not None:
            self.xgmi.check()

    def _seg_compute(self):
        self._forward(self.order_desc, self.step_t, self.period)
        self._backward()
        if self.sgd_split:
            # the branch SGDs read the step counter the tail increments: join first
            torch.cuda.current_stream(self.device).wait_stream(self.side_stream)
            self._sgd(mode=0, layers=(0, min(lo for lo, _ in self._sgd_points.values())))
        else:
            self._sgd(mode=1 if self.dp else 0)

    def _seg_apply(self):
        self._sgd(mode=2, scale=1.0)

    def _eager_step(self):
        self._seg_compute()
        if self.dp:
            self._allreduce(self.grad)
            self._seg_apply()

    def compute_gradients(self, idx: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Forward + backward + slab reduction only (no update); the flat gradient lands in ``grad``.
        ``idx``: explicit dataset rows (int32 [B]) instead of this step's generated batch."""
        if self.grad is None:
            self.grad = torch.zeros_like(self.master)
        if idx is not None:
            ids = self._padded(idx)
            self._stem_src = (ids, None, 1)
            try:
                self._forward(ids, None, 1)
                self._backward()
                self._sgd(mode=1)
            finally:
                self._stem_src = None
            return self.grad
        self._forward(self.order_desc, self.step_t, self.period)
        self._backward()
        self._sgd(mode=1)
        return self.grad

    # --- graph capture --------------------------------------------------------------------------
    @property
    def single_graph(self) -> bool:
        return not self.dp or self.capture_comm or self.xgmi is not None

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

    def capture(self, steps_per_graph: int = 8):
        """The whole step as one graph (N=1, xGMI, or RCCL with ``capture_comm``) plus chains of
        2, 4, ... ``steps_per_graph`` steps for :meth:`run`; RCCL without ``capture_comm``: compute
        and apply graphs around an eager all-reduce."""
        quiesce_for_capture(self.device, self.pg if self.dp else None)
        self.graphs, self.chains = [], {}
        pool = torch.cuda.graph_pool_handle()
        segs = [self._eager_step] if self.single_graph else [self._seg_compute, self._seg_apply]
        for fn in segs:
            self.graphs.append(self._capture_one(fn, pool))
        if self.single_graph:
            self.chains[1] = self.graphs[0]
            k = 2
            while k <= int(steps_per_graph):
                self.chains[k] = self._capture_one(lambda k=k: [self._eager_step() for _ in range(k)], pool)
                k *= 2
        torch.cuda.synchronize(self.device)

    def run(self, n: int):
        """``n`` training steps: longest chains first, then the binary decomposition of the rest."""
        n = int(n)
        if not self.chains:
            for _ in range(n):
                self.step()
            return
        for k in sorted(self.chains, reverse=True):
            while n >= k:
                self.chains[k].replay()
                self.host_step += k
                n -= k

    def step(self):
        if not self.graphs:
            self._eager_step()
        elif len(self.graphs) == 1:
            self.graphs[0].replay()
        else:
            self.graphs[0].replay()
            self._allreduce(self.grad)
            self.graphs[1].replay()
        self.host_step += 1

    # --- evaluation -----------------------------------------------------------------------------
    def eval_model(self):
        m = R.ResNet20(flat=self.master.detach()).to(self.device)
        m.state.copy_(self.state)
        m.eval()
        return m

    @torch.no_grad()
    def evaluate(self, data: torch.Tensor, labels: torch.Tensor, max_batches: int = 0) -> float:
        """Test accuracy with the BN moving statistics (eval-mode forward of the same weights)."""
        m = self.eval_model()
        n = data.shape[0]
        nb = math.ceil(n / self.Bv)
        if max_batches:
            nb = min(nb, max_batches)
        correct = total = 0
        for i in range(nb):
            x = data[i * self.Bv:(i + 1) * self.Bv].to(self.device).float()
            y = labels[i * self.Bv:(i + 1) * self.Bv].to(self.device).long()
            correct += int((m(x).argmax(1) == y).sum())
            total += y.numel()
        return correct / max(1, total)

    def _padded(self, idx: torch.Tensor) -> torch.Tensor:
        """An explicit list of Bv dataset rows, padded to the kernel batch (last row repeated)."""
        idx = idx.to(self.device, torch.int32).reshape(-1)
        assert idx.numel() == self.Bv, (idx.numel(), self.Bv)
        if self.Bv == self.B:
            return idx.contiguous()
        return torch.cat([idx, idx[-1:].expand(self.B - self.Bv)]).contiguous()

    @torch.no_grad()
    def forward_logits(self, idx: torch.Tensor) -> torch.Tensor:
        """Train-mode (batch statistics) logits of the Bv dataset rows ``idx`` via the fused kernels —
        for tests.  Writes activations / statistics but updates nothing."""
        self._forward(self._padded(idx), None, 1, logits_out=self.logits_buf)
        return self.logits_buf[:self.Bv].clone()

    # --- state ----------------------------------------------------------------------------------
    def read_stats(self, step: int) -> Dict[str, float]:
        row = self.stats[(step - 1) % self.stats.shape[0]].tolist()
        return {"global_step": int(row[0]), "loss": row[1], "accuracy": row[2], "lr": row[3]}

    def global_step(self) -> int:
        return int(self.step_t.item())

    def flat_params(self) -> torch.Tensor:
        return self.master.detach().cpu()

    def load_flat_params(self, flat: torch.Tensor, step: Optional[int] = None, state: Optional[torch.Tensor] = None):
        self.master.copy_(flat.to(self.device, torch.float32))
        if state is not None:
            self.state.copy_(state.to(self.device, torch.float32))
        if step is not None:
            self.set_step(step)
        self.refresh_shadows()
