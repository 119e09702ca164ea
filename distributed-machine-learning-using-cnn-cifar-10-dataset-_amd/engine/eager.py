"""Eager (PyTorch-op) training engine.

Used for (a) the CPU "plumbing" configuration (BASELINE config 1), (b) the fp32-accurate GPU mode
(``backend='hip_f32'``: the model's matmuls/convs on the fp32 HIP kernels of ops/f32.py, driven
step by step from here, optionally captured into one HIP graph), (c) the framework-default
comparison line of the benchmark, and (d) the numerics oracle for the fused engines.  Semantics follow the reference training step
(/root/reference/cifar10cnn.py:159-164, :230): sparse softmax cross-entropy (mean), plain SGD,
staircase LR decay, global_step++.  Data parallelism is synchronous: the flat gradient is
all-reduced in two buckets (fc first, then conv — SURVEY.md §2.D) and averaged.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.distributed as dist

from .. import config as C
from ..data.order import OrderSpec
from ..models import build_model


class EagerTrainer:
    def __init__(self, model: str, batch_size: int, data: torch.Tensor, labels: torch.Tensor, *,
                 device="cpu", world_size: int = 1, rank: int = 0, process_group=None, dtype: str = "fp32",
                 lr: float = C.LEARNING_RATE, lr_decay: float = C.LR_DECAY,
                 decay_steps: float = C.NUM_GENS_TO_WAIT, staircase: bool = True, relu_logits: bool = True,
                 crop: int = C.CROP_HEIGHT, seed: int = 0, flat_params: Optional[torch.Tensor] = None,
                 augment: bool = False, graph: bool = False, warmup_steps: int = 0, backend: str = "torch"):
        self.device = torch.device(device)
        if backend == "hip_f32" and (self.device.type != "cuda" or dtype != "fp32"):
            raise ValueError("the hip_f32 backend is the fp32 GPU path (device cuda, dtype fp32)")
        self.backend = backend
        self.model = build_model(model, seed=seed, relu_logits=relu_logits, flat=flat_params,
                                 backend=backend).to(self.device)
        self.B = int(batch_size)
        self.data = data.to(self.device)
        self.labels = labels.to(self.device).long()
        self.world_size, self.rank, self.pg = world_size, rank, process_group
        self.dtype = dtype
        self.lr0, self.decay, self.decay_steps, self.staircase = lr, lr_decay, decay_steps, staircase
        self.warmup = int(warmup_steps)
        self.crop = crop
        self.off = (32 - crop) // 2
        self.seed = seed
        self.augment = augment
        self.n_data = self.data.shape[0]
        # the same generated order as the fused kernels (data/order.py), so engines agree step by step
        self.order = OrderSpec(self.n_data, self.B, world_size, rank, seed)
        self.period = self.order.period
        self.cur_epoch = -1
        self.perm = None
        self.global_step = 0
        self.last_loss = float("nan")
        self.last_acc = float("nan")
        self.buckets = self.model.grad_buckets() if hasattr(self.model, "grad_buckets") else None
        # HIP-graph capture of the whole step (single process, GPU, no augmentation): static batch
        # buffers + a device-resident LR so the captured SGD stays valid across replays
        self.use_graph = graph and self.device.type == "cuda" and world_size == 1 and not augment
        self.graph = None
        self._warm = 0

    # ------------------------------------------------------------------------------------------
    def lr(self, step: int) -> float:
        lr = self.lr0 * self.decay ** math.floor(step / self.decay_steps) if self.staircase else self.lr0
        if step < self.warmup:                 # linear warm-up, as the fused SGD kernels (lr_of)
            lr *= (step + 1) / self.warmup
        return lr

    def epoch_permutation(self, epoch: int) -> torch.Tensor:
        return self.order.epoch_shard(epoch)

    def batch(self, step: int):
        epoch = step // self.period
        if epoch != self.cur_epoch:
            self.perm = self.epoch_permutation(epoch).to(self.device)
            self.cur_epoch = epoch
        row = step % self.period
        idx = self.perm[row * self.B:(row + 1) * self.B]
        return self.images(idx), self.labels[idx]

    def images(self, idx: torch.Tensor) -> torch.Tensor:
        o, c = self.off, self.crop
        x = self.data[idx]
        if self.augment:
            # random crop (±off) + horizontal flip, per batch (optional, D5)
            dy, dx = (int(v) for v in torch.randint(0, 2 * o + 1, (2,)))
            x = x[:, dy:dy + c, dx:dx + c, :]
            if torch.rand(()) < 0.5:
                x = x.flip(2)
        else:
            x = x[:, o:o + c, o:o + c, :]
        return x.float()

    def _allreduce_grads(self):
        if self.world_size == 1:
            return
        for b in (self.buckets or [None]):
            for p in self.model.parameters():
                if p.grad is None:
                    continue
                g = p.grad if b is None else p.grad.view(-1)[b[0]:b[1]]
                dist.all_reduce(g, group=self.pg)
                g.div_(self.world_size)
            if b is None:
                break

    def _fwd_bwd_sgd(self, x, y, lr):
        """One training step's device work; ``lr`` is a float or a 0-d device tensor."""
        use_amp = self.dtype == "bf16" and self.device.type == "cuda"
        with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=use_amp):
            logits = self.model(x)
        loss = torch.nn.functional.cross_entropy(logits.float(), y)
        loss.backward()
        self._allreduce_grads()
        with torch.no_grad():
            for p in self.model.parameters():
                if p.grad is not None:
                    if torch.is_tensor(lr):
                        p.addcmul_(p.grad, lr, value=-1.0)
                    else:
                        p.add_(p.grad, alpha=-lr)
        if hasattr(self.model, "after_step"):
            self.model.after_step()
        return loss.detach(), (logits.detach().argmax(1) == y).float().mean()

    def step(self):
        x, y = self.batch(self.global_step)
        self.model.train()
        if not self.use_graph:
            for p in self.model.parameters():
                p.grad = None
            self.last_loss, self.last_acc = self._fwd_bwd_sgd(x, y, self.lr(self.global_step))
            self.global_step += 1
            return
        if self.graph is None:
            if self._warm == 0:
                self._xs, self._ys = x.clone(), y.clone()
                self._lr_t = torch.zeros((), device=self.device)
                self._side = torch.cuda.Stream(device=self.device)
            self._xs.copy_(x)
            self._ys.copy_(y)
            self._lr_t.fill_(self.lr(self.global_step))
            self._side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self._side):          # warm-up off the capture stream
                for p in self.model.parameters():
                    p.grad = None
                self.last_loss, self.last_acc = self._fwd_bwd_sgd(self._xs, self._ys, self._lr_t)
            torch.cuda.current_stream(self.device).wait_stream(self._side)
            self._warm += 1
            self.global_step += 1
            if self._warm == 3:
                for p in self.model.parameters():
                    p.grad = None
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode="thread_local"):   # records only (model unchanged)
                    self._out = self._fwd_bwd_sgd(self._xs, self._ys, self._lr_t)
                self.graph = g
                torch.cuda.synchronize(self.device)
            return
        self._xs.copy_(x)
        self._ys.copy_(y)
        self._lr_t.fill_(self.lr(self.global_step))
        self.graph.replay()
        self.last_loss, self.last_acc = self._out
        self.global_step += 1

    def flat_params(self) -> torch.Tensor:
        return self.model.flat.detach().cpu().clone()

    @torch.no_grad()
    def load_flat_params(self, flat: torch.Tensor, step: Optional[int] = None):
        self.model.flat.copy_(flat.to(self.model.flat.device, self.model.flat.dtype))
        if hasattr(self.model, "after_load"):
            self.model.after_load()
        if step is not None:
            self.global_step = int(step)

    @torch.no_grad()
    def evaluate(self, data: torch.Tensor, labels: torch.Tensor, max_batches: int = 0) -> float:
        self.model.eval()
        n = data.shape[0]
        nb = math.ceil(n / self.B)
        if max_batches:
            nb = min(nb, max_batches)
        correct = total = 0
        o, c = self.off, self.crop
        for i in range(nb):
            x = data[i * self.B:(i + 1) * self.B].to(self.device)[:, o:o + c, o:o + c, :].float()
            y = labels[i * self.B:(i + 1) * self.B].to(self.device).long()
            with torch.autocast(self.device.type, dtype=torch.bfloat16,
                                enabled=self.dtype == "bf16" and self.device.type == "cuda"):
                logits = self.model(x)
            correct += int((logits.argmax(1) == y).sum())
            total += y.numel()
        return correct / max(1, total)
