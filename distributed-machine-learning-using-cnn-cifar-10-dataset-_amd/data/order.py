"""Training-data order: a keyed per-epoch permutation that every kernel can evaluate by itself.

The reference shuffles with TF queue runners -- ``string_input_producer`` (filename order reshuffled
every epoch) feeding a ``RandomShuffleQueue`` of >= 5000 examples (/root/reference/cifar10cnn.py:82,
:85-90) -- and every worker reads the whole, unsharded training set.
Here the order of epoch ``e`` is a bijection ``perm_e`` of ``[0, n)``: a 4-round balanced Feistel
network on ``2*half_bits`` bits with round keys derived from ``(seed, e)``, cycle-walked back into
``[0, n)``.  Because it is a pure function of ``(position, seed, epoch)``, the HIP kernels compute the
dataset row of every batch row from the device step counter (csrc/kernels/common.h ``order_perm``,
``batch_index``): there is no permutation buffer, no host ``randperm`` at an epoch boundary, and a
captured multi-step HIP graph runs across epochs unchanged.

Sharding (D6): at step ``s`` (epoch ``s // period``, row ``j = s % period``) rank ``r`` of ``W`` reads
positions ``(j*W + r)*B + b``.  The union over ranks of one step is therefore positions
``[j*W*B, (j+1)*W*B)`` in rank order -- exactly the batch one rank with batch ``W*B`` reads -- so a
W-rank data-parallel step equals the single-process step on the union batch.

This module is the host twin (bit-identical; tests pin it against the kernels) used by the eager
engine, the tests and the descriptor handed to the kernels.
"""
from __future__ import annotations

import dataclasses

import torch

M32 = 0xFFFFFFFF


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """uint32 avalanche mixer on int64 tensors (values in [0, 2^32)); twin of common.h mix32."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & M32
    return x ^ (x >> 16)


def _mix32_int(x: int) -> int:
    x &= M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    return x ^ (x >> 16)


def half_bits_for(n: int) -> int:
    """Smallest h >= 1 with 4**h >= n (the Feistel domain 2^(2h) covers [0, n))."""
    h = 1
    while (1 << (2 * h)) < n:
        h += 1
    return h


def epoch_key(seed: int, epoch: int) -> int:
    return _mix32_int(_mix32_int((seed & M32) ^ 0x5BD1E995) ^ _mix32_int((epoch * 0x85EBCA77 + 0x632BE5AB) & M32))


def permute(pos: torch.Tensor, n: int, seed: int, epoch: int) -> torch.Tensor:
    """perm_epoch(pos) for int tensor ``pos`` (values in [0, n)); returns int64."""
    h = half_bits_for(n)
    mask = (1 << h) - 1
    ek = epoch_key(seed, epoch)
    keys = [(ek + k * 0x9E3779B9) & M32 for k in range(4)]
    x = pos.to(torch.int64).clone()

    def rounds(v):
        left, right = v >> h, v & mask
        for k in keys:
            left, right = right, left ^ (_mix32(right ^ k) & mask)
        return (left << h) | right

    todo = torch.ones_like(x, dtype=torch.bool)
    while bool(todo.any()):
        x[todo] = rounds(x[todo])
        todo = x >= n
    return x


@dataclasses.dataclass(frozen=True)
class OrderSpec:
    """The generated training order of one rank: ``n`` dataset rows, batch ``B`` (valid rows per
    step), ``world`` ranks, this ``rank``, shuffle ``seed``."""
    n: int
    B: int
    world: int = 1
    rank: int = 0
    seed: int = 0

    def __post_init__(self):
        if self.n < self.world * self.B:
            raise ValueError(f"dataset of {self.n} rows holds no full step of {self.world} x {self.B}")

    @property
    def period(self) -> int:
        """Steps per epoch (every rank reads ``period * B`` distinct rows per epoch)."""
        return self.n // (self.world * self.B)

    def descriptor(self) -> torch.Tensor:
        """Host int64 [6] descriptor the kernels take in place of an index list (check.h index_src)."""
        return torch.tensor([self.n, half_bits_for(self.n), self.world, self.rank, self.B, self.seed & M32],
                            dtype=torch.int64)

    def batch(self, step: int, rank: int = None) -> torch.Tensor:
        """Dataset rows (int64 [B]) of ``rank``'s batch at global step ``step``."""
        r = self.rank if rank is None else rank
        epoch, j = divmod(int(step), self.period)
        pos = (j * self.world + r) * self.B + torch.arange(self.B, dtype=torch.int64)
        return permute(pos, self.n, self.seed, epoch)

    def epoch_shard(self, epoch: int) -> torch.Tensor:
        """This rank's rows for a whole epoch, batch after batch (int64 [period * B])."""
        j = torch.arange(self.period, dtype=torch.int64).view(-1, 1)
        pos = (j * self.world + self.rank) * self.B + torch.arange(self.B, dtype=torch.int64).view(1, -1)
        return permute(pos.reshape(-1), self.n, self.seed, epoch)
