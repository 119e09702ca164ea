"""Generated training order (data/order.py): bijection, sharding, union-batch property, and the
vectorised host twin against a scalar re-implementation of the kernels' Feistel network
(csrc/kernels/common.h order_perm).  Replaces the reference's RandomShuffleQueue order
(/root/reference/cifar10cnn.py:82-90) with a per-epoch permutation that every kernel evaluates."""
import pytest
import torch

from dmlc.data.order import OrderSpec, half_bits_for, permute

M = 0xFFFFFFFF


def _mix(x):
    x &= M
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M
    x ^= x >> 15
    x = (x * 0x846CA68B) & M
    return x ^ (x >> 16)


def _scalar_perm(pos, n, seed, epoch):
    """Line-by-line twin of common.h order_perm (uint32 arithmetic)."""
    h = 1
    while (1 << (2 * h)) < n:
        h += 1
    ek = _mix(_mix((seed ^ 0x5BD1E995) & M) ^ _mix((epoch * 0x85EBCA77 + 0x632BE5AB) & M))
    mask = (1 << h) - 1
    x = pos
    while True:
        l, r = x >> h, x & mask
        for k in range(4):
            t = l ^ (_mix(r ^ ((ek + k * 0x9E3779B9) & M)) & mask)
            l, r = r, t
        x = (l << h) | r
        if x < n:
            return x


@pytest.mark.parametrize("n", [1, 2, 5, 16, 17, 1000, 50000])
def test_permutation_is_a_bijection(n):
    p = permute(torch.arange(n), n, seed=3, epoch=7)
    assert sorted(p.tolist()) == list(range(n))


def test_vectorised_matches_scalar_twin():
    n = 50000
    pos = torch.tensor([0, 1, 2, 12345, 49999, 31337, 777])
    for seed, epoch in [(0, 0), (5, 1), (123456789, 4000000000 % (1 << 32))]:
        got = permute(pos, n, seed, epoch).tolist()
        assert got == [_scalar_perm(int(q), n, seed, epoch) for q in pos], (seed, epoch)


def test_epochs_and_seeds_differ():
    n = 1000
    a = permute(torch.arange(n), n, 0, 0)
    assert not torch.equal(a, permute(torch.arange(n), n, 0, 1))
    assert not torch.equal(a, permute(torch.arange(n), n, 1, 0))
    assert not torch.equal(a, torch.arange(n))


def test_half_bits():
    assert [half_bits_for(n) for n in (1, 4, 5, 16, 17, 50000, 65536, 65537)] == [1, 1, 2, 2, 3, 8, 8, 9]


def test_rank_shards_disjoint_and_union_batch():
    n, B, W = 1000, 16, 4
    specs = [OrderSpec(n, B, W, r, seed=9) for r in range(W)]
    single = OrderSpec(n, W * B, 1, 0, seed=9)
    assert specs[0].period == single.period == n // (W * B)
    for step in (0, 1, single.period - 1, single.period, 3 * single.period + 2):
        union = torch.cat([s.batch(step) for s in specs])
        assert torch.equal(union, single.batch(step)), step
    shards = [set(s.epoch_shard(2).tolist()) for s in specs]
    assert all(len(x) == single.period * B for x in shards)
    assert len(set.union(*shards)) == W * single.period * B


def test_epoch_shard_matches_batches():
    o = OrderSpec(500, 7, 2, 1, seed=1)
    e = 3
    sh = o.epoch_shard(e)
    for j in range(o.period):
        assert torch.equal(sh[j * 7:(j + 1) * 7], o.batch(e * o.period + j))


def test_descriptor_and_validation():
    o = OrderSpec(50000, 256, 8, 3, seed=11)
    assert o.descriptor().tolist() == [50000, 8, 8, 3, 256, 11]
    assert o.period == 24
    with pytest.raises(ValueError):
        OrderSpec(100, 64, 2, 0)
