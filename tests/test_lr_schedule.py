"""Learning-rate machinery: the reference's staircase decay (cifar10cnn.py:159-164), plus the
large-batch recipe of BASELINE config 5 -- linear scaling with the global batch and a linear warm-up
-- on the eager engine (the fused SGD kernels' lr_of is checked against the same formula in
tests/test_fused_gpu.py)."""
import math

import pytest

from dmlc import cli
from dmlc import config as C
from dmlc.engine.eager import EagerTrainer
from dmlc.data import synthetic


def _want(step, lr0, decay=0.9, every=250.0, warmup=0, staircase=True):
    lr = lr0 * decay ** math.floor(step / every) if staircase else lr0
    return lr * (step + 1) / warmup if step < warmup else lr


def test_flags_reach_the_config_and_scale_linearly():
    cfg, _ = cli.parse(["--batch_size", "1024", "--lr_scaling", "linear", "--warmup_steps", "50"])
    assert cfg.lr_scaling == "linear" and cfg.warmup_steps == 50 and cfg.lr_base_batch == 128
    # global batch 8192 = 8 GPUs x 1024: 64x the reference's 128
    assert C.effective_lr(cfg, 8) == pytest.approx(cfg.learning_rate * 64)
    assert C.effective_lr(C.TrainConfig(), 8) == C.TrainConfig().learning_rate     # default: reference


@pytest.mark.parametrize("warmup,staircase", [(0, True), (5, True), (7, False)])
def test_eager_schedule(warmup, staircase):
    x, y = synthetic(64, seed=1)
    tr = EagerTrainer("cifar_cnn", 8, x, y, lr=0.2, lr_decay=0.5, decay_steps=3, staircase=staircase,
                      warmup_steps=warmup)
    for s in range(12):
        assert tr.lr(s) == pytest.approx(_want(s, 0.2, 0.5, 3.0, warmup, staircase)), s
