"""CIFAR-10 input: locate / (optionally) download / extract / read, plus synthetic data.

Reference behaviour (/root/reference/cifar10cnn.py:34-91) and the fixes:
  * ``download_data`` (:34-52) ran in EVERY process against a relative ``./cifar10data`` (race R1),
    extracted only when it had just downloaded (D9) and used ``urllib`` without importing
    ``urllib.request`` (D8).  Here only the chief (rank 0) prepares the data, the others wait on a
    barrier; extraction happens whenever the batches folder is missing; downloading is opt-in
    (``allow_download``) because training boxes are offline.
  * ``--data_dir`` is honoured (D7): ``<data_dir>/cifar-10-batches-bin/*.bin`` or ``<data_dir>/*.bin``.
  * Records are parsed by the native reader (``csrc/runtime/records_cifar.cpp``, mmap +
    multithreaded CHW→HWC) once, into a uint8 NHWC tensor that is then kept resident in HBM; the
    per-batch gather/crop/cast happens inside the first convolution kernel (N1-N3 of SURVEY §2.B).
  * Train files ``data_batch_1..5.bin``, test file ``test_batch.bin`` (:78-80).
"""
from __future__ import annotations

import os
import tarfile
from typing import Callable, List, Optional, Tuple

import numpy as np
import torch

from .. import config as C
from ..ops import _ext

TRAIN_FILES = [f"data_batch_{i}.bin" for i in range(1, 6)]
TEST_FILES = ["test_batch.bin"]
ARCHIVE = "cifar-10-binary.tar.gz"


def resolve_data_dir(data_dir: Optional[str]) -> str:
    """The reference's ``--data_dir`` default (/tmp/mnist_data) was a leftover and ignored; an unset
    or default value falls back to the reference's hard-coded ``./cifar10data`` (:26)."""
    if not data_dir or data_dir == "/tmp/mnist_data":
        return os.path.abspath(C.DATA_DIR)
    return os.path.abspath(data_dir)


def batches_dir(data_dir: str) -> Optional[str]:
    for d in (os.path.join(data_dir, C.EXTRACT_FOLDER), data_dir):
        if all(os.path.exists(os.path.join(d, f)) for f in TRAIN_FILES + TEST_FILES):
            return d
    return None


def prepare(data_dir: str, allow_download: bool = False, barrier: Optional[Callable[[], None]] = None,
            is_chief: bool = True) -> Optional[str]:
    """Make ``<data_dir>/cifar-10-batches-bin`` exist (chief only, others wait); return its path or
    None when the data is unavailable (offline and no archive)."""
    if is_chief and batches_dir(data_dir) is None:
        os.makedirs(data_dir, exist_ok=True)
        archive = os.path.join(data_dir, ARCHIVE)
        if not os.path.exists(archive) and allow_download:
            import urllib.request   # D8: the reference imported only `urllib`
            tmp = archive + ".part"
            urllib.request.urlretrieve(C.CIFAR10_URL, tmp)
            os.replace(tmp, archive)
        if os.path.exists(archive):
            with tarfile.open(archive, "r:gz") as tf:
                members = [m for m in tf.getmembers() if m.isfile() and m.name.endswith(".bin")
                           and not os.path.isabs(m.name) and ".." not in m.name.split("/")]
                tf.extractall(data_dir, members=members)
    if barrier is not None:
        barrier()
    return batches_dir(data_dir)


def read_records(files: List[str], threads: int = 8) -> Tuple[torch.Tensor, torch.Tensor]:
    """Native parse of CIFAR-10 binary files -> (uint8 [N,32,32,3] NHWC, int32 [N])."""
    img, lab, n = _ext.rt().read_cifar(list(files), threads)
    images = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).view(n, 32, 32, 3)
    labels = torch.from_numpy(np.frombuffer(lab, dtype=np.int32).copy())
    return images, labels


def load_cifar10(data_dir: str, train: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    d = batches_dir(data_dir)
    if d is None:
        raise FileNotFoundError(f"CIFAR-10 binary batches not found under {data_dir}")
    files = [os.path.join(d, f) for f in (TRAIN_FILES if train else TEST_FILES)]
    return read_records(files)


def write_records(path: str, images: torch.Tensor, labels: torch.Tensor) -> None:
    """Write uint8 NHWC images + labels in the CIFAR-10 binary record format (test fixtures)."""
    imgs = images.to(torch.uint8).cpu().numpy()
    chw = imgs.transpose(0, 3, 1, 2).reshape(imgs.shape[0], 3072)
    rec = np.concatenate([labels.cpu().numpy().astype(np.uint8)[:, None], chw], axis=1)
    with open(path, "wb") as f:
        f.write(rec.tobytes())


def synthetic(n: int, seed: int = 0, learnable: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """Synthetic CIFAR-shaped data (uint8 [n,32,32,3], int32 labels).  ``learnable`` ties the label
    to the image (mean red intensity decile) so convergence tests have signal."""
    g = torch.Generator().manual_seed(seed)
    images = torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, generator=g)
    if learnable:
        labels = (images[:, 4:28, 4:28, 0].float().mean(dim=(1, 2)) - 112.0).div(3.2).clamp(0, 9).to(torch.int32)
    else:
        labels = torch.randint(0, 10, (n,), dtype=torch.int32, generator=g)
    return images, labels


def dataset(cfg, is_chief: bool = True, barrier=None):
    """(train_images, train_labels, test_images, test_labels) for a TrainConfig."""
    if cfg.synthetic:
        tr = synthetic(cfg.synthetic_size, seed=cfg.seed, learnable=True)
        te = synthetic(max(cfg.batch_size, cfg.synthetic_size // 5), seed=cfg.seed + 1, learnable=True)
        return tr + te
    d = resolve_data_dir(cfg.data_dir)
    if prepare(d, allow_download=getattr(cfg, "download", False), barrier=barrier, is_chief=is_chief) is None:
        raise FileNotFoundError(
            f"no CIFAR-10 binary batches in {d} (and no {ARCHIVE}); pass --synthetic or --download")
    return load_cifar10(d, True) + load_cifar10(d, False)
