"""CIFAR-10 binary reader (native), data-dir resolution / extraction, TFRecord event files."""
import io
import os
import struct
import tarfile

import pytest
import torch

from dmlc import config as C
from dmlc import data as Dt
from dmlc.utils.events import EventsWriter, read_tfrecords


def _fixture(dirpath, n_per_file=7, seed=0):
    g = torch.Generator().manual_seed(seed)
    os.makedirs(dirpath, exist_ok=True)
    ref = []
    for f in Dt.cifar.TRAIN_FILES + Dt.cifar.TEST_FILES:
        x = torch.randint(0, 256, (n_per_file, 32, 32, 3), dtype=torch.uint8, generator=g)
        y = torch.randint(0, 10, (n_per_file,), dtype=torch.int32, generator=g)
        Dt.write_records(os.path.join(dirpath, f), x, y)
        ref.append((x, y))
    return ref


def test_reader_matches_reference_decode(tmp_path):
    d = tmp_path / C.EXTRACT_FOLDER
    ref = _fixture(str(d))
    x, y = Dt.load_cifar10(str(tmp_path), train=True)
    assert x.shape == (35, 32, 32, 3) and x.dtype == torch.uint8 and y.dtype == torch.int32
    assert torch.equal(x, torch.cat([r[0] for r in ref[:5]])) and torch.equal(y, torch.cat([r[1] for r in ref[:5]]))
    # the reference decode by hand (cifar10cnn.py:57-65): byte 0 = label, bytes 1.. = CHW -> HWC
    raw = open(d / "data_batch_1.bin", "rb").read()
    rec = raw[3073:2 * 3073]
    assert rec[0] == int(y[1])
    chw = torch.tensor(list(rec[1:]), dtype=torch.uint8).view(3, 32, 32)
    assert torch.equal(chw.permute(1, 2, 0), x[1])
    xt, yt = Dt.load_cifar10(str(tmp_path), train=False)
    assert torch.equal(xt, ref[5][0])


def test_reader_rejects_truncated_file(tmp_path):
    p = tmp_path / "bad.bin"
    p.write_bytes(b"\0" * 3072)
    with pytest.raises(RuntimeError, match="3073"):
        Dt.read_records([str(p)])


def test_prepare_extracts_archive_without_download(tmp_path):
    src = tmp_path / "src"
    _fixture(str(src / C.EXTRACT_FOLDER), n_per_file=2)
    arc = tmp_path / "data" / Dt.cifar.ARCHIVE
    arc.parent.mkdir()
    with tarfile.open(arc, "w:gz") as tf:
        tf.add(src / C.EXTRACT_FOLDER, arcname=C.EXTRACT_FOLDER)
    calls = []
    d = Dt.prepare(str(tmp_path / "data"), allow_download=False, barrier=lambda: calls.append(1))
    assert d == str(tmp_path / "data" / C.EXTRACT_FOLDER) and calls == [1]
    assert Dt.prepare(str(tmp_path / "empty"), allow_download=False) is None


def test_data_dir_resolution():
    assert Dt.resolve_data_dir("/tmp/mnist_data") == os.path.abspath("cifar10data")   # reference default
    assert Dt.resolve_data_dir("/data/c10") == "/data/c10"


def test_synthetic_learnable_labels():
    x, y = Dt.synthetic(64, seed=1, learnable=True)
    assert x.shape == (64, 32, 32, 3) and int(y.min()) >= 0 and int(y.max()) <= 9
    x2, y2 = Dt.synthetic(64, seed=1, learnable=True)
    assert torch.equal(x, x2) and torch.equal(y, y2)


def test_events_file_is_valid_tfrecord(tmp_path):
    w = EventsWriter(str(tmp_path))
    w.scalars(100, {"global_step/sec": 12.5, "loss": 2.0})
    w.close()
    recs = list(read_tfrecords(w.path))
    assert len(recs) == 2
    assert b"brain.Event:2" in recs[0]
    ev = recs[1]
    assert ev[0] == 0x09                              # wall_time (double)
    assert ev[9:11] == bytes([0x10, 100])             # step = 100
    assert b"global_step/sec" in ev and struct.pack("<f", 12.5) in ev
