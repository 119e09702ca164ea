"""TensorBundle-V2 checkpoint format (native writer/reader, csrc/runtime/tensor_bundle.cpp).

TensorFlow is not installed, so compatibility is pinned by (a) golden values from the format specs
(crc32c check value, LevelDB footer magic, proto3 encodings written out by hand below) and (b) an
independent pure-Python SSTable/proto parser in this file that must agree with the native code.
Reference contract: SURVEY.md §5.4 (/root/reference/cifar10cnn.py:222)."""
import os
import struct

import pytest
import torch

from dmlc import checkpoint as CK
from dmlc.models import cifar_cnn as M
from dmlc.ops import _ext


@pytest.fixture(scope="module")
def rt():
    return _ext.rt()


# ---- independent pure-Python oracle ---------------------------------------------------------------
def py_crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
    return c ^ 0xFFFFFFFF


def py_mask(c):
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def varint(buf, i):
    r = s = 0
    while True:
        b = buf[i]
        i += 1
        r |= (b & 0x7F) << s
        s += 7
        if not b & 0x80:
            return r, i


def py_parse_block(blk):
    nrest = struct.unpack("<I", blk[-4:])[0]
    end = len(blk) - 4 - 4 * nrest
    i, key, out = 0, b"", []
    while i < end:
        sh, i = varint(blk, i)
        ns, i = varint(blk, i)
        vl, i = varint(blk, i)
        key = key[:sh] + blk[i:i + ns]
        i += ns
        out.append((key, blk[i:i + vl]))
        i += vl
    return out


def py_read_table(img):
    footer = img[-48:]
    assert struct.unpack("<Q", footer[40:])[0] == 0xDB4775248B80FB57
    _, i = varint(footer, 0)
    _, i = varint(footer, i)
    io, i = varint(footer, i)
    isz, i = varint(footer, i)

    def block(off, size):
        data = img[off:off + size]
        assert img[off + size] == 0
        crc = struct.unpack("<I", img[off + size + 1:off + size + 5])[0]
        assert crc == py_mask(py_crc32c(data + b"\x00"))
        return py_parse_block(data)

    kv = []
    for _, h in block(io, isz):
        off, j = varint(h, 0)
        size, _ = varint(h, j)
        kv += block(off, size)
    return kv


def py_parse_proto(b):
    i, out = 0, []
    while i < len(b):
        tag, i = varint(b, i)
        f, w = tag >> 3, tag & 7
        if w == 0:
            v, i = varint(b, i)
        elif w == 5:
            v = struct.unpack("<I", b[i:i + 4])[0]
            i += 4
        elif w == 2:
            n, i = varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError(w)
        out.append((f, v))
    return out


# ---- golden values --------------------------------------------------------------------------------
def test_crc32c_golden(rt):
    assert rt.crc32c(b"123456789") == 0xE3069283          # RFC 3720 check value
    assert rt.crc32c(b"") == 0
    data = os.urandom(1000)
    assert rt.crc32c(data) == py_crc32c(data)
    assert rt.crc32c(data[500:], rt.crc32c(data[:500])) == rt.crc32c(data)
    for v in (0, 1, 0xDEADBEEF, 0xFFFFFFFF):
        assert rt.crc_unmask(rt.crc_mask(v)) == v
        assert rt.crc_mask(v) == py_mask(v)


def test_header_and_entry_encoding_golden(rt):
    # BundleHeaderProto{num_shards: 1, version{producer: 1}}
    assert rt.encode_header(1) == bytes([0x08, 0x01, 0x1A, 0x02, 0x08, 0x01])
    # BundleEntryProto{dtype: DT_FLOAT, shape{dim{size:2} dim{size:3}}, offset: 0, size: 24, crc32c}
    e = rt.encode_entry(1, [2, 3], 0, 0, 24, 0x12345678)
    assert e[:12] == bytes([0x08, 0x01, 0x12, 0x08, 0x12, 0x02, 0x08, 0x02, 0x12, 0x02, 0x08, 0x03])
    assert e[12:14] == bytes([0x28, 24]) and e[14] == 0x35
    assert struct.unpack("<I", e[15:19])[0] == py_mask(0x12345678)
    # a scalar keeps an (empty) shape field; a non-zero offset is encoded as field 4
    s = rt.encode_entry(9, [], 0, 40, 8, 0)
    assert s[:4] == bytes([0x08, 0x09, 0x12, 0x00]) and s[4:6] == bytes([0x20, 40])


def test_table_roundtrip_multi_block_and_separators(rt):
    keys = [b""] + [f"k{i:04d}/name".encode() for i in range(300)]
    vals = [os.urandom(i % 50) for i in range(len(keys))]
    img = rt.build_table(keys, vals, 256, 16)                  # tiny blocks -> many data blocks
    got = rt.read_table(img)
    assert [k for k, _ in got] == keys and [v for _, v in got] == vals
    assert py_read_table(img) == list(zip(keys, vals))
    # empty table: footer + empty metaindex + empty index
    assert rt.read_table(rt.build_table([], [])) == []


def test_corruption_is_detected(rt, tmp_path):
    prefix = str(tmp_path / "model.ckpt-1")
    CK.write_bundle(prefix, {"a": torch.arange(10, dtype=torch.float32)})
    data = prefix + ".data-00000-of-00001"
    raw = bytearray(open(data, "rb").read())
    raw[3] ^= 0xFF
    open(data, "wb").write(bytes(raw))
    with pytest.raises(RuntimeError, match="crc32c"):
        CK.read_bundle(prefix)
    idx = bytearray(open(prefix + ".index", "rb").read())
    idx[2] ^= 0x01
    open(prefix + ".index", "wb").write(bytes(idx))
    with pytest.raises(RuntimeError):
        CK.read_bundle(prefix)


def test_model_checkpoint_layout(tmp_path):
    flat = M.init_flat_params(torch.Generator().manual_seed(0))
    tensors = CK.model_tensors(flat, global_step=1234, generation_num=0)
    prefix = str(tmp_path / "model.ckpt-1234")
    CK.write_bundle(prefix, tensors)
    assert os.path.exists(prefix + ".index") and os.path.exists(prefix + ".data-00000-of-00001")
    img = open(prefix + ".index", "rb").read()
    kv = py_read_table(img)
    keys = [k.decode() for k, _ in kv]
    expect = sorted([s.name for s in M.PARAM_SPECS] + ["global_step", "Variable"])
    assert keys == [""] + expect
    blob = open(prefix + ".data-00000-of-00001", "rb").read()
    assert len(blob) == 4 * M.NUM_PARAMS + 8 + 4
    # every entry: dtype / shape / offset / size / crc against the raw data file
    off = 0
    for k, v in kv[1:]:
        fields = dict()
        dims = []
        for f, val in py_parse_proto(v):
            if f == 2:
                dims = [dict(py_parse_proto(d)).get(1, 0) for ff, d in py_parse_proto(val) if ff == 2]
            else:
                fields[f] = val
        name = k.decode()
        t = tensors[name]
        assert tuple(dims) == tuple(t.shape), name
        assert fields[1] == {torch.float32: 1, torch.int64: 9, torch.int32: 3}[t.dtype]
        assert fields.get(4, 0) == off
        size = fields[5]
        assert size == t.numel() * t.element_size()
        assert fields[6] == py_mask(py_crc32c(blob[off:off + size]))
        off += size
    back = CK.read_bundle(prefix)
    for k, t in tensors.items():
        assert back[k].dtype == t.dtype and torch.equal(back[k], t), k
    # conv kernels HWIO, fc weights [in,out], full_weight_1 rows = 6*6*64 NHWC flatten order
    assert tuple(back["model_definition/conv1/conv1_kernel"].shape) == (5, 5, 3, 64)
    assert tuple(back["model_definition/full1/full_weight_1"].shape) == (2304, 384)
    flat2, step, gen = CK.load_model_tensors(back)
    assert step == 1234 and gen == 0
    assert torch.equal(flat2, flat)


def test_manager_state_file_and_max_to_keep(tmp_path):
    flat = torch.zeros(M.FLAT_SIZE)
    mgr = CK.CheckpointManager(str(tmp_path), max_to_keep=5, secs=600)
    assert mgr.due()
    for step in range(0, 700, 100):
        mgr.save(step, CK.model_tensors(flat, step))
    assert not mgr.due()
    latest, all_paths = CK.read_state(str(tmp_path))
    assert latest == str(tmp_path / "model.ckpt-600")
    assert all_paths == [str(tmp_path / f"model.ckpt-{s}") for s in range(200, 700, 100)]
    assert CK.latest_checkpoint(str(tmp_path)) == latest
    assert not os.path.exists(tmp_path / "model.ckpt-100.index")
    text = open(tmp_path / "checkpoint").read().splitlines()
    assert text[0] == f'model_checkpoint_path: "{tmp_path}/model.ckpt-600"'
    assert text[1].startswith("all_model_checkpoint_paths: ")
    # a relative path (as TF writes with save_relative_paths) is resolved against log_dir
    (tmp_path / "checkpoint").write_text('model_checkpoint_path: "model.ckpt-500"\n')
    assert CK.latest_checkpoint(str(tmp_path)) == str(tmp_path / "model.ckpt-500")
    # a new manager picks up the kept list
    mgr2 = CK.CheckpointManager(str(tmp_path), max_to_keep=2)
    assert mgr2.kept == [str(tmp_path / "model.ckpt-500")]


def test_bf16_and_int_tensors_roundtrip(tmp_path):
    t = {"w": torch.randn(3, 4).to(torch.bfloat16), "i8": torch.arange(-5, 5, dtype=torch.int8),
         "u8": torch.arange(0, 200, dtype=torch.uint8), "h": torch.randn(7).half()}
    CK.write_bundle(str(tmp_path / "x"), t)
    back = CK.read_bundle(str(tmp_path / "x"))
    for k in t:
        assert torch.equal(back[k], t[k]), k


def test_save_without_protobuf_keeps_bundle(tmp_path, monkeypatch):
    """metagraph imports google.protobuf lazily, so a missing protobuf runtime must be
    caught around the .meta build/write, not only around the module import; the bundle + state file
    are still written and the manager stops trying."""
    import builtins
    from dmlc.utils import metagraph as MG
    real_import = builtins.__import__

    def no_protobuf(name, *args, **kw):
        if name.startswith("google.protobuf") or (name == "google" and args and args[2] and "protobuf" in args[2]):
            raise ImportError("No module named 'google.protobuf' (simulated)")
        return real_import(name, *args, **kw)

    if hasattr(MG._classes, "cache_clear"):
        MG._classes.cache_clear()
    monkeypatch.setattr(MG, "_F", None, raising=False)
    monkeypatch.setattr(builtins, "__import__", no_protobuf)
    flat = torch.arange(M.FLAT_SIZE, dtype=torch.float32) * 1e-6
    mgr = CK.CheckpointManager(str(tmp_path), max_to_keep=5, graph_info=dict(model="cifar_cnn", batch=128, crop=24,
                                                                          relu_logits=True))
    prefix = mgr.save(7, CK.model_tensors(flat, 7))
    assert os.path.exists(prefix + ".index") and os.path.exists(prefix + ".data-00000-of-00001")
    assert not os.path.exists(prefix + ".meta")
    assert mgr.graph_info is None
    assert CK.latest_checkpoint(str(tmp_path)) == prefix
    monkeypatch.setattr(builtins, "__import__", real_import)
    if hasattr(MG._classes, "cache_clear"):
        MG._classes.cache_clear()
    back = CK.read_bundle(prefix)
    flat2, step, _ = CK.load_model_tensors(back)
    n = sum(sp.numel for sp in M.PARAM_SPECS)       # the flat buffer's padding tail is not saved
    assert step == 7 and torch.equal(flat2[:n], flat[:n])
