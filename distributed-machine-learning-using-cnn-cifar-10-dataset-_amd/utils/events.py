"""Observability: TensorBoard-compatible event files (native TFRecord framing) and JSONL metrics.

The reference's only timing signal is TF1's implicit chief StepCounterHook writing
``global_step/sec`` into ``<log_dir>/events.out.tfevents.*`` (MonitoredTrainingSession,
/root/reference/cifar10cnn.py:222).  :class:`EventsWriter` writes the same
file format (TFRecord of tf.Event protos, encoded by csrc/runtime/records_cifar.cpp) so TensorBoard
can read it; :class:`MetricsLog` adds the machine-readable JSONL stream (loss, accuracy, lr,
images/sec, step time).
"""
from __future__ import annotations

import json
import os
import socket
import time
from typing import Dict, Optional

from ..ops import _ext


class EventsWriter:
    def __init__(self, log_dir: str, suffix: str = ""):
        os.makedirs(log_dir, exist_ok=True)
        self.rt = _ext.rt()
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}{suffix}"
        self.path = os.path.join(log_dir, name)
        self.f = open(self.path, "ab")
        self.f.write(self.rt.tfrecord_frame(self.rt.event_file_version(time.time())))
        self.f.flush()

    def scalars(self, step: int, values: Dict[str, float]):
        ev = self.rt.event_scalars(time.time(), int(step), list(values), [float(v) for v in values.values()])
        self.f.write(self.rt.tfrecord_frame(ev))
        self.f.flush()

    def close(self):
        if self.f:
            self.f.close()
            self.f = None


class MetricsLog:
    def __init__(self, path: Optional[str]):
        self.f = None
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self.f = open(path, "a")

    def write(self, **rec):
        if self.f:
            rec.setdefault("time", time.time())
            self.f.write(json.dumps(rec) + "\n")
            self.f.flush()

    def close(self):
        if self.f:
            self.f.close()
            self.f = None


def read_tfrecords(path: str):
    """Yield the payloads of a TFRecord file, verifying both masked crc32c (for tests/tools)."""
    import struct
    rt = _ext.rt()
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack("<Q", data[i:i + 8])
        (lc,) = struct.unpack("<I", data[i + 8:i + 12])
        if rt.crc_mask(rt.crc32c(data[i:i + 8])) != lc:
            raise ValueError("TFRecord length crc mismatch")
        payload = data[i + 12:i + 12 + n]
        (dc,) = struct.unpack("<I", data[i + 12 + n:i + 16 + n])
        if rt.crc_mask(rt.crc32c(payload)) != dc:
            raise ValueError("TFRecord data crc mismatch")
        yield payload
        i += 16 + n
