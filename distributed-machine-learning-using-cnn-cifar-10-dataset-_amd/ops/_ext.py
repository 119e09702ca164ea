"""Loading of the native libraries.

``hip()`` makes ``torch.ops.dmlc.*`` (the CDNA4 kernels) available and FAILS LOUDLY when it cannot:
on a GPU box a silent fallback to PyTorch ops would hide that the native path is not running.
``rt()`` returns the native CPU runtime module (``_dmlc_rt``, pybind11).  Both build in-tree on first use if the
shared object is missing (``_build.py``; a prebuilt ``.so`` in the tree is used as is).
"""
from __future__ import annotations

import os
import threading

import torch

from .. import _build

_lock = threading.Lock()
_loaded = {"hip": False, "rt": False}


def _ensure(kind: str) -> str:
    path = _build.HIP_LIB if kind == "hip" else _build.RT_LIB
    if not os.path.exists(path) or os.environ.get("DMLC_REBUILD"):
        _build.build(hip=(kind == "hip"), rt=(kind == "rt"))
    return path


def hip() -> None:
    with _lock:
        if _loaded["hip"]:
            return
        path = _ensure("hip")
        torch.ops.load_library(path)
        _loaded["hip"] = True


def rt():
    """The native CPU runtime module (pybind11, ``csrc/runtime``)."""
    with _lock:
        if _loaded["rt"]:
            return _loaded["rt"]
        path = _ensure("rt")
        import importlib.util
        spec = importlib.util.spec_from_file_location("_dmlc_rt", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _loaded["rt"] = mod
        return mod


def hip_available() -> bool:
    """True when a GPU is present and the HIP kernels are loaded (raises if the GPU is present but
    the library cannot be built/loaded)."""
    if not torch.cuda.is_available():
        return False
    hip()
    return True
