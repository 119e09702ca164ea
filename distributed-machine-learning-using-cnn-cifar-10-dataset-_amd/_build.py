"""In-tree build of the native libraries (no hipify, no JIT cache outside the repo).

* ``_lib/libdmlc_hip.so`` — CDNA4 HIP kernels (``csrc/kernels/*.hip``, hipcc --offload-arch=gfx950)
  + their torch.ops bindings (``csrc/bindings/torch_ops.cpp``).
* ``_lib/_dmlc_rt*.so``   — CPU runtime, a pybind11 module (``csrc/runtime/*.cpp``): CIFAR-10
  binary reader, TF TensorBundle-V2 checkpoint writer/reader, crc32c, TFRecord/event writer.

Objects are rebuilt only when a content hash of their sources + flags changes, so importing the
package (or running the tests) after a build costs nothing.  ``python -m dmlc._build`` forces a
build; ``DMLC_BUILD_VERBOSE=1`` prints the commands.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
LIB_DIR = os.path.join(PKG_DIR, "_lib")
OBJ_DIR = os.path.join(REPO, "build", "obj")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

# DMLC_TIMING=1 builds a separate diagnostic library with per-phase s_memrealtime stamps
# (tools/ktiming.py); the default library never contains them.
TIMING = os.environ.get("DMLC_TIMING") == "1"
# DMLC_VARIANT="name:-DFLAG ..." builds an experiment library libdmlc_hip_<name>.so with extra hipcc
# flags (A/B kernel variants on the GPU box without touching the production library)
_VAR = os.environ.get("DMLC_VARIANT", "")
VARIANT, VARIANT_FLAGS = (_VAR.split(":", 1)[0], _VAR.split(":", 1)[1].split()) if _VAR else ("", [])
_SUFFIX = "_timing" if TIMING else (f"_{VARIANT}" if VARIANT else "")
HIP_LIB = os.path.join(LIB_DIR, f"libdmlc_hip{_SUFFIX}.so")
RT_LIB = os.path.join(LIB_DIR, "_dmlc_rt" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


def _torch_paths():
    import torch.utils.cpp_extension as ce
    import torch
    inc = ce.include_paths()
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hash(paths, flags) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _run(cmd):
    if os.environ.get("DMLC_BUILD_VERBOSE"):
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _compile(src, deps, out, cmd_prefix, flags):
    stamp = out + ".stamp"
    key = _hash([src] + deps, cmd_prefix + flags)
    if os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == key:
        return False
    os.makedirs(os.path.dirname(out), exist_ok=True)
    _run(cmd_prefix + flags + ["-c", src, "-o", out])
    with open(stamp, "w") as f:
        f.write(key)
    return True


def _link(objs, out, cmd):
    stamp = out + ".stamp"
    key = _hash(objs, cmd)
    if os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == key:
        return False
    tmp = out + ".tmp"
    _run(cmd + objs + ["-o", tmp])
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(key)
    return True


def build(hip: bool = True, rt: bool = True, jobs: int | None = None) -> dict:
    """Build (incrementally) and return {'hip': path|None, 'rt': path|None}."""
    inc, torch_lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    jobs = jobs or min(8, os.cpu_count() or 4)
    os.makedirs(LIB_DIR, exist_ok=True)
    torch_flags = ["-std=c++17", "-O2", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__",
                   "-DUSE_ROCM", "-DTORCH_EXTENSION_NAME=dmlc", f"-I{ROCM}/include", f"-I{py_inc}"]
    torch_flags += [f"-I{p}" for p in inc]
    torch_link = [f"-L{torch_lib}", f"-Wl,-rpath,{torch_lib}", "-lc10", "-ltorch_cpu", "-ltorch"]
    headers = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    out = {"hip": None, "rt": None}
    jobs_list = []
    hip_objs, rt_objs = [], []
    if hip:
        hipcc = os.path.join(ROCM, "bin", "hipcc")
        hip_flags = ["-std=c++17", "-O3", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
        if TIMING:   # the stamp buffer is one __device__ symbol shared by every kernel TU
            hip_flags += ["-DDMLC_TIMING", "-fgpu-rdc"]
        hip_flags += VARIANT_FLAGS
        for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
            o = os.path.join(OBJ_DIR, os.path.basename(src) + (f"{_SUFFIX.replace('_', '.')}.o" if _SUFFIX else ".o"))
            hip_objs.append(o)
            jobs_list.append((src, headers, o, [hipcc], hip_flags))
        bheaders = headers + glob.glob(os.path.join(CSRC, "bindings", "*.h"))
        for bsrc in sorted(glob.glob(os.path.join(CSRC, "bindings", "*.cpp"))):
            o = os.path.join(OBJ_DIR, os.path.basename(bsrc) + ".o")
            hip_objs.append(o)
            jobs_list.append((bsrc, bheaders, o, ["g++"], torch_flags))
    if rt:
        rt_headers = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
        import pybind11
        rt_flags = ["-std=c++17", "-O3", "-fPIC", "-fvisibility=hidden", f"-I{py_inc}",
                    f"-I{pybind11.get_include()}"]
        for src in sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))):
            o = os.path.join(OBJ_DIR, "rt_" + os.path.basename(src) + ".o")
            rt_objs.append(o)
            jobs_list.append((src, rt_headers, o, ["g++"], rt_flags))
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, *j) for j in jobs_list]
        for f in futs:
            f.result()
    if hip:
        hipcc = os.path.join(ROCM, "bin", "hipcc")
        _link(hip_objs, HIP_LIB, [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}"]
              + (["-fgpu-rdc"] if TIMING else []) + torch_link
              + [f"-L{torch_lib}", "-lc10_hip", "-ltorch_hip"])
        out["hip"] = HIP_LIB
    if rt and rt_objs:
        _link(rt_objs, RT_LIB, ["g++", "-shared", "-fPIC", "-pthread"])
        out["rt"] = RT_LIB
    return out


def clean():
    shutil.rmtree(OBJ_DIR, ignore_errors=True)
    shutil.rmtree(LIB_DIR, ignore_errors=True)


if __name__ == "__main__":
    if "--clean" in sys.argv:
        clean()
    print(build())
