#!/usr/bin/env python3
"""What does a side-channel copy of the fc gradient bucket cost the single-GPU step when it runs
beside the wgrad launch?  ("a committed one-GPU probe showing that a
3.84 MB side-channel copy running beside k_wgrad costs <= 1 us/step".)

   python tools/side_copy_probe.py [--batch 256] [--steps 300] [--rounds 2]

The single-GPU step (conv12 | fc chain | wgrad+SGD) is graph-captured as usual; each variant forks a
side stream right after the fc chain launch -- the point where the fc bucket of a DP step is final --
and copies ``--mb`` MB of the fp32 master (the fc bucket's size by default) with hipMemcpyAsync on
that stream.  The copy is joined before the NEXT step's fc chain (its first reader in the
owner-computes design), so it may run beside the wgrad launch and the next conv12 forward, exactly
where an fc-bucket exchange would run.  Variants:
  none        no side stream (the single-GPU step)
  fork        fork + join only (the cost of the graph edges)
  d2d         device -> device on the same GPU (a blit kernel on the CUs: the CU-driven path RCCL and
              the xGMI kernel take)
  d2h         device -> pinned host (the SDMA engines: the CU-free path a graph's peer copies take);
              PCIe-bound, so its size is --d2h-mb (default 0.25 MB ~ 5 us of PCIe) -- it measures the
              interference of an SDMA stream with the step, not the link
  kern        the same bytes moved by a PyTorch elementwise kernel (dst = src * 1, hundreds of
              workgroups on the CUs) -- a kernel node instead of a memcpy node
  xgmi8       the xGMI exchange kernel (xgmi_allreduce.hip) on a one-rank context over the bucket,
              8 workgroups (one release/acquire pair each): the <= 8-workgroup P2P kernel of the
              round-5 review, its fixed cost beside the wgrad launch
  xgmi        the same with the launcher's default workgroup count
Prints one JSON line per measurement and a summary with the per-step delta against ``none``."""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dmlc  # noqa: E402,F401
from dmlc.engine.fused import FusedCifarEngine  # noqa: E402

_hip = None


def hip():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        _hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        _hip.hipHostFree.argtypes = [ctypes.c_void_p]
    return _hip


class SideCopyEngine(FusedCifarEngine):
    def __init__(self, *args, mode="none", nbytes=0, **kw):
        super().__init__(*args, **kw)
        self.mode, self.nbytes = mode, int(nbytes)
        self.side = torch.cuda.Stream(device=self.device)
        n4 = max(1, self.nbytes // 4)
        self.src = torch.empty(n4, dtype=torch.float32, device=self.device).normal_()
        self.dst = None
        self.host = ctypes.c_void_p()
        if mode == "d2d":
            self.dst = torch.empty_like(self.src)
        elif mode == "d2h":
            rc = hip().hipHostMalloc(ctypes.byref(self.host), self.nbytes, 0)
            assert rc == 0, rc
        elif mode == "kern":
            self.dst = torch.empty_like(self.src)
        elif mode.startswith("xgmi"):
            from dmlc.parallel.xgmi import XgmiAllReduce
            self.xg = XgmiAllReduce(n4, 0, 1)
            self.xg.buf.normal_()

    def _copy(self):
        if self.mode == "kern":
            torch.mul(self.src, 1.0, out=self.dst)
            return
        if self.mode.startswith("xgmi"):
            self.xg.all_reduce(0, self.xg.numel, blocks=8 if self.mode == "xgmi8" else 0)
            return
        s = ctypes.c_void_p(self.side.cuda_stream)
        if self.mode == "d2d":
            rc = hip().hipMemcpyAsync(ctypes.c_void_p(self.dst.data_ptr()), ctypes.c_void_p(self.src.data_ptr()),
                                      self.nbytes, 3, s)
        else:
            rc = hip().hipMemcpyAsync(self.host, ctypes.c_void_p(self.src.data_ptr()), self.nbytes, 2, s)
        assert rc == 0, rc

    def _eager_step_body(self):
        if self.mode == "none":
            return super()._eager_step_body()
        assert not self.dp and self.fc1_epilogue and self.wgrad_apply, "probe of the single-GPU step only"
        main = torch.cuda.current_stream(self.device)
        self._forward(self.bidx, None, 1, train=True)
        self._join_comm()                       # last step's copy: joined before this fc chain
        self._fc_backward(fused_sgd=True)
        ev = torch.cuda.Event()
        ev.record(main)
        self.side.wait_event(ev)
        if self.mode != "fork":
            with torch.cuda.stream(self.side):
                self._copy()
        done = torch.cuda.Event()
        done.record(self.side)
        self._conv_backward(apply=True)
        self._pending_comm = done

    def close(self):
        if getattr(self, "xg", None) is not None:
            self.xg.check()
            self.xg.close()
            self.xg = None
        if self.host.value:
            hip().hipHostFree(self.host)
            self.host = ctypes.c_void_p()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--mb", type=float, default=3.84)
    ap.add_argument("--d2h-mb", type=float, default=0.25)
    ap.add_argument("--variants", default="none,fork,d2d,d2h,kern,xgmi8,xgmi")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (50000,), dtype=torch.int32, generator=g)
    names = a.variants.split(",")
    best = {}
    for r in range(a.rounds):
        for name in (names if r % 2 == 0 else names[::-1]):
            nb = int((a.d2h_mb if name == "d2h" else a.mb) * 1e6) // 16 * 16
            eng = SideCopyEngine(a.batch, data, labels, device="cuda:0", lr=1e-4, relu_logits=False,
                                 mode=name, nbytes=nb)
            eng.step()
            eng.capture(steps_per_graph=32)
            eng.run(256)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(a.steps)
            torch.cuda.synchronize()
            us = 1e6 * (time.perf_counter() - t0) / a.steps
            eng.check_barriers()
            assert torch.isfinite(eng.master).all()
            best[name] = min(best.get(name, 1e30), us)
            print(json.dumps({"variant": name, "round": r, "bytes": nb if name != "none" and name != "fork" else 0,
                              "us_per_step": round(us, 2)}), flush=True)
            eng.close()
            del eng
            torch.cuda.empty_cache()
    print(json.dumps({"batch": a.batch, "steps": a.steps, "min_us_per_step": {k: round(v, 2) for k, v in best.items()},
                      "delta_vs_none_us": {k: round(v - best["none"], 2) for k, v in best.items()}
                      if "none" in best else {}}), flush=True)


if __name__ == "__main__":
    main()
