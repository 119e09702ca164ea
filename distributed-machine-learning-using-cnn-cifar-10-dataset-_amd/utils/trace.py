"""Tracing / profiling hooks (SURVEY.md §5.1 — the reference has none).

* ``--trace roctx``: named ranges around every phase of the training loop (step, log, eval, ckpt)
  through ``torch.cuda.nvtx``, which PyTorch-ROCm routes to roctx, so ``rocprofv3 --marker-trace``
  shows the step structure next to the kernel trace.  Costs one host call per range.
* ``--trace torch``: a ``torch.profiler`` window of ``trace_steps`` steps (after a 5-step warm-up),
  exported as a Chrome trace into ``log_dir`` -- host launch overhead, graph replays, collectives.
Per-kernel device time comes from ``rocprofv3 --kernel-trace --stats``; per-phase time INSIDE the
fused kernels from the DMLC_TIMING build (tools/ktiming.py).
"""
from __future__ import annotations

import contextlib
import os

import torch


class Tracer:
    def __init__(self, mode: str = "", log_dir: str = "", steps: int = 20, rank: int = 0):
        self.mode = mode
        self.roctx = mode == "roctx" and torch.cuda.is_available()
        self.prof = None
        self.window = (5, 5 + steps)
        self.log_dir = log_dir
        self.rank = rank
        self.n = 0

    @contextlib.contextmanager
    def range(self, name: str):
        if self.roctx:
            torch.cuda.nvtx.range_push(name)
            try:
                yield
            finally:
                torch.cuda.nvtx.range_pop()
        else:
            yield

    def step_done(self):
        """Call once per training step (drives the torch.profiler window)."""
        if self.mode != "torch":
            return
        self.n += 1
        if self.n == self.window[0] and self.prof is None:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.prof = torch.profiler.profile(activities=acts)
            self.prof.__enter__()
        elif self.n == self.window[1] and self.prof is not None:
            self.close()

    def close(self):
        if self.prof is not None:
            self.prof.__exit__(None, None, None)
            if self.log_dir:
                os.makedirs(self.log_dir, exist_ok=True)
                self.prof.export_chrome_trace(os.path.join(self.log_dir, f"trace_rank{self.rank}.json"))
            self.prof = None
