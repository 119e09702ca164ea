"""Liveness heartbeat and replica-divergence check for the synchronous data-parallel world.

The reference inherits failure handling from TF1's gRPC runtime: a dead PS/worker surfaces as
``UnavailableError`` and ``MonitoredTrainingSession``'s ``_RecoverableSession`` re-creates the session
(/root/reference/cifar10cnn.py:222).  In synchronous DP one dead rank stalls every
collective, and a collective captured inside a HIP graph is invisible to the process group's own
watchdog, so two bounded detectors run beside training:

* :class:`Heartbeat` -- a daemon thread per rank bumps ``dmlc/hb/<rank>`` in the rendezvous TCPStore
  every ``interval_s`` (process liveness, independent of training progress: a rank blocked in a
  collective keeps beating) and watches every peer's counter.  A peer whose counter has not moved
  for ``timeout_s`` -- killed, SIGSTOPped, its host gone -- or a store that stops answering (the
  store host died) ends this rank with exit code 75 (``EXIT_COMM_FAILURE``), so survivors leave a
  stalled collective within ``timeout_s + interval_s`` instead of the 300 s process-group timeout,
  with or without the ``dmlc.launch`` supervisor (which then restarts the world from the latest
  checkpoint).  A rank that finishes cleanly marks ``dmlc/hb_done/<rank>`` first.
* :func:`replica_checksum` / :func:`replicas_agree` -- every replica must hold bit-identical
  parameters after each synchronous step (deterministic kernels, one all-reduced gradient); a
  two-word integer checksum of the fp32 parameter bits is compared across ranks with one MAX
  all-reduce.  A mismatch (e.g. a coherence bug in the custom xGMI all-reduce) is reported instead
  of training silently on divergent replicas.
"""
from __future__ import annotations

import datetime
import os
import sys
import threading
import time
from typing import Callable, Optional

import torch
import torch.distributed as dist

EXIT_COMM_FAILURE = 75
DIVERGENCE_MARKER = ".dmlc_replica_divergence"


class Heartbeat:
    """Per-rank liveness thread over a private TCPStore client (see module docstring)."""

    def __init__(self, rank: int, world_size: int, host: str, port: int, interval_s: float = 1.0,
                 timeout_s: float = 20.0, on_failure: Optional[Callable[[str], None]] = None,
                 prefix: str = "dmlc"):
        self.rank, self.world = int(rank), int(world_size)
        self.interval, self.timeout = float(interval_s), float(timeout_s)
        self.host, self.port, self.prefix = host, int(port), prefix
        self.on_failure = on_failure or _exit_comm_failure
        self.active = False
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._store = None
        self.failure: Optional[str] = None

    def _key(self, what: str, r: int) -> str:
        return f"{self.prefix}/{what}/{r}"

    def start(self) -> "Heartbeat":
        if self.world <= 1:
            return self
        # a client of its own: the process group's store connection is never shared across threads
        self._store = dist.TCPStore(self.host, self.port, None, is_master=False,
                                    timeout=datetime.timedelta(seconds=max(1.0, self.timeout)),
                                    wait_for_workers=False)
        self._store.add(self._key("hb", self.rank), 1)
        self.active = True
        self._thread = threading.Thread(target=self._loop, name="dmlc-heartbeat", daemon=True)
        self._thread.start()
        return self

    def _loop(self):
        st = self._store
        peers = [r for r in range(self.world) if r != self.rank]
        seen = {r: (-1, time.monotonic()) for r in peers}      # last counter value, when it last moved
        done = set()
        while not self._stop.wait(self.interval):
            try:
                st.add(self._key("hb", self.rank), 1)
                now = time.monotonic()
                for r in peers:
                    if r in done:
                        continue
                    if st.add(self._key("hb_done", r), 0) > 0:
                        done.add(r)
                        continue
                    v = st.add(self._key("hb", r), 0)
                    if v != seen[r][0]:
                        seen[r] = (v, now)
                    elif now - seen[r][1] > self.timeout:
                        self._fail(f"rank {r} silent for {now - seen[r][1]:.1f} s (heartbeat timeout "
                                   f"{self.timeout:.0f} s)")
                        return
            except Exception as e:                      # store host gone / unreachable
                if self._stop.is_set() or not self.active:
                    return
                if 0 in done:
                    # the store lives in rank 0's process (reference-CLI worlds) or beside it: rank 0
                    # marked itself finished, so its store going away is its clean exit, not a failure
                    # (this rank is about to finish too: its own collectives completed with rank 0's).
                    # Rank 0 itself gets no such exemption: a store hosted in its own process cannot
                    # vanish before stop() (which sets _stop first), so an unreachable store seen by
                    # rank 0 is one hosted elsewhere (a torchrun agent, the ps role) -- a real failure.
                    return
                self._fail(f"rendezvous store unreachable ({type(e).__name__}: {e})")
                return

    def _fail(self, why: str):
        if not self.active:
            return
        self.failure = why
        self.on_failure(f"rank {self.rank}: {why}")

    def stop(self, done: bool = True, wait_peers_s: Optional[float] = None):
        """Stop beating; ``done`` marks this rank finished so peers stop watching it.  Rank 0 then
        waits (bounded by ``wait_peers_s``, default the heartbeat timeout) until every peer has marked
        itself finished too: in reference-CLI worlds rank 0's process hosts the rendezvous store, and
        tearing it down under a slower peer's heartbeat would make that peer report a failure (exit
        75) for a run that succeeded."""
        if not self.active:
            return
        self.active = False
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2 * self.interval + 1.0)
        if not done or self._store is None:
            return
        try:
            self._store.add(self._key("hb_done", self.rank), 1)
        except Exception:
            return
        if self.rank != 0:
            return
        deadline = time.monotonic() + (self.timeout if wait_peers_s is None else float(wait_peers_s))
        pending = set(range(1, self.world))
        while pending and time.monotonic() < deadline:
            try:
                pending = {r for r in pending if self._store.add(self._key("hb_done", r), 0) == 0}
            except Exception:
                return
            if pending:
                time.sleep(min(0.05, self.interval))


def _exit_comm_failure(msg: str):
    print(f"[dmlc] {msg}; exiting for restart (code {EXIT_COMM_FAILURE})", flush=True)
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(EXIT_COMM_FAILURE)


_WEIGHTS = {}


def replica_checksum(t: torch.Tensor) -> torch.Tensor:
    """int64 [2] = (sum of the fp32 bit patterns, position-weighted sum) of ``t`` -- exact integer
    arithmetic: |bits| < 2^31 and position weights <= 2039 < 2^11 keep every product below 2^42,
    so the sums cannot overflow for up to 2^21 elements (the CNN has 1,068,298 parameters; past
    2^21 they wrap, identically on every rank, so equality still compares replicas).  Equal only
    for replicas that agree bit for bit up to an astronomically unlikely collision; catches value
    AND position (e.g. a shifted bucket) differences."""
    v = t.detach().contiguous().view(-1).view(torch.int32).to(torch.int64)
    key = (v.numel(), v.device)
    w = _WEIGHTS.get(key)
    if w is None:
        w = _WEIGHTS[key] = torch.arange(v.numel(), device=v.device, dtype=torch.int64) % 2039 + 1
    return torch.stack([v.sum(), (v * w).sum()])


def replicas_agree(checksum: torch.Tensor, group=None, device: Optional[torch.device] = None) -> bool:
    """One MAX all-reduce of (c, -c): every rank learns whether all ranks hold the same checksum."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return True
    dev = device if device is not None else checksum.device
    both = torch.cat([checksum, -checksum]).to(dev)
    dist.all_reduce(both, op=dist.ReduceOp.MAX, group=group)
    n = checksum.numel()
    return bool(torch.equal(both[:n], -both[n:]))


def mark_divergence(log_dir: str, info: str) -> Optional[str]:
    if not log_dir:
        return None
    os.makedirs(log_dir, exist_ok=True)
    p = os.path.join(log_dir, DIVERGENCE_MARKER)
    with open(p, "a") as f:
        f.write(f"{time.strftime('%Y-%m-%dT%H:%M:%S')} {info}\n")
    return p


def divergence_marked(log_dir: str) -> bool:
    """True when an earlier run in ``log_dir`` saw replicas diverge WHILE using the custom xGMI
    all-reduce (the one component a downgrade to RCCL can rule out).  Divergence under RCCL, the
    eager engine or fault injection is recorded too but forces nothing."""
    if not log_dir:
        return False
    p = os.path.join(log_dir, DIVERGENCE_MARKER)
    if not os.path.exists(p):
        return False
    with open(p) as f:
        return any("allreduce=xgmi" in line.split() for line in f)


def clear_divergence(log_dir: str) -> bool:
    """Remove the marker (a later xGMI run completed its replica checks cleanly)."""
    p = os.path.join(log_dir, DIVERGENCE_MARKER) if log_dir else ""
    if p and os.path.exists(p):
        os.remove(p)
        return True
    return False
