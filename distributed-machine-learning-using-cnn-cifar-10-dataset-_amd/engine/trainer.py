"""Training session: the reference's ``main()`` (/root/reference/cifar10cnn.py:179-242) rebuilt around
synchronous data parallelism, the fused MI355X engine and explicit hooks.

Hook semantics follow what TF1's MonitoredTrainingSession gave the reference (SURVEY.md §3.2, §3.5,
§5.1-§5.5):
  * StopAtStepHook(last_step=generations): stop once global_step >= last_step (absolute, so a
    resumed run finishes at the same step; :219);
  * chief-only checkpoint saver: at session start, every ``checkpoint_secs`` and at the end,
    ``max_to_keep`` newest kept; restore of the latest checkpoint at start-up (:222);
  * chief step counter: ``global_step/sec`` into the events file every 100 steps;
  * console lines kept verbatim: ``Starting Training``, ``global_step %s, task:%d_step %d, training
    accuracy %g`` every ``output_every`` local iterations (:232-235) and `` --- Test Accuracy =
    {:.2f}%.`` every ``eval_every`` (:237-241).
Reference defects fixed: D1 the eval actually evaluates the test set; D2 one
authoritative global_step shared by all ranks; D3 the staircase LR decays with global_step
(``--lr_schedule=constant`` reproduces the reference as run); D6 every rank trains on a disjoint
shard of each epoch's permutation; D11 the printed training accuracy is that of the batch just
trained on (fused into the loss kernel) instead of an extra forward pass on a fresh batch.
"""
from __future__ import annotations

import math
import os
import sys
import time
from typing import Dict, Optional

import torch

from .. import checkpoint as CK
from .. import config as C
from ..parallel import dist as D
from ..parallel import health as H
from ..utils.events import EventsWriter, MetricsLog
from ..utils.trace import Tracer


EXIT_COMM_FAILURE = H.EXIT_COMM_FAILURE   # a peer stopped participating / no device progress / replicas diverged


class CommFailure(RuntimeError):
    """The gradient exchange can no longer complete (dead peer, stalled collective)."""


# --- engine adapters: one interface over the fused HIP engine and the eager torch engine ------------
class _FusedAdapter:
    kind = "fused"
    TUNE_ITERS = 20

    def __init__(self, cfg: C.TrainConfig, info: D.DistInfo, data, labels):
        from .fused import FusedCifarEngine
        self.eng = FusedCifarEngine(cfg.batch_size, data, labels, device=info.device, world_size=info.world_size,
                                    rank=max(0, info.rank), seed=cfg.seed, lr=C.effective_lr(cfg, info.world_size), warmup_steps=cfg.warmup_steps,
                                    lr_decay=cfg.lr_decay, decay_steps=cfg.num_gens_to_wait,
                                    staircase=cfg.lr_schedule == "staircase", relu_logits=cfg.relu_logits,
                                    crop_offset=((32 - cfg.crop) // 2,) * 2, comm_dtype=cfg.comm_dtype,
                                    dtype=cfg.dtype, allreduce=cfg.allreduce,
                                    dp_schedule="serial" if cfg.dp_schedule == "auto" else cfg.dp_schedule)
        self.cfg = cfg
        self.graph = cfg.graph
        from ..models import cifar_cnn as M
        self.specs = M.PARAM_SPECS

    def start(self, log=print):
        """Before the loop: one eager step (lazy code-object load, LDS attributes), then capture the
        step and its chains.  With --dp_schedule=auto and enough steps left, both DP schedules are
        timed on real training steps (max over ranks: one decision everywhere) and the faster kept."""
        if not self.graph or self.cfg.generations <= self.global_step:
            return
        self.eng.step()
        self.eng.capture(self.cfg.steps_per_graph)
        windows = 4 * (self.TUNE_ITERS + self.cfg.steps_per_graph)
        if (self.cfg.dp_schedule == "auto" and self.eng.dp and hasattr(self.eng, "tune_schedule")
                and self.cfg.generations - self.global_step >= 10 * windows):
            self.eng.tune_schedule(iters=self.TUNE_ITERS, steps_per_graph=self.cfg.steps_per_graph, log=log)

    def run(self, n: int):
        """``n`` training steps, as chained graph replays once captured (asynchronous)."""
        if self.eng.graphs:
            self.eng.run(n)
        else:
            for _ in range(n):
                self.eng.step()

    def step(self):
        self.run(1)

    def device_event(self):
        # the wgrad barrier error word rides along with every chunk (pinned copy, no sync)
        if hasattr(self.eng, "queue_error_copy"):
            self.eng.queue_error_copy()
        ev = torch.cuda.Event()
        ev.record()
        return ev

    def check_comm(self):
        # a timed-out wgrad sub-grid barrier is not a peer failure (a restart would repeat it): a plain
        # RuntimeError, raised before anything (e.g. a checkpoint) can use the step's weights
        # (the engine's message names the kernel whose wait timed out and the switch that turns it off)
        if hasattr(self.eng, "check_barriers"):
            self.eng.check_barriers(cached=True)
        try:
            if getattr(self.eng, "xgmi", None) is not None:
                self.eng.xgmi.check()
        except RuntimeError as e:
            raise CommFailure(str(e)) from e

    @property
    def global_step(self) -> int:
        return self.eng.host_step

    def stats(self) -> Dict[str, float]:
        st = self.eng.read_stats(self.eng.host_step)     # (a device sync: the error word is current too)
        if hasattr(self.eng, "check_barriers"):
            # a persistent launch's wait that timed out (its blocks were not co-resident) leaves wrong
            # weights: stop loudly (the message names the kernel and its off switch)
            self.eng.check_barriers()
        return st

    def tf_tensors(self) -> Dict[str, torch.Tensor]:
        return CK.model_tensors(self.eng.flat_params(), self.eng.host_step, 0, specs=self.specs)

    def load_tf_tensors(self, tensors):
        flat, step, _ = CK.load_model_tensors(tensors, flat_size=self.eng.master.numel(), specs=self.specs)
        self.eng.load_flat_params(flat, step)

    def broadcast_from_chief(self, info):
        """Every rank adopts rank 0's parameters and global_step (after a chief-only restore)."""
        step = torch.tensor([self.eng.host_step], dtype=torch.int64, device=self.eng.device)
        D.broadcast_(self.eng.master, info)
        D.broadcast_(step, info)
        self.eng.set_step(int(step.item()))
        self.eng.refresh_shadows()

    def evaluate(self, x, y, max_batches=0) -> float:
        return self.eng.evaluate(x, y, max_batches)

    def sync(self):
        torch.cuda.synchronize(self.eng.device)

    def param_checksum(self) -> torch.Tensor:
        return H.replica_checksum(self.eng.master)

    def perturb_replica(self):            # fault injection (DMLC_FAULT_MODE=diverge)
        self.eng.master[0] += 1e-3


class _FusedResNetAdapter(_FusedAdapter):
    """ResNet-20 on the fused HIP engine (engine/fused_resnet.py): parameters + BN moving statistics
    checkpointed under the same names as the eager model."""

    def __init__(self, cfg: C.TrainConfig, info: D.DistInfo, data, labels):
        from .fused_resnet import FusedResNetEngine
        from ..models import resnet as R
        self.eng = FusedResNetEngine(cfg.batch_size, data, labels, device=info.device, world_size=info.world_size,
                                     rank=max(0, info.rank), seed=cfg.seed, lr=C.effective_lr(cfg, info.world_size), warmup_steps=cfg.warmup_steps,
                                     lr_decay=cfg.lr_decay, decay_steps=cfg.num_gens_to_wait,
                                     staircase=cfg.lr_schedule == "staircase", comm_dtype=cfg.comm_dtype,
                                     allreduce=cfg.allreduce)
        self.cfg = cfg
        self.graph = cfg.graph
        self.specs, self.state_specs = R.PARAM_SPECS, R.STATE_SPECS

    def tf_tensors(self) -> Dict[str, torch.Tensor]:
        d = CK.model_tensors(self.eng.flat_params(), self.eng.host_step, 0, specs=self.specs)
        st = self.eng.state.detach().cpu()
        d.update({s.name: st[s.offset:s.offset + s.numel].view(s.shape).clone() for s in self.state_specs})
        return d

    def load_tf_tensors(self, tensors):
        flat, step, _ = CK.load_model_tensors(tensors, flat_size=self.eng.master.numel(), specs=self.specs)
        state = torch.zeros_like(self.eng.state, device="cpu")
        for s in self.state_specs:
            if s.name not in tensors:
                raise KeyError(f"checkpoint is missing {s.name}")
            state[s.offset:s.offset + s.numel] = tensors[s.name].float().reshape(-1)
        self.eng.load_flat_params(flat, step, state=state)

    def broadcast_from_chief(self, info):
        D.broadcast_(self.eng.state, info)
        super().broadcast_from_chief(info)


class _EagerAdapter:
    kind = "eager"

    def __init__(self, cfg: C.TrainConfig, info: D.DistInfo, data, labels, backend: str = "torch"):
        from .eager import EagerTrainer
        self.tr = EagerTrainer(cfg.model, cfg.batch_size, data, labels, device=info.device,
                               world_size=info.world_size, rank=max(0, info.rank), dtype=cfg.dtype,
                               lr=C.effective_lr(cfg, info.world_size), warmup_steps=cfg.warmup_steps, lr_decay=cfg.lr_decay, decay_steps=cfg.num_gens_to_wait,
                               staircase=cfg.lr_schedule == "staircase", relu_logits=cfg.relu_logits,
                               crop=cfg.crop, seed=cfg.seed, augment=cfg.augment, backend=backend,
                               graph=backend == "hip_f32" and cfg.graph and info.world_size == 1)
        self.specs = self.tr.model.specs

    def start(self, log=print):
        pass

    def run(self, n: int):
        for _ in range(n):
            self.tr.step()

    def step(self):
        self.tr.step()

    def device_event(self):
        if self.tr.device.type != "cuda":
            return None
        ev = torch.cuda.Event()
        ev.record()
        return ev

    def check_comm(self):
        pass

    @property
    def global_step(self) -> int:
        return self.tr.global_step

    def stats(self) -> Dict[str, float]:
        return {"global_step": self.tr.global_step, "loss": float(self.tr.last_loss),
                "accuracy": float(self.tr.last_acc), "lr": self.tr.lr(self.tr.global_step - 1)}

    def tf_tensors(self) -> Dict[str, torch.Tensor]:
        return CK.module_tensors(self.tr.model, self.tr.global_step, 0)

    def load_tf_tensors(self, tensors):
        self.tr.global_step = CK.load_module_tensors(self.tr.model, tensors)

    def broadcast_from_chief(self, info):
        dev = info.device if info.backend == "nccl" else torch.device("cpu")
        m = self.tr.model
        bufs = [m.flat.data] + ([m.state] if hasattr(m, "state") else [])
        step = torch.tensor([self.tr.global_step], dtype=torch.int64)
        for b in bufs + [step]:
            t = b.to(dev)
            D.broadcast_(t, info)
            b.copy_(t.to(b.device))
        self.tr.global_step = int(step.item())

    def evaluate(self, x, y, max_batches=0) -> float:
        return self.tr.evaluate(x, y, max_batches)

    def sync(self):
        if self.tr.device.type == "cuda":
            torch.cuda.synchronize(self.tr.device)

    def param_checksum(self) -> torch.Tensor:
        return H.replica_checksum(self.tr.model.flat)

    def perturb_replica(self):            # fault injection (DMLC_FAULT_MODE=diverge)
        with torch.no_grad():
            self.tr.model.flat.data[0] += 1e-3


def pick_impl(cfg: C.TrainConfig, device: torch.device) -> str:
    if cfg.impl != "auto":
        return cfg.impl
    if (device.type == "cuda" and cfg.model == "cifar_cnn" and cfg.dtype in ("bf16", "fp8") and cfg.crop == 24
            and not cfg.augment):
        return "fused"                    # any batch size: masked tail rows (engine/fused.py)
    if device.type == "cuda" and cfg.model == "cifar_cnn" and cfg.dtype == "fp32":
        return "hipf32"                   # reference precision on the fp32 HIP kernels (ops/f32.py)
    if (device.type == "cuda" and cfg.model == "resnet20" and cfg.dtype == "bf16" and cfg.crop == 32
            and not cfg.augment):
        return "fused"                    # any batch size: padding images masked out of BN (resnet.hip)
    return "eager"


def _fault_step() -> Optional[int]:
    """Test hook: DMLC_FAULT_STEP / DMLC_FAULT_RANK kill this rank hard at a step,
    on the first attempt only (DMLC_RESTART_COUNT is set by the launcher)."""
    fs = os.environ.get("DMLC_FAULT_STEP")
    if fs is None or int(os.environ.get("DMLC_RESTART_COUNT", "0")) > 0:
        return None
    return int(fs)


def _fault_injection(step: int, rank: int, engine=None):
    """DMLC_FAULT_MODE: ``exit`` (default; the process dies, exit 17), ``stop`` (SIGSTOP: alive but
    silent -- only the heartbeat can detect it), ``diverge`` (this rank's replica is perturbed: the
    replica check must catch it)."""
    fs = _fault_step()
    if fs is not None and step == fs and rank == int(os.environ.get("DMLC_FAULT_RANK", "0")):
        mode = os.environ.get("DMLC_FAULT_MODE", "exit")
        if mode == "stop":
            print(f"[fault-injection] rank {rank} stopping (SIGSTOP) at global_step {step}", flush=True)
            import signal
            os.kill(os.getpid(), signal.SIGSTOP)
        elif mode == "diverge" and engine is not None:
            print(f"[fault-injection] rank {rank} perturbing its replica at global_step {step}", flush=True)
            engine.perturb_replica()
        else:
            print(f"[fault-injection] rank {rank} exiting at global_step {step}", flush=True)
            os._exit(17)


class Session:
    """One worker's training session."""

    def __init__(self, cfg: C.TrainConfig, info: D.DistInfo, log=print):
        self.cfg, self.info, self.log = cfg, info, log
        self.chief = info.rank == 0
        self._replica_checks = 0
        tr_x, tr_y, te_x, te_y = _load_data(cfg, info)
        self.test = (te_x, te_y)
        impl = pick_impl(cfg, info.device)
        fused = _FusedResNetAdapter if cfg.model == "resnet20" else _FusedAdapter
        if impl == "fused":
            self.engine = fused(cfg, info, tr_x, tr_y)
        else:
            self.engine = _EagerAdapter(cfg, info, tr_x, tr_y, backend="hip_f32" if impl == "hipf32" else "torch")
        self.impl = impl
        self.ckpt = None
        self.events = None
        self.metrics = MetricsLog(None)
        self.tracer = Tracer(cfg.trace, cfg.log_dir, cfg.trace_steps, max(0, info.rank))
        if self.chief and cfg.log_dir:
            if cfg.save_checkpoints:
                self.ckpt = CK.CheckpointManager(
                    cfg.log_dir, cfg.max_to_keep, cfg.checkpoint_secs,
                    graph_info=dict(model=cfg.model, batch=cfg.batch_size, crop=cfg.crop, relu_logits=cfg.relu_logits))
            self.events = EventsWriter(cfg.log_dir)
            self.metrics = MetricsLog(cfg.metrics_file or os.path.join(cfg.log_dir, "metrics.jsonl"))

    # --- checkpoint --------------------------------------------------------------------------------
    def restore(self) -> int:
        """Chief loads the latest checkpoint in log_dir (if any); every rank then adopts the chief's
        parameters and global_step (one authoritative step counter, D2)."""
        if self.chief and self.cfg.log_dir:
            path = CK.latest_checkpoint(self.cfg.log_dir)
            if path:
                self.engine.load_tf_tensors(CK.read_bundle(path))
                self.log(f"Restored {path} (global_step {self.engine.global_step})")
        if self.info.world_size > 1:
            self.engine.broadcast_from_chief(self.info)
        return self.engine.global_step

    def save(self, force=False):
        if self.ckpt is not None and (force or self.ckpt.due()):
            self.ckpt.save(self.engine.global_step, self.engine.tf_tensors())

    # --- main loop -----------------------------------------------------------------------------------
    def _chunk(self, gs: int, i: int) -> int:
        """Steps until the next host-side event: an output / eval point (local iteration counts, as in
        the reference), the StopAtStep target, a fault-injection step; 1 under a torch.profiler
        window (it counts steps)."""
        cfg = self.cfg
        n = min(cfg.generations - gs, cfg.output_every - i % cfg.output_every, cfg.eval_every - i % cfg.eval_every)
        fs = _fault_step()
        if fs is not None and gs < fs:
            n = min(n, fs - gs)
        if cfg.trace == "torch":
            n = 1
        return max(1, n)

    def _wait_progress(self, ev):
        """Device progress watchdog: the previous chunk must finish within the process-group timeout.
        Collectives captured inside a graph are invisible to the process group's own watchdog, and a
        stalled one would otherwise hold this rank forever; an xGMI barrier that timed out has set the
        engine's error word, which check_comm() turns into a CommFailure."""
        if ev is None:
            return
        deadline = time.time() + self.cfg.pg_timeout_s
        while not ev.query():
            if time.time() > deadline:
                raise CommFailure(f"no device progress for {self.cfg.pg_timeout_s:.0f} s "
                                  f"(rank {self.info.rank}, global_step ~{self.engine.global_step})")
            time.sleep(0.0002)
        self.engine.check_comm()

    def _allreduce_path(self) -> str:
        info = getattr(getattr(self.engine, "eng", None), "comm_info", None) or {}
        return str(info.get("allreduce", self.info.backend))

    def _check_replicas(self):
        """Every synchronous replica must hold bit-identical parameters (parallel/health.py)."""
        if self.info.world_size <= 1 or not self.cfg.check_replicas or not hasattr(self.engine, "param_checksum"):
            return
        cs = self.engine.param_checksum()
        dev = self.info.device if self.info.backend == "nccl" else torch.device("cpu")
        self._replica_checks += 1
        if not H.replicas_agree(cs, device=dev):
            # the all-reduce this run actually used (xgmi / rccl / gloo ...), not the flag value
            marker = H.mark_divergence(self.cfg.log_dir, f"rank {self.info.rank} global_step {self.engine.global_step} "
                                                        f"allreduce={self._allreduce_path()}")
            raise CommFailure(f"replica divergence at global_step {self.engine.global_step} "
                              f"(marker {marker}: the next start uses --allreduce=rccl)")

    def run(self) -> Dict[str, float]:
        cfg, eng = self.cfg, self.engine
        self.restore()
        self.save(force=True)            # CheckpointSaverHook.after_create_session
        # the pre-capture step of start() is a real training step: it is fault-injectable and
        # counts as a local iteration (i below), like every other step
        start = eng.global_step
        _fault_injection(eng.global_step, self.info.rank, eng)
        eng.start(log=self.log)
        self.log(f"[dmlc] engine={self.impl} model={cfg.model} dtype={cfg.dtype} batch={cfg.batch_size} "
                 f"world={self.info.world_size} device={self.info.device}")
        self.log("Starting Training")
        last_t, last_step = time.time(), eng.global_step
        result = {}
        pending = None
        while eng.global_step < cfg.generations:        # StopAtStepHook(last_step=GENERATIONS)
            _fault_injection(eng.global_step, self.info.rank, eng)
            i = eng.global_step - start                  # local iterations so far (the reference's i)
            n = self._chunk(eng.global_step, i)
            with self.tracer.range("steps"):
                eng.run(n)
            self.tracer.step_done()
            ev = eng.device_event()
            self._wait_progress(pending)                 # one chunk in flight behind the host
            pending = ev
            i += n
            if i % cfg.output_every == 0:
                self._wait_progress(pending)
                with self.tracer.range("stats"):
                    st = eng.stats()
                now = time.time()
                steps = eng.global_step - last_step
                ips = steps * cfg.batch_size * self.info.world_size / max(1e-9, now - last_t)
                self.log("global_step %s, task:%d_step %d, training accuracy %g"
                         % (eng.global_step, cfg.task_index, i - 1, st["accuracy"]))
                self.metrics.write(step=eng.global_step, loss=st["loss"], accuracy=st["accuracy"], lr=st["lr"],
                                   images_per_sec=ips, step_ms=1000.0 * (now - last_t) / max(1, steps))
                if self.events is not None:
                    self.events.scalars(eng.global_step, {"global_step/sec": steps / max(1e-9, now - last_t),
                                                          "loss": st["loss"], "accuracy": st["accuracy"],
                                                          "learning_rate": st["lr"]})
                last_t, last_step = now, eng.global_step
                result = dict(st, images_per_sec=ips)
                self._check_replicas()
            if i % cfg.eval_every == 0:
                self._wait_progress(pending)
                with self.tracer.range("eval"):
                    acc = eng.evaluate(*self.test, max_batches=cfg.eval_batches)
                self.log(" --- Test Accuracy = {:.2f}%.".format(100.0 * acc))
                self.metrics.write(step=eng.global_step, test_accuracy=acc)
                result["test_accuracy"] = acc
                last_t = time.time()                      # eval time is not training throughput
            if self.ckpt is not None and self.ckpt.due():
                self._wait_progress(pending)             # never save weights of a broken exchange
                with self.tracer.range("checkpoint"):
                    self.save()
        # the watchdog first: a collective captured in the last chunk that stalls on a dead peer must
        # become a CommFailure (exit 75), not a rank blocked forever inside synchronize()
        self._wait_progress(pending)
        eng.sync()
        eng.stats()                      # also checks the device error words once more
        self._check_replicas()
        if self._replica_checks and self.info.rank == 0 and self._allreduce_path() == "xgmi":
            H.clear_divergence(self.cfg.log_dir)   # the xGMI path passed every replica check again
        self.tracer.close()
        self.save(force=True)            # CheckpointSaverHook.end
        result["global_step"] = eng.global_step
        if self.events is not None:
            self.events.close()
        self.metrics.close()
        return result


def _load_data(cfg: C.TrainConfig, info: D.DistInfo):
    from ..data import dataset
    return dataset(cfg, is_chief=info.rank == 0, barrier=lambda: D.barrier(info))


def main(argv=None) -> int:
    """CLI entry (``python cifar10cnn.py ...`` / ``python -m dmlc.train ...``)."""
    from .. import cli
    cfg, _unparsed = cli.parse(argv)
    role = cli.resolve_role(cfg)
    if role.kind == "none":
        return 0                          # unknown --job_name: the reference silently did nothing
    if role.kind == "ps":
        return D.serve_ps(role, log=lambda m: print(m, flush=True))
    if cfg.allreduce == "auto" and H.divergence_marked(cfg.log_dir):
        print(f"[dmlc] {os.path.join(cfg.log_dir, H.DIVERGENCE_MARKER)} exists (replicas diverged in an earlier "
              "run): using --allreduce=rccl", flush=True)
        cfg = cfg.replace(allreduce="rccl")
    info = D.init(D.role_info(role), device=cfg.device, timeout_s=cfg.pg_timeout_s, rccl_channels=cfg.rccl_channels)
    hb = None
    if info.world_size > 1 and cfg.heartbeat_timeout_s > 0:
        hb = H.Heartbeat(info.rank, info.world_size, info.master_addr, info.master_port,
                         interval_s=cfg.heartbeat_s, timeout_s=cfg.heartbeat_timeout_s).start()
    try:
        sess = Session(cfg, info, log=lambda m: print(m, flush=True))
        res = sess.run()
        if hb is not None:
            hb.stop(done=True)
        if info.rank == 0:
            print(f"done: {res}", flush=True)
        D.report_done(info)
    except CommFailure as e:
        # fail fast: a dead peer must not leave this rank training on un-reduced gradients or
        # waiting forever in a collective; exit without the (collective) teardown, the launcher
        # restarts the world from the latest checkpoint (RecoverableSession, cifar10cnn.py:222)
        print(f"[dmlc] rank {info.rank}: gradient exchange failed: {e}; exiting for restart", flush=True)
        os._exit(EXIT_COMM_FAILURE)
    finally:
        D.shutdown(info)
    return 0


if __name__ == "__main__":
    sys.exit(main())
