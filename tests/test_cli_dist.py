"""CLI compatibility, role mapping, gloo data-parallel equivalence, the reference's ps/worker recipe,
and launcher fault injection + resume ('Distributed (fake cluster)', §5.3, §5.6)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from dmlc import checkpoint as CK
from dmlc import cli
from dmlc.config import TrainConfig

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENTRY = os.path.join(REPO, "cifar10cnn.py")


# ---- flags ----------------------------------------------------------------------------------------
def test_reference_flags_and_defaults():
    cfg, rest = cli.parse([])
    # cifar10cnn.py:249-272 defaults
    assert (cfg.ps_hosts, cfg.worker_hosts, cfg.job_name, cfg.task_index) == ("", "", "", 0)
    assert cfg.data_dir == "/tmp/mnist_data" and cfg.log_dir == "/tmp/train_logs"
    # cifar10cnn.py:9-27 constants
    assert (cfg.batch_size, cfg.generations, cfg.learning_rate, cfg.lr_decay, cfg.num_gens_to_wait) == \
        (128, 20000, 0.1, 0.9, 250.0)
    assert (cfg.output_every, cfg.eval_every, cfg.crop) == (200, 500, 24)
    cfg, rest = cli.parse(["--ps_hosts=localhost:2222", "--worker_hosts=localhost:2223,localhost:2224",
                           "--job_name=worker", "--task_index=1", "--some_tf_flag=3", "--log_dir", "/x"])
    assert cfg.task_index == 1 and cfg.log_dir == "/x" and rest == ["--some_tf_flag=3"]


def test_bool_flags():
    cfg, _ = cli.parse(["--relu_logits=false", "--synthetic"])
    assert cfg.relu_logits is False and cfg.synthetic is True
    with pytest.raises(SystemExit):
        cli.parse(["--relu_logits=maybe"])


def test_dp_schedule_flag():
    assert cli.parse([])[0].dp_schedule == "auto"
    assert cli.parse(["--dp_schedule=overlap"])[0].dp_schedule == "overlap"
    assert cli.parse(["--dp_schedule=serial"])[0].dp_schedule == "serial"
    assert cli.parse(["--steps_per_graph=4"])[0].steps_per_graph == 4
    with pytest.raises(SystemExit):
        cli.parse(["--dp_schedule=ring"])


def test_allreduce_flag():
    assert cli.parse([])[0].allreduce == "auto"
    assert cli.parse(["--allreduce=xgmi"])[0].allreduce == "xgmi"
    with pytest.raises(SystemExit):
        cli.parse(["--allreduce=mpi"])


def test_xgmi_selection_is_rccl_without_gpu():
    """CPU / world 1: the selector never builds the IPC path (no device kernels off-GPU)."""
    from dmlc.parallel import xgmi
    ar, info = xgmi.select(1024, 0, 1, torch.device("cpu"), [(0, 1024)])
    assert ar is None and info["allreduce"] == "rccl"


def test_xgmi_selection_falls_back_when_self_test_raises(monkeypatch):
    """A self-test that raises (a first cross-GPU mapping problem) selects RCCL on every rank instead
    of leaving the collective (gloo world 1 stands in for the group; the IPC context is a stub)."""
    import torch.distributed as dist
    from dmlc.cli import free_port
    from dmlc.parallel import xgmi

    class Stub:
        closed = False

        def __init__(self, *a, **k):
            pass

        def self_test(self):
            raise RuntimeError("hipErrorIllegalAddress")

        def close(self):
            Stub.closed = True

    monkeypatch.setattr(xgmi, "XgmiAllReduce", Stub)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
    try:
        ar, info = xgmi.select(1024, 0, 2, torch.device("cuda", 0), [(0, 1024)])
    finally:
        dist.destroy_process_group()
    assert ar is None and info["allreduce"] == "rccl" and Stub.closed
    assert "self-test raised RuntimeError" in info["xgmi_unavailable"]


def test_role_mapping():
    base = dict(ps_hosts="localhost:2222", worker_hosts="localhost:2223,localhost:2224,otherhost:2225")
    r = cli.resolve_role(TrainConfig(job_name="worker", task_index=1, **base), env={})
    assert (r.kind, r.rank, r.world_size, r.local_rank) == ("worker", 1, 3, 1)
    assert (r.master_addr, r.master_port, r.store_is_ps) == ("127.0.0.1", 2222, True)
    r = cli.resolve_role(TrainConfig(job_name="worker", task_index=2, **base), env={})
    assert r.local_rank == 0                      # first worker on otherhost
    r = cli.resolve_role(TrainConfig(job_name="ps", task_index=0, **base), env={})
    assert r.kind == "ps" and r.world_size == 3
    r = cli.resolve_role(TrainConfig(job_name="worker", task_index=0, worker_hosts="localhost:5000,localhost:5001"),
                         env={})
    assert r.master_port == 5000 and not r.store_is_ps
    assert cli.resolve_role(TrainConfig(job_name="chief"), env={}).kind == "none"
    r = cli.resolve_role(TrainConfig(), env={"RANK": "3", "WORLD_SIZE": "8", "LOCAL_RANK": "3",
                                             "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "1234"})
    assert (r.rank, r.world_size, r.master_port, r.from_env) == (3, 8, 1234, True)
    with pytest.raises(ValueError):
        cli.resolve_role(TrainConfig(job_name="worker", task_index=5, **base), env={})


# ---- gloo DP equivalence ----------------------------------------------------------------------------
def _dp_worker(rank, world, port, out, steps, B):
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    import dmlc  # noqa: F401
    from dmlc.data import synthetic
    from dmlc.engine.eager import EagerTrainer
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    x, y = synthetic(256, seed=1)
    tr = EagerTrainer("cifar_cnn", B, x, y, world_size=world, rank=rank, lr=1e-4, relu_logits=False, seed=3)
    for _ in range(steps):
        tr.step()
    torch.save(tr.flat_params(), os.path.join(out, f"rank{rank}.pt"))
    dist.destroy_process_group()


def test_gloo_dp_equals_single_process_large_batch(tmp_path):
    import torch.multiprocessing as mp
    from dmlc.data import synthetic
    from dmlc.engine.eager import EagerTrainer
    from dmlc.models import cifar_cnn as M
    world, B, steps = 2, 16, 3
    mp.spawn(_dp_worker, args=(world, cli.free_port(), str(tmp_path), steps, B), nprocs=world, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert torch.equal(r0, r1)                   # replicas stay identical
    # single process, global batch = union of the ranks' shards, mean loss over 2B
    x, y = synthetic(256, seed=1)
    ranks = [EagerTrainer("cifar_cnn", B, x, y, world_size=world, rank=r, seed=3) for r in range(world)]
    flat = M.init_flat_params(torch.Generator().manual_seed(3)).requires_grad_(True)
    for s in range(steps):
        idx = torch.cat([t.epoch_permutation(s // t.period)[(s % t.period) * B:(s % t.period + 1) * B]
                         for t in ranks])
        xb = x[idx][:, 4:28, 4:28, :].float()
        loss = M.cifar_loss(M.cnn_forward(xb, M.views(flat), relu_logits=False), y[idx])
        g, = torch.autograd.grad(loss, flat)
        lr = 1e-4 * 0.9 ** (s // 250)
        flat = (flat - lr * g).detach().requires_grad_(True)
    init = M.init_flat_params(torch.Generator().manual_seed(3))
    d_dp, d_ref = r0 - init, flat.detach() - init
    # fp32 summation-order noise only (a missing 1/world average would give ~1.0)
    assert float((d_dp - d_ref).norm() / d_ref.norm()) < 1e-3


def test_rank_shards_are_disjoint():
    from dmlc.data import synthetic
    from dmlc.engine.eager import EagerTrainer
    x, y = synthetic(100, seed=0)
    shards = [set(EagerTrainer("cifar_cnn", 10, x, y, world_size=4, rank=r).epoch_permutation(0).tolist())
              for r in range(4)]
    assert all(len(s) == 20 for s in shards)
    assert len(set.union(*shards)) == 80


# ---- the reference's 3-terminal recipe (1 ps + 2 workers), CPU / gloo ---------------------------------
COMMON = ["--synthetic", "--synthetic_size=512", "--batch_size=16", "--device=cpu", "--learning_rate=0.0001",
          "--relu_logits=false", "--output_every=5", "--eval_every=10", "--eval_batches=1"]


def _env():
    e = dict(os.environ)
    e["OMP_NUM_THREADS"] = "2"
    e.pop("RANK", None)
    e.pop("WORLD_SIZE", None)
    return e


@pytest.mark.timeout(300)
def test_ps_worker_recipe(tmp_path):
    p0, p1, p2 = cli.free_port(), cli.free_port(), cli.free_port()
    hosts = [f"--ps_hosts=localhost:{p0}", f"--worker_hosts=localhost:{p1},localhost:{p2}"]
    flags = hosts + COMMON + [f"--log_dir={tmp_path}", "--generations=12"]
    ps = subprocess.Popen([sys.executable, ENTRY, "--job_name=ps", "--task_index=0"] + flags, env=_env(),
                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    ws = [subprocess.Popen([sys.executable, ENTRY, "--job_name=worker", f"--task_index={k}"] + flags, env=_env(),
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for k in range(2)]
    outs = [w.communicate(timeout=240)[0] for w in ws]
    ps_out = ps.communicate(timeout=60)[0]
    assert [w.returncode for w in ws] == [0, 0], outs
    assert ps.returncode == 0, ps_out
    assert "all 2 worker(s) finished" in ps_out
    assert "Starting Training" in outs[0] and "global_step 10, task:0_step 9, training accuracy" in outs[0]
    assert "global_step 10, task:1_step 9, training accuracy" in outs[1]
    assert " --- Test Accuracy = " in outs[0]
    assert CK.latest_checkpoint(str(tmp_path)).endswith("model.ckpt-12")
    # only the chief writes checkpoints / events / metrics
    recs = [json.loads(l) for l in open(tmp_path / "metrics.jsonl")]
    assert recs[-1]["step"] == 10 or recs[-1].get("test_accuracy") is not None


@pytest.mark.timeout(300)
def test_launcher_fault_injection_resumes_from_checkpoint(tmp_path):
    env = _env()
    env.update(DMLC_FAULT_STEP="7", DMLC_FAULT_RANK="1")
    cmd = [sys.executable, "-m", "dmlc.launch", "--nproc", "2", "--max_restarts", "2", "--"] + COMMON + \
          [f"--log_dir={tmp_path}", "--generations=15", "--checkpoint_secs=0"]
    r = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stdout
    assert "[fault-injection] rank 1 exiting at global_step 7" in r.stdout
    assert "restart 1/2" in r.stdout
    assert "Restored" in r.stdout                 # the relaunched chief resumed from a checkpoint
    path = CK.latest_checkpoint(str(tmp_path))
    assert path.endswith("model.ckpt-15")
    assert int(CK.read_bundle(path)["global_step"]) == 15


@pytest.mark.timeout(300)
def test_bench_gpus2_self_launches_two_ranks(tmp_path):
    """``python bench.py --gpus 2`` without a torchrun environment starts its own two ranks (before
    any GPU call) and the JSON line proves the world it ran in."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--impl", "eager",
                          "--batch", "8", "--steps", "2", "--warmup", "1", "--dataset-size", "256"],
                         env=env, capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout              # rank 0 only
    rec = lines[0]
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    comm = rec["config"]["comm"]
    assert comm["world_size_seen"] == 2 and comm["backend"] == "gloo", comm
    assert rec["config"]["global_batch"] == 16


@pytest.mark.timeout(120)
def test_bench_rejects_world_size_mismatch():
    import subprocess
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--impl", "eager",
                          "--batch", "8", "--steps", "1", "--warmup", "1", "--dataset-size", "64"],
                         env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 3, (out.returncode, out.stderr[-2000:])


def test_rccl_channel_env(monkeypatch):
    """--rccl_channels sets NCCL_MIN_NCHANNELS (and a matching max) before the communicator exists;
    values already in the environment win; 0 leaves RCCL's own choice."""
    from dmlc.parallel import dist as D
    for k in D.RCCL_ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    assert D.rccl_env(0) == {}
    assert D.rccl_env(14) == {"NCCL_MIN_NCHANNELS": "14", "NCCL_MAX_NCHANNELS": "14"}
    monkeypatch.setenv("NCCL_MIN_NCHANNELS", "28")
    monkeypatch.setenv("NCCL_MAX_NCHANNELS", "16")
    assert D.rccl_env(7) == {"NCCL_MIN_NCHANNELS": "28", "NCCL_MAX_NCHANNELS": "28"}
    from dmlc import cli
    assert cli.parse(["--rccl_channels=7"])[0].rccl_channels == 7


# ---- bounded failure detection without the dmlc.launch supervisor (parallel/health.py) ----------------
def _two_workers(tmp_path, extra_env, flags, timeout=200):
    p1, p2 = cli.free_port(), cli.free_port()
    hosts = [f"--worker_hosts=localhost:{p1},localhost:{p2}"]
    env = _env()
    env.update(extra_env)
    ws = [subprocess.Popen([sys.executable, ENTRY, "--job_name=worker", f"--task_index={k}"] + hosts + COMMON + flags
                           + [f"--log_dir={tmp_path}"], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                           text=True, start_new_session=True) for k in range(2)]
    return ws


@pytest.mark.timeout(300)
def test_heartbeat_survivor_exits_75_when_peer_goes_silent(tmp_path):
    """A SIGSTOPped peer (alive, silent) holds every collective: only the heartbeat can see it.  The
    survivor must exit 75 within the heartbeat timeout (5 s here; the bound asked for is <= 30 s), not
    after the 300 s process-group timeout -- launched as the reference's terminals, no supervisor."""
    import signal
    import time
    ws = _two_workers(tmp_path, dict(DMLC_FAULT_STEP="6", DMLC_FAULT_RANK="1", DMLC_FAULT_MODE="stop"),
                      ["--generations=100000", "--heartbeat_timeout_s=5", "--output_every=1000", "--eval_every=100000"])
    try:
        t0 = None
        out0 = ""
        deadline = time.time() + 240
        while time.time() < deadline and ws[0].poll() is None:
            time.sleep(0.2)
        out0 = ws[0].communicate(timeout=30)[0]
        assert ws[0].returncode == 75, out0
        assert "silent for" in out0 and "exiting for restart" in out0, out0
    finally:
        for w in ws:
            if w.poll() is None:
                os.killpg(w.pid, signal.SIGKILL)
                w.wait()
    out1 = ws[1].communicate()[0]
    assert "[fault-injection] rank 1 stopping (SIGSTOP) at global_step 6" in out1, out1


@pytest.mark.timeout(300)
def test_heartbeat_detection_time_is_bounded(tmp_path):
    """Time from the peer's fault to the survivor's exit is within heartbeat timeout + slack."""
    import signal
    import time
    ws = _two_workers(tmp_path, dict(DMLC_FAULT_STEP="4", DMLC_FAULT_RANK="1", DMLC_FAULT_MODE="stop"),
                      ["--generations=100000", "--heartbeat_timeout_s=8", "--output_every=1000", "--eval_every=100000"])
    try:
        # wait for the fault line on rank 1 (its stdout is a pipe: read until it stops)
        t_fault = None
        deadline = time.time() + 200
        while time.time() < deadline:
            line = ws[1].stdout.readline()
            if "stopping (SIGSTOP)" in line:
                t_fault = time.time()
                break
            if not line and ws[1].poll() is not None:
                break
        assert t_fault is not None
        ws[0].wait(timeout=60)
        dt = time.time() - t_fault
        assert ws[0].returncode == 75
        assert dt <= 30.0, dt
    finally:
        for w in ws:
            if w.poll() is None:
                os.killpg(w.pid, signal.SIGKILL)
                w.wait()


@pytest.mark.timeout(300)
def test_replica_divergence_is_detected_and_forces_rccl(tmp_path):
    """A replica that stops matching the others (here: perturbed on rank 1) is caught at the next
    output point on EVERY rank (exit 75) and a marker naming the all-reduce the run really used is
    left in log_dir.  Only a divergence under the custom xGMI all-reduce makes the next start fall
    back to RCCL (this CPU world all-reduces over gloo: its marker forces nothing)."""
    ws = _two_workers(tmp_path, dict(DMLC_FAULT_STEP="3", DMLC_FAULT_RANK="1", DMLC_FAULT_MODE="diverge"),
                      ["--generations=50", "--output_every=5", "--eval_every=100000"])
    outs = [w.communicate(timeout=240)[0] for w in ws]
    assert [w.returncode for w in ws] == [75, 75], outs
    assert all("replica divergence at global_step 5" in o for o in outs), outs
    marker = tmp_path / ".dmlc_replica_divergence"
    assert marker.exists() and "allreduce=gloo" in marker.read_text(), marker.read_text()
    ws = _two_workers(tmp_path, {}, ["--generations=6", "--output_every=5", "--eval_every=100000"])
    outs = [w.communicate(timeout=240)[0] for w in ws]
    assert [w.returncode for w in ws] == [0, 0], outs
    assert "using --allreduce=rccl" not in outs[0]
    with open(marker, "a") as f:                   # as a divergence under the xGMI path records it
        f.write("2026-01-01T00:00:00 rank 0 global_step 5 allreduce=xgmi\n")
    ws = _two_workers(tmp_path, {}, ["--generations=12", "--output_every=5", "--eval_every=100000"])
    outs = [w.communicate(timeout=240)[0] for w in ws]
    assert [w.returncode for w in ws] == [0, 0], outs
    assert "using --allreduce=rccl" in outs[0]
    assert marker.exists()                         # an RCCL run does not clear an xGMI marker
