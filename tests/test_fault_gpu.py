"""Fail-fast on peer loss over the xGMI all-reduce, through the reference CLI (cifar10cnn.py).

The reference inherited TF1's RecoverableSession / die-fast behaviour from MonitoredTrainingSession
(/root/reference/cifar10cnn.py:222).  Here a dead peer makes the surviving rank's
xGMI barrier time out (5 s), which sets the sticky error word mirrored in host memory; the training
loop polls it at every chunk boundary and exits with code 75 (no collective teardown), and the local
launcher restarts the world from the latest checkpoint.  Two ranks share the test box's one GPU and
rendezvous over gloo (RCCL refuses two ranks per GPU); the all-reduce is the IPC xGMI kernel."""
import os
import subprocess
import sys
import time

import pytest

from dmlc import checkpoint as CK
from dmlc import cli

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENTRY = os.path.join(REPO, "cifar10cnn.py")
FLAGS = ["--synthetic", "--synthetic_size=2048", "--batch_size=32", "--learning_rate=0.0001",
         "--relu_logits=false", "--output_every=20", "--eval_every=1000000", "--allreduce=xgmi",
         "--dp_schedule=serial", "--pg_timeout_s=60"]


def _env(**kw):
    env = dict(os.environ, DMLC_DIST_BACKEND="gloo", PYTHONUNBUFFERED="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "DMLC_RESTART_COUNT"):
        env.pop(k, None)
    env.update(kw)
    return env


@pytest.mark.timeout(200)
def test_survivor_exits_fast_when_peer_dies(tmp_path):
    p1, p2 = cli.free_port(), cli.free_port()
    flags = [f"--worker_hosts=localhost:{p1},localhost:{p2}", f"--log_dir={tmp_path}", "--generations=100000"] + FLAGS
    env = _env(DMLC_FAULT_STEP="60", DMLC_FAULT_RANK="1")
    logs = [open(tmp_path / f"w{k}.log", "w+") for k in range(2)]
    ws = [subprocess.Popen([sys.executable, ENTRY, "--job_name=worker", f"--task_index={k}"] + flags, env=env,
                           stdout=logs[k], stderr=subprocess.STDOUT, text=True, start_new_session=True)
          for k in range(2)]
    try:
        rc1 = ws[1].wait(timeout=150)
        t_dead = time.time()
        rc0 = ws[0].wait(timeout=40)
        t_exit = time.time()
    finally:
        for w in ws:
            if w.poll() is None:
                w.kill()
                w.wait()
    out = [open(tmp_path / f"w{k}.log").read() for k in range(2)]
    assert rc1 == 17, out[1][-3000:]
    assert "[fault-injection] rank 1 exiting at global_step 60" in out[1]
    assert rc0 == 75, out[0][-3000:]
    assert "gradient exchange failed" in out[0], out[0][-3000:]
    assert t_exit - t_dead < 30, t_exit - t_dead      # 5 s barrier timeout + one chunk


@pytest.mark.timeout(300)
def test_launcher_restarts_world_after_peer_loss(tmp_path):
    env = _env(DMLC_FAULT_STEP="60", DMLC_FAULT_RANK="1")
    cmd = [sys.executable, "-m", "dmlc.launch", "--nproc", "2", "--max_restarts", "2", "--",
           f"--log_dir={tmp_path}", "--generations=100", "--checkpoint_secs=0"] + FLAGS
    r = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "[fault-injection] rank 1 exiting at global_step 60" in r.stdout
    assert "restart 1/2" in r.stdout and "Restored" in r.stdout, r.stdout[-4000:]
    path = CK.latest_checkpoint(str(tmp_path))
    assert path.endswith("model.ckpt-100")
    assert int(CK.read_bundle(path)["global_step"]) == 100


@pytest.mark.timeout(200)
def test_survivor_exits_75_when_peer_dies_in_final_chunk(tmp_path):
    """a peer lost inside the LAST chunk (generations 70, output points every 20: the
    final chunk is steps 60..70 and rank 1 leaves at 60) -- the survivor's loop must run its progress
    watchdog before the final device synchronisation, so it exits 75 instead of blocking in it."""
    p1, p2 = cli.free_port(), cli.free_port()
    flags = [f"--worker_hosts=localhost:{p1},localhost:{p2}", f"--log_dir={tmp_path}", "--generations=70"] + FLAGS
    env = _env(DMLC_FAULT_STEP="60", DMLC_FAULT_RANK="1")
    logs = [open(tmp_path / f"w{k}.log", "w+") for k in range(2)]
    ws = [subprocess.Popen([sys.executable, ENTRY, "--job_name=worker", f"--task_index={k}"] + flags, env=env,
                           stdout=logs[k], stderr=subprocess.STDOUT, text=True, start_new_session=True)
          for k in range(2)]
    try:
        rc1 = ws[1].wait(timeout=150)
        rc0 = ws[0].wait(timeout=40)
    finally:
        for w in ws:
            if w.poll() is None:
                w.kill()
                w.wait()
    out = [open(tmp_path / f"w{k}.log").read() for k in range(2)]
    assert rc1 == 17, out[1][-3000:]
    assert rc0 == 75, out[0][-3000:]
    assert "global_step 60" in out[0] and "global_step 70" not in out[0], out[0][-3000:]
