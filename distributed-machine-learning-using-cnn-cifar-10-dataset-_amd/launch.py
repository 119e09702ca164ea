"""Local multi-process launcher with failure detection and restart-from-checkpoint.

Automates the reference's manual recipe (/root/reference/README.md:9-14: one terminal per task on
localhost ports) and adds the recovery the TF1 MonitoredTrainingSession only half-provided
(SURVEY.md §5.3): it starts N worker processes of ``cifar10cnn.py`` (one per GPU, ranks 0..N-1,
rendezvous at 127.0.0.1:<port>), watches them, and when any worker dies it terminates the rest and
relaunches the whole world, which resumes from the latest checkpoint in ``--log_dir``
(global_step restored, so ``--generations`` stays absolute).

  python -m dmlc.launch --nproc 8 [--max_restarts 3] -- --log_dir=/tmp/run --synthetic ...
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time
from typing import List

from .cli import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENTRY = os.path.join(REPO, "cifar10cnn.py")


def _spawn(nproc: int, port: int, flags: List[str], restart: int, env_extra=None) -> List[subprocess.Popen]:
    hosts = ",".join(f"127.0.0.1:{port + (i if i else 0)}" for i in range(nproc))
    procs = []
    for k in range(nproc):
        env = dict(os.environ)
        env["DMLC_RESTART_COUNT"] = str(restart)
        env.update(env_extra or {})
        cmd = [sys.executable, ENTRY, f"--worker_hosts={hosts}", "--job_name=worker", f"--task_index={k}"] + flags
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    return procs


def _terminate(procs: List[subprocess.Popen], grace: float = 10.0):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + grace
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def run(nproc: int, flags: List[str], max_restarts: int = 3, poll_s: float = 0.2, log=print) -> int:
    restart = 0
    while True:
        procs = _spawn(nproc, free_port(), flags, restart)
        failed = None
        try:
            while True:
                codes = [p.poll() for p in procs]
                bad = [(k, c) for k, c in enumerate(codes) if c not in (None, 0)]
                if bad:
                    failed = bad[0]
                    break
                if all(c == 0 for c in codes):
                    return 0
                time.sleep(poll_s)
        except KeyboardInterrupt:
            _terminate(procs)
            return 130
        log(f"[launch] worker {failed[0]} exited with code {failed[1]}; stopping the world", flush=True)
        _terminate(procs)
        if restart >= max_restarts:
            log(f"[launch] giving up after {restart} restart(s)", flush=True)
            return 1
        restart += 1
        log(f"[launch] restart {restart}/{max_restarts}: relaunching {nproc} worker(s) from the latest checkpoint",
            flush=True)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--max_restarts", type=int, default=3)
    ap.add_argument("flags", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    flags = a.flags[1:] if a.flags and a.flags[0] == "--" else a.flags
    return run(a.nproc, flags, a.max_restarts)


if __name__ == "__main__":
    sys.exit(main())
