"""Failure-detection helpers (parallel/health.py): the heartbeat's clean-shutdown
protocol and the replica-divergence marker semantics.  CPU only (a TCPStore on 127.0.0.1)."""
import datetime
import socket
import time

import torch.distributed as dist

from dmlc.parallel import health as H


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_divergence_marker_forces_rccl_only_for_xgmi(tmp_path):
    d = str(tmp_path)
    assert not H.divergence_marked(d)
    H.mark_divergence(d, "rank 1 global_step 5 allreduce=gloo")
    H.mark_divergence(d, "rank 0 global_step 5 allreduce=rccl")
    assert not H.divergence_marked(d)
    H.mark_divergence(d, "rank 0 global_step 9 allreduce=xgmi")
    assert H.divergence_marked(d)
    assert H.clear_divergence(d) and not H.divergence_marked(d)
    assert not H.clear_divergence(d)


def _store(port):
    return dist.TCPStore("127.0.0.1", port, None, is_master=True, timeout=datetime.timedelta(seconds=10),
                         wait_for_workers=False)


def test_rank0_waits_for_peers_before_its_store_goes_away():
    """Rank 0 (the store host in reference-CLI worlds) finishes first; its stop() must not return
    until the slower peer has marked itself done, so tearing the store down afterwards is never seen
    as a failure by that peer."""
    port = _free_port()
    store = _store(port)
    fails = []
    hb0 = H.Heartbeat(0, 2, "127.0.0.1", port, interval_s=0.1, timeout_s=5.0, on_failure=fails.append).start()
    hb1 = H.Heartbeat(1, 2, "127.0.0.1", port, interval_s=0.1, timeout_s=5.0, on_failure=fails.append).start()
    import threading
    t1 = threading.Timer(0.6, lambda: hb1.stop(done=True))
    t0 = time.monotonic()
    t1.start()
    hb0.stop(done=True)                      # returns once rank 1 is done (~0.6 s), not at once
    waited = time.monotonic() - t0
    t1.join()
    assert 0.4 < waited < 4.0, waited
    del store
    time.sleep(0.3)
    assert fails == [], fails


def test_store_loss_after_rank0_finished_is_a_clean_exit():
    """A peer whose heartbeat is still running when rank 0's store disappears -- after rank 0 marked
    itself done -- stops quietly instead of exiting 75."""
    port = _free_port()
    store = _store(port)
    fails = []
    hb0 = H.Heartbeat(0, 2, "127.0.0.1", port, interval_s=0.1, timeout_s=5.0, on_failure=fails.append).start()
    hb1 = H.Heartbeat(1, 2, "127.0.0.1", port, interval_s=0.1, timeout_s=5.0, on_failure=fails.append).start()
    hb0.stop(done=True, wait_peers_s=0.0)
    time.sleep(0.5)                          # rank 1's loop sees rank 0's done mark
    del store                                # rank 0's process (and its store) exits
    time.sleep(1.0)
    hb1.stop(done=True)
    assert fails == [], fails


def test_rank0_reports_a_store_hosted_elsewhere_going_away():
    """a store hosted outside rank 0's process (a torchrun agent, the ps role) that
    disappears mid-run is a real failure for rank 0 too -- its heartbeat must report it, not return
    quietly and stop watching its peers."""
    port = _free_port()
    store = _store(port)
    fails = []
    hb0 = H.Heartbeat(0, 2, "127.0.0.1", port, interval_s=0.1, timeout_s=5.0, on_failure=fails.append).start()
    time.sleep(0.3)
    del store                                # the external store host dies; rank 0 is still running
    deadline = time.monotonic() + 5.0
    while not fails and time.monotonic() < deadline:
        time.sleep(0.1)
    hb0.stop(done=False)
    assert fails and "store unreachable" in fails[0], fails
