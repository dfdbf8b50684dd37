"""Consistency properties of the TCP parameter server (SURVEY §5.2 e, §7.6):
  * SSP(s) bound as a hypothesis property over random worker speed profiles;
  * ASP convergence smoke (two asynchronous workers, no barrier semantics);
  * fault injection: a BSP barrier with a dead worker times out instead of hanging forever
    (the reference's barrier spins forever, net/PServer.java:251-258).
"""
import threading
import time

import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from ps_amd.parallel.tcp import PServer, PSClient


@settings(max_examples=12, deadline=None)
@given(s=st.integers(0, 2), W=st.integers(2, 4),
       delays=st.lists(st.lists(st.integers(0, 3), min_size=6, max_size=6), min_size=4, max_size=4))
def test_ssp_clock_bound_property(s, W, delays):
    """No CLOCK(t) call returns to a worker while t - min_w clock_w > s."""
    srv = PServer(0, workers=W, mode="ssp", staleness=s, barrier_timeout_s=30).start()
    clocks = [0] * W
    violations = []
    errors = []

    def worker(w):
        try:
            c = PSClient("127.0.0.1", srv.port)
            for t in range(1, 7):
                time.sleep(delays[w][t - 1] * 1e-3)
                clocks[w] = t  # announced before the call: the monitor never under-reads
                c.clock(w, t)
                if t - min(clocks) > s:
                    violations.append((w, t, list(clocks)))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(W)]
    try:
        [t.start() for t in ts]
        [t.join(timeout=60) for t in ts]
    finally:
        srv.stop()
    assert not errors, errors
    assert not violations, violations


def test_asp_two_workers_converge():
    """ASP: pushes are applied on arrival, barriers return at once; two unsynchronised
    workers still drive a least-squares loss down."""
    srv = PServer(0, workers=2, mode="asp").start()
    torch.manual_seed(0)
    w_true = torch.randn(16)
    X = torch.randn(256, 16)
    Y = X @ w_true
    spec = "simple@eta:0.05@"
    losses = {0: [], 1: []}

    def worker(wid):
        c = PSClient("127.0.0.1", srv.port)
        c.register_updater(spec)
        c.update("w", torch.zeros(16), replace=False)
        for step in range(60):
            w = c.get("w").reshape(-1)
            xb, yb = X[wid::2][(step * 16) % 128:(step * 16) % 128 + 16], Y[wid::2][(step * 16) % 128:(step * 16) % 128 + 16]
            err = xb @ w - yb
            losses[wid].append(float((err ** 2).mean()))
            c.push({"w": (2 * xb.t() @ err / xb.shape[0])}, spec)
            assert c.barrier(wid) >= 0  # async barrier: returns immediately

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(2)]
    try:
        [t.start() for t in ts]
        [t.join(timeout=120) for t in ts]
    finally:
        srv.stop()
    for wid in range(2):
        assert losses[wid][-1] < 0.05 * losses[wid][0], losses[wid][::10]


def test_bsp_barrier_with_dead_worker_times_out():
    """Fault injection: one of two BSP workers never arrives -> the live worker's barrier
    fails with a timeout (the driver can then restart from the last checkpoint)."""
    srv = PServer(0, workers=2, mode="bsp", barrier_timeout_s=0.5).start()
    try:
        c = PSClient("127.0.0.1", srv.port)
        t0 = time.time()
        with pytest.raises(RuntimeError, match="timed out"):
            c.barrier(0)
        assert time.time() - t0 < 10
        # the server stays usable: a full barrier of both workers goes through afterwards
        c2 = PSClient("127.0.0.1", srv.port)
        out = []
        th = threading.Thread(target=lambda: out.append(c2.barrier(1)))
        th.start()
        out.append(c.barrier(0))
        th.join(timeout=10)
        assert len(out) == 2 and out[0] == out[1] == 1
    finally:
        srv.stop()


def test_async_ctl_protocol_under_tsan(tmp_path):
    """host ThreadSanitizer build of the async-PS control protocol stress
    (csrc/runtime/tests/async_ctl_stress.cpp: owners' serve_loop vs workers' push / SSP gate /
    pin-copy-unpin on plain host memory) -- no data race, every push applied once, no slot
    rewritten while pinned, SSP bound held."""
    import os
    import shutil
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cxx = "/opt/rocm/lib/llvm/bin/clang++"
    if not os.path.exists(cxx):
        cxx = shutil.which("clang++") or shutil.which("g++")
    exe = str(tmp_path / "stress")
    subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread", f"-I{root}/csrc/include",
                    f"{root}/csrc/runtime/tests/async_ctl_stress.cpp", "-o", exe], check=True, timeout=300)
    r = subprocess.run([exe, "3", "150", "1"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0 and "violations=0" in r.stdout, r.stdout + r.stderr[-3000:]
