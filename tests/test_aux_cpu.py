"""Auxiliary subsystems: sharded checkpoint/resume, heartbeat watchdog + fault injection,
collective-order checker, roctx tracing (no-op without a profiler)."""
import time

import torch
import torch.nn.functional as F

from ps_amd.obs import trace
from ps_amd.parallel.colocated import ColocatedPS
from ps_amd.parallel.sparse_table import SparseTable
from ps_amd.parallel.updaters import AdagradUpdater, AdamUpdater
from ps_amd.utils.checkpoint import CheckpointManager
from ps_amd.utils.fault import FaultInjector, Heartbeat, Watchdog, parse_fault
from tests import dist_util


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 2))


def _train(m, ps, x, y, n):
    for _ in range(n):
        F.cross_entropy(m(x), y).backward()
        ps.finish_step()


def test_checkpoint_resume_bitwise(tmp_path):
    x, y = torch.randn(32, 8), torch.randint(0, 2, (32,))
    # run A: 3 steps, checkpoint, 3 more steps
    m = _model()
    ps = ColocatedPS(m, AdamUpdater(0.01, bias_correction="step"), bucket_mb=0.0005)
    tab = SparseTable("t", 4, 100, AdagradUpdater(0.1), init=(-0.1, 0.1), seed=1)
    tab.push(torch.tensor([1, 5]), torch.ones(2, 4))
    _train(m, ps, x, y, 3)
    ck = CheckpointManager(str(tmp_path))
    ck.save(3, ps, {"t": tab}, extra={"cursor": 96}, blocking=False)
    ck.wait()
    _train(m, ps, x, y, 3)
    final_a = [p.detach().clone() for p in m.parameters()]
    # run B: fresh objects, resume from the checkpoint, 3 steps
    m2 = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 2))
    ps2 = ColocatedPS(m2, AdamUpdater(0.01, bias_correction="step"), bucket_mb=0.0005)
    tab2 = SparseTable("t", 4, 100, AdagradUpdater(0.1), init=(-0.1, 0.1), seed=1)
    st = CheckpointManager(str(tmp_path)).load(None, ps2, {"t": tab2})
    assert st["extra"]["cursor"] == 96 and ps2.round == 3
    assert torch.equal(tab2.table, tab.table) and torch.equal(tab2.states[0], tab.states[0])
    _train(m2, ps2, x, y, 3)
    for a, b in zip(final_a, m2.parameters()):
        assert torch.equal(a, b.detach())
    assert (tmp_path / "step00000003" / "manifest.json").exists()


def test_fault_spec_and_injector():
    spec = parse_fault("kill:rank=1:step=5,delay_push:ms=20,drop_push:p=1.0")
    assert spec["kill"] == {"rank": "1", "step": "5"} and spec["delay_push"]["ms"] == "20"
    fi = FaultInjector("delay_push:ms=20,drop_push:p=1.0", rank=0)
    t0 = time.time()
    fi.before_push()
    assert time.time() - t0 >= 0.019 and fi.drop()
    fi.at_step(5)  # kill targets rank 1 only: no exit here


def test_heartbeat_watchdog_detects_dead_rank():
    from torch.distributed import TCPStore

    port = dist_util.free_port()
    store = TCPStore("127.0.0.1", port, 2, True, wait_for_workers=False)
    hb0 = Heartbeat(store, 0, period=0.05).start()
    store.set("hb/1", str(time.time()))  # rank 1 beat once, then "died"
    failures = []
    wd = Watchdog(store, 2, timeout=0.3, period=0.05, on_failure=lambda r, s: failures.append(r)).start()
    time.sleep(0.8)
    wd.stop()
    hb0.stop()
    assert failures == [1]


def _order_body(tp, diverge):
    from ps_amd.parallel.transport import Transport

    t = Transport(check_order=True)
    x = torch.ones(4)
    t.all_reduce(x)
    if diverge and tp.rank == 1:
        t._note("ag", torch.ones(3))  # simulate a rank that would issue a different collective
    try:
        t.verify_order()
        return "ok"
    except RuntimeError:
        return "mismatch"


def test_collective_order_checker():
    assert dist_util.run(_order_body, 2, (False,)) == ["ok", "ok"]
    assert dist_util.run(_order_body, 2, (True,)) == ["mismatch", "mismatch"]


def test_trace_ranges_noop_safe():
    st = trace.StepTimer()
    with st.phase("push"):
        with trace.range("inner"):
            pass
    st.step_done()
    assert "push" in st.summary()


def test_native_ps_server_threadsanitizer(tmp_path):
    """SURVEY §5.2 c: the native PS server under ThreadSanitizer -- W concurrent clients x R BSP
    rounds (exact result check) + an SSP clock-bound phase; any TSan report fails the test."""
    import os
    import shutil
    import subprocess

    import pytest

    cxx = os.environ.get("CXX", "/opt/rocm/lib/llvm/bin/clang++")
    if not (os.path.exists(cxx) or shutil.which(cxx)):
        pytest.skip("no clang++ with a TSan runtime")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "ps_stress_tsan")
    subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread",
                    f"-I{root}/csrc/runtime", f"{root}/csrc/runtime/ps_server.cpp",
                    f"{root}/csrc/runtime/tests/ps_stress.cpp", "-o", exe], check=True, timeout=300)
    r = subprocess.run([exe, "4", "10", "8"], capture_output=True, text=True, timeout=300,
                       env={**os.environ, "TSAN_OPTIONS": "halt_on_error=1"})
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "ps_stress ok" in out and "ThreadSanitizer" not in out, out[-3000:]


def test_fault_kill_at_step_exits_the_rank():
    """PS_AMD_FAULT=kill:rank=0:step=2 ends the process hard at the start of PS round 2."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys, torch, torch.nn.functional as F\n"
        f"sys.path.insert(0, {root!r})\n"
        "from ps_amd.parallel.colocated import ColocatedPS\n"
        "from ps_amd.parallel.updaters import SimpleUpdater\n"
        "m = torch.nn.Linear(4, 2); ps = ColocatedPS(m, SimpleUpdater(0.1))\n"
        "for i in range(5):\n"
        "    F.mse_loss(m(torch.ones(3, 4)), torch.zeros(3, 2)).backward(); ps.finish_step()\n"
        "    print('step', i, flush=True)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env={**os.environ, "PS_AMD_FAULT": "kill:rank=0:step=2"})
    assert r.returncode == 17, r.stderr[-2000:]
    assert r.stdout.split() == ["step", "0", "step", "1"]


def test_wgrad_side_stream_policy(monkeypatch):
    """ops/side_stream.enabled: batches <= 512 per GPU always, larger ones only when the rank
    owns its GPU (profiles/r4_wgrad_stream_policy.txt; tests/test_stream_policy_cpu.py);
    PS_AMD_WGRAD_STREAM_MAX_IMAGES sets the cap, PS_AMD_WGRAD_STREAM=0 / 1 forces it; a Fork on
    the CPU never turns on."""
    from ps_amd.ops import side_stream as side
    from ps_amd.parallel import transport

    monkeypatch.delenv("PS_AMD_WGRAD_STREAM", raising=False)
    monkeypatch.delenv("PS_AMD_WGRAD_STREAM_MAX_IMAGES", raising=False)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert side.enabled(256) and side.enabled(1024) and not side.enabled()
    monkeypatch.setenv("WORLD_SIZE", "8")  # one rank per GPU: still the single-process policy
    assert side.enabled(512) and side.enabled(1024)
    monkeypatch.setattr(transport, "_RANKS_PER_DEVICE", 8)  # eight ranks sharing one GPU
    assert side.enabled(512) and not side.enabled(1024)
    monkeypatch.setenv("PS_AMD_WGRAD_STREAM_MAX_IMAGES", "2048")
    assert side.enabled(1024)
    monkeypatch.delenv("WORLD_SIZE")
    monkeypatch.setattr(transport, "_RANKS_PER_DEVICE", None)
    monkeypatch.setenv("PS_AMD_WGRAD_STREAM_MAX_IMAGES", "512")
    assert side.enabled(512) and not side.enabled(1024)
    monkeypatch.setenv("PS_AMD_WGRAD_STREAM", "0")
    assert not side.enabled(256)
    monkeypatch.setenv("PS_AMD_WGRAD_STREAM", "1")
    assert side.enabled(4096) and side.enabled()
    assert not side.Fork(torch.device("cpu"), (), images=8).on
