"""Registry / range partitioner properties, KVStore semantics, native TCP parameter server
(BASELINE config 1: 1 server + 2 workers over TCP loopback) in BSP / SSP / ASP."""
import threading

import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from ps_amd.context import Stat, ctx
from ps_amd.parallel.kvstore import KVStore
from ps_amd.parallel.registry import Registry, hash_router
from ps_amd.parallel.tcp import PServer, PSClient, PSRouterClient
from ps_amd.parallel.updaters import AdamUpdater, SimpleUpdater


@settings(max_examples=60, deadline=None)
@given(sizes=st.lists(st.integers(1, 5000), min_size=1, max_size=12), world=st.integers(1, 8),
       bucket=st.integers(64, 20000), last=st.integers(0, 4000))
def test_partition_covers_every_element_once(sizes, world, bucket, last):
    r = Registry(world, bucket_bytes=bucket * 4, align=16, last_bucket_bytes=last * 4 or None)
    for i, n in enumerate(sizes):
        r.add(f"k{i}", (n,), torch.float32)
    r.finalize()
    for b in r.buckets:
        assert b.size % (world * 16) == 0 and b.chunk * world == b.size
    for k, ki in r.keys.items():
        covered = np.zeros(ki.numel, dtype=np.int64)
        for rank, lo, hi in r.owner_of(k):
            covered[lo - ki.offset:hi - ki.offset] += 1
        assert (covered == 1).all()
    # buckets tile the group buffer without overlap
    end = 0
    for b in r.buckets:
        assert b.start == end
        end += b.size
    assert end == r.group_size["float32"]


def test_hash_router_nonnegative():
    route = hash_router(3)
    ids = [route(f"emF{i}.{j}") for i in range(5) for j in range(200)]
    assert min(ids) >= 0 and max(ids) <= 2 and len(set(ids)) == 3


def test_kvstore_standalone_semantics():
    kv = KVStore()
    w = kv.get("fc0.weights", lambda: torch.ones(2, 2))
    assert kv.get("missing") is None
    assert kv.get("fc0.weights", lambda: torch.zeros(2, 2)) is w  # init only once
    kv.sum("fc0.weights", torch.full((2, 2), 2.0))
    kv.sum("fc0.weights", torch.full((2, 2), 4.0))  # average of 2 contributions = 3
    kv.update({"default": SimpleUpdater(0.5)})
    assert torch.allclose(w, torch.full((2, 2), -0.5))
    kv.clear()
    # loss-surface interpolation w = s*w0 + (1-s)*w  (KVStore.java:153-155)
    ctx.status, ctx.weights_scale = Stat.LOSS_SURFACE_EVAL, 1.0
    try:
        assert torch.allclose(kv.get("fc0.weights"), torch.ones(2, 2))
    finally:
        ctx.status, ctx.weights_scale = Stat.TRAINING, 0.0
    kv.async_get("b", lambda: torch.full((3,), 7.0))
    kv.async_wait()
    assert torch.equal(kv.get("b"), torch.full((3,), 7.0))


def _mlp(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(20, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3))


def test_tcp_one_server_two_workers_bsp_equals_large_batch():
    """BASELINE config 1: 2-layer MLP, 1 server + 2 workers on TCP loopback, BSP.
    Two workers on half batches == one process on the full batch (grad average)."""
    srv = PServer(0, workers=2, mode="bsp", barrier_timeout_s=60).start()
    try:
        x = torch.randn(64, 20)
        y = torch.randint(0, 3, (64,))
        upd = {"default": AdamUpdater(0.01, bias_correction="reference")}
        losses = {}
        models = [_mlp(), _mlp()]  # built in the main thread: torch's global RNG is not per-thread

        def worker(wid):
            m = models[wid]
            kv = KVStore(PSClient("127.0.0.1", srv.port), worker_id=wid)
            xs, ys = x[wid::2], y[wid::2]
            for step in range(5):
                kv.pull_into(m)
                m.zero_grad()
                torch.nn.functional.cross_entropy(m(xs), ys).backward()
                kv.sum_from(m)
                kv.update(upd)
                kv.clear()
            kv.pull_into(m)
            losses[wid] = m

        ts = [threading.Thread(target=worker, args=(w,)) for w in range(2)]
        [t.start() for t in ts]
        [t.join(timeout=60) for t in ts]
        assert len(losses) == 2
        # single-process oracle: full batch == mean of the two half-batch gradients
        ref = _mlp()
        u = AdamUpdater(0.01, bias_correction="reference")
        for step in range(5):
            ref.zero_grad()
            g = {}
            for wid in range(2):
                ref.zero_grad()
                torch.nn.functional.cross_entropy(ref(x[wid::2]), y[wid::2]).backward()
                for n, p in ref.named_parameters():
                    g[n] = g.get(n, 0) + p.grad.detach().clone() / 2
            with torch.no_grad():
                for n, p in ref.named_parameters():
                    u.update(n, p.data, g[n])
        for (n, p), (_, q) in zip(losses[0].named_parameters(), ref.named_parameters()):
            torch.testing.assert_close(p, q, rtol=1e-4, atol=1e-5)
        st_ = PSClient("127.0.0.1", srv.port).stats()
        assert st_["generation"] == 5 and st_["mode"] == "bsp"
    finally:
        srv.stop()


def test_tcp_asp_and_first_writer_wins():
    srv = PServer(0, workers=2, mode="asp").start()
    try:
        c1, c2 = PSClient("127.0.0.1", srv.port), PSClient("127.0.0.1", srv.port)
        a = c1.update("w", torch.ones(3), replace=False)
        b = c2.update("w", torch.zeros(3), replace=False)
        assert torch.equal(a, b) and torch.equal(b.reshape(-1), torch.ones(3))
        c1.push({"w": torch.ones(3)}, "simple@eta:0.5@")  # ASP: applied immediately
        assert torch.allclose(c2.get("w").reshape(-1), torch.full((3,), 0.5))
        assert c1.barrier(0) == 0  # async barrier returns at once
    finally:
        srv.stop()


def test_tcp_ssp_clock_bound():
    srv = PServer(0, workers=2, mode="ssp", staleness=1, barrier_timeout_s=30).start()
    try:
        fast, slow = PSClient("127.0.0.1", srv.port), PSClient("127.0.0.1", srv.port)
        assert fast.clock(0, 1) == 0  # 1 - 0 <= 1: proceeds
        done = threading.Event()

        def ahead():
            fast.clock(0, 2)  # 2 - 0 > 1: must block until the slow worker advances
            done.set()

        t = threading.Thread(target=ahead)
        t.start()
        assert not done.wait(0.3)
        slow.clock(1, 1)
        assert done.wait(5)
        t.join()
    finally:
        srv.stop()


def test_tcp_router_checkpoint(tmp_path):
    s1, s2 = PServer(0, 1, "bsp").start(), PServer(0, 1, "bsp").start()
    try:
        rc = PSRouterClient([f"127.0.0.1:{s1.port}", f"127.0.0.1:{s2.port}"])
        vals = {f"emF{i}.{j}": torch.full((4,), float(i * 10 + j)) for i in range(3) for j in range(10)}
        rc.update_list(vals)
        got = rc.get_list(list(vals))
        assert all(torch.equal(got[k].reshape(-1), v) for k, v in vals.items())
        counts = [s["keys"] for s in rc.stats()]
        assert sum(counts) == 30 and min(counts) > 0  # both shards used
        rc.push({k: torch.ones(4) for k in vals}, "simple@eta:1.0@")
        rc.barrier(0)
        rc.save(str(tmp_path / "ckpt"))
        rc.push({k: torch.ones(4) for k in vals}, "simple@eta:1.0@")
        rc.barrier(0)
        rc.load(str(tmp_path / "ckpt"))
        got = rc.get_list(list(vals))
        assert all(torch.equal(got[k].reshape(-1), v - 1) for k, v in vals.items())
    finally:
        s1.stop()
        s2.stop()


class _SlowClient:
    """A PS client whose batched reads take ``delay`` seconds (a slow / remote server)."""

    def __init__(self, delay):
        import threading

        self.delay, self.vals, self.calls = delay, {}, 0
        self.mu = threading.Lock()

    def get_list(self, keys):
        import time

        time.sleep(self.delay)
        with self.mu:
            self.calls += 1
            return {k: (self.vals[k].clone() if k in self.vals else None) for k in keys}

    def update_list(self, items, replace=False):
        with self.mu:
            for k, v in items.items():
                self.vals.setdefault(k, v.clone())
            return {k: self.vals[k].clone() for k in items}

    def get(self, key):
        return self.get_list([key])[key]


def test_prefetch_thread_overlaps_a_slow_server():
    """KVStore docstring: async_get queues keys for a real prefetch thread;
    after update/clear a worker re-fetches its dropped keys in the background, so the next
    step's pull overlaps the caller's work instead of paying the server latency again."""
    import time

    c = _SlowClient(0.3)
    kv = KVStore(c, worker_id=0, consistency="asp")
    for k in ("a", "b", "c"):
        kv.async_get(k, lambda k=k: torch.full((2,), float(ord(k))))
    t0 = time.perf_counter()
    kv.async_wait()  # one batched round trip for the three keys
    assert time.perf_counter() - t0 < 0.55 and c.calls == 1
    assert torch.equal(kv.get("b"), torch.full((2,), 98.0))
    c.vals["b"] = torch.full((2,), 5.0)  # the server moved on
    kv.clear()  # drops the cache and starts re-fetching a, b, c in the background
    time.sleep(0.4)  # the caller's compute
    t1 = time.perf_counter()
    for k in ("a", "b", "c"):
        kv.async_get(k, lambda: torch.zeros(2))
    kv.async_wait()
    assert time.perf_counter() - t1 < 0.1  # already fetched while we computed
    assert torch.equal(kv.get("b"), torch.full((2,), 5.0))
    assert kv.prefetch_batches == 2
