"""Config parsing (reference -D flags) and optimizer math vs independent numpy oracles
transcribed from the reference Java (update/*.java)."""
import numpy as np
import pytest
import torch

from ps_amd.config import Config
from ps_amd.context import Context, Mode, Stat
from ps_amd.parallel.updaters import (AdagradUpdater, AdamUpdater, FtrlUpdater, MomentumUpdater, SimpleUpdater,
                                      parse_updater, resolve_updater)


def test_config_reference_flags():
    c = Config.from_args(["-Dmode=dist", "-DisPs=1", "-DisAsync=1", "-DworkerNum=3", "-DpsAddrs=a:1,b:2",
                          "-Dthread=4", "--staleness", "2", "--consistency=ssp"], base=Config())
    assert c.mode == "dist" and c.ps and c.ps_async and c.worker_num == 3
    assert c.ps_addr_list == ["a:1", "b:2"] and c.thread == 4 and c.staleness == 2
    assert c.effective_consistency == "ssp"
    c2 = Config.from_args(["-Dmode=standalone", "-DisPsAsync=1"], base=Config())
    assert c2.mode == "stand" and c2.effective_consistency == "asp"
    with pytest.raises(KeyError):
        Config().set("nope", 1)


def test_config_env():
    c = Config.from_env({"PS_AMD_WORKER_NUM": "5", "PS_AMD_PS": "true", "PS_AMD_BUCKET_MB": "8.5"})
    assert c.worker_num == 5 and c.ps is True and c.bucket_mb == 8.5


def test_context_predicates():
    cx = Context(Config(mode="dist", is_major=True))
    assert cx.is_distributed() and not cx.is_standalone() and cx.is_training()
    assert cx.is_report_ui()  # no thread-local set: no NPE (Q12)
    cx.model_index = 1
    assert not cx.is_report_ui()
    cx.status = Stat.LOSS_SURFACE_EVAL
    assert not cx.is_training() and cx.mode == Mode.DISTRIBUTED
    assert cx.incr_step() == 1


def test_spec_strings_roundtrip():
    for u in [SimpleUpdater(0.1), MomentumUpdater(0.2, 0.8, 1e-4, True), AdamUpdater(0.005, 0.9, 0.999, 1e-8),
              AdamUpdater(0.005, bias_correction="reference"), AdagradUpdater(0.05, 1e-6),
              FtrlUpdater(0.005, 1.0, 0.001, 0.001), FtrlUpdater(0.01, mode="reference")]:
        v = parse_updater(u.name)
        assert type(v) is type(u) and v.name == u.name
    # reference spellings
    a = parse_updater("adam@alfa:0.005@beta1:0.9@beta2:0.999@epsilon:1.0E-8@")
    assert isinstance(a, AdamUpdater) and a.bias_correction == "reference" and a.alfa == 0.005
    f = parse_updater("adam@alfa:0.005@beta:1.0@l1:0.001@l2:0.001@")  # FtrlUpdater.getName() quirk
    assert isinstance(f, FtrlUpdater) and f.mode == "reference"
    assert parse_updater("simple@eta:0.5@").eta == 0.5


def test_resolve_updater_prefix():
    d, w, wb = SimpleUpdater(1), SimpleUpdater(2), SimpleUpdater(3)
    m = {"default": d, "wide": w, "wide.bias": wb}
    assert resolve_updater("wide.bias", m) is wb
    assert resolve_updater("wide.weights.7", m) is w
    assert resolve_updater("fc0.weights", m) is d
    with pytest.raises(KeyError):
        resolve_updater("x", {"wide": w})


# ---------------- numpy oracles transcribed from the Java sources ----------------------
def np_adam_ref(w, m, v, g, alfa, b1, b2, eps):  # AdamUpdater.java:57-70
    m = g * (1 - b1) + m * b1
    v = g * g * (1 - b2) + v * b2
    mm, vv = m / (1 - b1), v / (1 - b2)
    return w + (mm / (np.sqrt(vv) + eps)) * (-alfa), m, v


def np_ftrl_ref(w, z, n, dw, alfa, beta, l1, l2):  # FtrlUpdater.java:51-76
    if dw[0] == 0:
        return w, z, n
    w = w.copy()
    for i in range(len(w)):
        if abs(z[i]) <= l1:
            w[i] = 0
        else:
            sign = 1 if z[i] >= 0 else -1
            w[i] = -(z[i] - sign * l1) / ((l2 + (beta + np.sqrt(n[i]))) / alfa)
    s = np.sqrt(n + dw ** 2) - np.sqrt(n / alfa)
    z = z + (dw - s * w)
    n = n + dw ** 2
    return w, z, n


def test_adam_reference_matches_java():
    rng = np.random.default_rng(0)
    w = rng.standard_normal(50).astype(np.float32)
    u = AdamUpdater(0.005, 0.9, 0.999, 1e-8, bias_correction="reference")
    t = torch.tensor(w)
    m = np.zeros(50, np.float32)
    v = np.zeros(50, np.float32)
    for _ in range(5):
        g = rng.standard_normal(50).astype(np.float32)
        u.update("k", t, torch.tensor(g))
        w, m, v = np_adam_ref(w, m, v, g, 0.005, 0.9, 0.999, 1e-8)
    np.testing.assert_allclose(t.numpy(), w, rtol=1e-5, atol=1e-6)


def test_adam_step_bias_matches_torch():
    p = torch.nn.Parameter(torch.randn(20))
    q = p.detach().clone()
    opt = torch.optim.Adam([p], lr=0.01)
    u = AdamUpdater(0.01, 0.9, 0.999, 1e-8, bias_correction="step")
    for i in range(5):
        g = torch.randn(20)
        p.grad = g.clone()
        opt.step()
        u.update("k", q, g)
    torch.testing.assert_close(q, p.detach(), rtol=1e-5, atol=1e-6)


def test_ftrl_reference_matches_java():
    rng = np.random.default_rng(1)
    w = np.zeros(10, np.float32)
    z = np.zeros(10, np.float32)
    n = np.zeros(10, np.float32)
    t = torch.zeros(10)
    u = FtrlUpdater(0.005, 1.0, 0.001, 0.001, mode="reference")
    for i in range(6):
        g = rng.standard_normal(10).astype(np.float32)
        if i == 3:
            g[0] = 0.0  # whole key skipped (FtrlUpdater.java:52-54)
        u.update("wide.weights.1", t, torch.tensor(g))
        w, z, n = np_ftrl_ref(w, z, n, g, 0.005, 1.0, 0.001, 0.001)
    np.testing.assert_allclose(t.numpy(), w, rtol=1e-4, atol=1e-6)


def test_ftrl_canonical_sparsifies():
    u = FtrlUpdater(0.1, 1.0, 5.0, 0.0)
    t = torch.zeros(100)
    for _ in range(3):
        u.update("k", t, torch.randn(100) * 0.1)
    assert (t == 0).float().mean() > 0.9  # strong L1 -> mostly exact zeros


def test_momentum_matches_torch():
    p = torch.nn.Parameter(torch.randn(30))
    q = p.detach().clone()
    opt = torch.optim.SGD([p], lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True)
    u = MomentumUpdater(0.1, 0.9, 1e-3, nesterov=True)
    for _ in range(4):
        g = torch.randn(30)
        p.grad = g.clone()
        opt.step()
        u.update("k", q, g)
    torch.testing.assert_close(q, p.detach(), rtol=1e-5, atol=1e-6)


def test_adagrad_matches_torch():
    p = torch.nn.Parameter(torch.randn(30))
    q = p.detach().clone()
    opt = torch.optim.Adagrad([p], lr=0.1, eps=1e-10)
    u = AdagradUpdater(0.1, 1e-10)
    for _ in range(4):
        g = torch.randn(30)
        p.grad = g.clone()
        opt.step()
        u.update("k", q, g)
    torch.testing.assert_close(q, p.detach(), rtol=1e-5, atol=1e-6)


def test_simple_updater():
    t = torch.ones(4)
    SimpleUpdater(0.5).update("k", t, torch.full((4,), 2.0))
    assert torch.equal(t, torch.zeros(4))
