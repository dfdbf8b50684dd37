"""Reference-parity models on CPU: MNIST MLP on the reference's own bundled 1000-row CSV,
CNN, DNN / Wide&Deep on synthetic CTR data with a known optimum, Trainer micro-batching,
loss surface, layer-level parity with the reference TestConv cases."""
import os

import numpy as np
import pytest
import torch

from ps_amd.context import ctx
from ps_amd.data.dataset import load_reference_mnist, synthetic_ctr
from ps_amd.eval.loss_surface import LossSurface
from ps_amd.eval.metrics import AUC, SoftmaxPrecision, auc_exact
from ps_amd.models import layers as L
from ps_amd.models.reference import CNN, DNN, FullConnectedNN, WideDeepNN, local_table_factory
from ps_amd.parallel.kvstore import KVStore
from ps_amd.train.trainer import CollectiveEngine, KVEngine, Trainer

MNIST = "/root/reference/src/main/resources/mnist_test.csv"


@pytest.mark.skipif(not os.path.exists(MNIST), reason="reference MNIST fixture not mounted")
@pytest.mark.parametrize("kind,threshold", [("mlp", 0.86), ("cnn", 0.88)])
def test_mnist_reference_config_quality(kind, threshold):
    """The reference's MNIST models with the reference hyper-parameters (Adam 0.005 with the
    constant bias correction, softmax T=10000 on RAW 0-255 pixels as MnistParser feeds them,
    MLP 4 replicas x 100, CNN 1 x 100, early stop at loss <= 0.01) on the 800/200 split of the
    bundled CSV.  Measured (docs/PARITY.md, scripts/mnist_parity.py): MLP 0.89-0.92, CNN
    0.915-0.93 held-out over seeds 0-2; README claims ~0.92 / ~0.96 with the absent 60K
    training file."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    from mnist_parity import run

    r = run(kind, 1, 100)
    assert r["heldout_acc"] > threshold, r


@pytest.mark.skipif(not os.path.exists(MNIST), reason="reference MNIST fixture not mounted")
def test_mnist_cnn_vs_mlp_relative_quality():
    """The CNN-over-MLP margin on identical rows (README.md:29-31 claims 0.96 vs 0.92 on the
    reference's absent training file).  Named cause of the small margin at the reference config
    (docs/PARITY.md, profiles/r5_cnn_vs_mlp_parity.txt): with softmax T = 1e4 on raw 0-255 pixels
    the CNN's logits run ~11x hotter than the MLP's (std 53K vs 4.7K at init), its softmax
    saturates and one batch reaches the per-batch early stop (loss <= 0.01) by epoch 8-12; at
    T = 1e5 the CNN trains longer and the margin is the README's ~4 points.  Pinned over seeds
    0-2: CNN >= MLP at the reference config, CNN - MLP >= 2.5 points at T = 1e5."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    from mnist_parity import run

    def mean(kind, temp):
        return sum(run(kind, s, 100, temp=temp)["heldout_acc"] for s in (0, 1, 2)) / 3

    assert mean("cnn", 1e4) >= mean("mlp", 1e4)
    assert mean("cnn", 1e5) - mean("mlp", 1e5) >= 0.025


def test_cnn_reference_shapes_and_grad():
    gen = torch.Generator().manual_seed(1)
    m = CNN.build_model(28, 28, 1, [150, 50, 10], gen=gen)
    keys = [n for n, _ in m.named_parameters()]
    assert keys[:4] == ["conv1.weights", "conv1.bias", "conv2.weights", "conv2.bias"]
    assert "fc0.weights" in keys and m.fc[0].weights.shape == (150, 1568)
    x = torch.rand(4, 784)
    y = torch.randint(0, 10, (4,))
    loss = m.train_batch({"X": x, "Y": y})
    assert np.isfinite(loss)
    assert all(p.grad is not None for p in m.parameters())
    # im2col path == torch conv
    c = m.conv1
    z1 = c(x.view(4, 1, 28, 28))
    z2 = torch.relu(torch.nn.functional.conv2d(x.view(4, 1, 28, 28), c.weights, c.bias, 1, 1))
    torch.testing.assert_close(z1, z2, rtol=1e-4, atol=1e-5)


def test_reference_testconv_cases():
    # TestConv.testImg2Col: 3x3x1 image, N=2, k=2 -> im2col/col2im round trip counts overlaps
    x = torch.arange(1, 19, dtype=torch.float32).view(2, 1, 3, 3)
    from ps_amd.ops import nn_ops as N

    col = N.im2col(x, 2, 1, 0)
    assert col.shape == (2 * 4, 4)
    back = N.col2im(col, x.shape, 2, 1, 0)
    mult = torch.tensor([[1, 2, 1], [2, 4, 2], [1, 2, 1]], dtype=torch.float32)
    torch.testing.assert_close(back, x * mult)
    # TestConv.testPool: 4x4 max-pool 2/2 forward + accumulating backward
    pool = L.PoolingLayer("pool", 4, 4, 1, 2, 2)
    f = torch.arange(1, 33, dtype=torch.float32).view(2, 1, 4, 4).requires_grad_()
    z = pool(f)
    assert z.shape == (2, 1, 2, 2) and z[0, 0, 0, 0] == 6 and z[1, 0, 1, 1] == 32
    z.backward(z.detach())
    assert f.grad.sum() == z.sum() and f.grad[0, 0, 1, 1] == 6
    # TestConv.testConvPool shapes: conv(28, k3, p0) -> 26, pool(2/2, pad 1) -> 14
    conv = L.Conv2DLayer("conv", 28, 28, 1, 3, 1, 1, 0, impl="im2col")
    assert conv.output_w == 26
    p2 = L.PoolingLayer("pool", conv.output_w, conv.output_h, conv.k, 2, 2, padding=1)
    assert p2.output_w == 14
    out = p2(conv(torch.rand(1, 784)))
    assert out.shape == (1, 1, 14, 14)


def _ctr_batches(n_batches, bs, seed, **kw):
    return [synthetic_ctr(bs, seed=seed * 1000 + i, **kw) for i in range(n_batches)]


def test_dnn_ctr_learns_and_keys():
    ctx.init()
    gen = torch.Generator().manual_seed(0)
    m = DNN.build_model(5, 4, 6, [16, 8, 1], gen=gen, emb_rows=4096,
                        table_factory=local_table_factory(id_mode="map"), init_scale=0.1)
    names = [n for n, _ in m.named_parameters()]
    assert names == ["fc0.weights", "fc0.bias", "fc1.weights", "fc1.bias", "fc2.weights", "fc2.bias"]
    assert set(m.tables()) == {"emF"} and m.tables()["emF"].fields == 5  # one table, key = (field, id)
    tr = Trainer(m, CollectiveEngine(m))
    test = synthetic_ctr(2000, fields=5, numeric=6, ids_per_field=50, seed=999)
    base = auc_exact(tr.predict([test])[0], test["Y"])
    for b in _ctr_batches(200, 256, 1, fields=5, numeric=6, ids_per_field=50):
        tr.train([b])
    after = auc_exact(tr.predict([test])[0], test["Y"])
    # Bayes-optimal AUC of this generator is 0.774; plain torch (nn.Embedding + Adam) gets ~0.73
    assert after > base + 0.1 and after > 0.7, (base, after)
    assert len(m.embedding.table.shard.idmap) <= 5 * 50  # rows exist only for ids seen


def test_widedeep_ftrl_wide_part():
    ctx.init()
    gen = torch.Generator().manual_seed(0)
    m = WideDeepNN.build_model(5, 4, 6, [16, 8, 1], 1000, gen=gen, emb_rows=4096, init_scale=0.1)
    assert "wide.bias" in dict(m.named_parameters())
    assert type(m.tables()["wide.weights"].updater).__name__ == "FtrlUpdater"
    tr = Trainer(m, CollectiveEngine(m))
    losses = [tr.train([b]) for b in _ctr_batches(30, 256, 2, fields=5, numeric=6, ids_per_field=50, wide_k=5,
                                                  wide_size=1000)]
    assert np.mean(losses[-5:]) < np.mean(losses[:5])
    wt = m.tables()["wide.weights"]
    assert wt.table.abs().sum() > 0  # zero-initialised rows need no first-touch init


def test_trainer_microbatches_equal_big_batch():
    """n replicas x b samples == one batch of n*b (reference thread-DP, Trainer.java:70-101)."""
    torch.manual_seed(0)
    gen = torch.Generator().manual_seed(0)
    m1 = FullConnectedNN.build_model(20, [16, 5], gen=gen, softmax_temp=1.0, reference_backward=False)
    m2 = FullConnectedNN.build_model(20, [16, 5], gen=torch.Generator().manual_seed(0), softmax_temp=1.0,
                                     reference_backward=False)
    t1 = Trainer(m1, CollectiveEngine(m1), n_threads=4)
    t2 = Trainer(m2, CollectiveEngine(m2), n_threads=1)
    x = torch.randn(64, 20)
    y = torch.randint(0, 5, (64,))
    for _ in range(3):
        t1.train([{"X": x[i:i + 16], "Y": y[i:i + 16]} for i in range(0, 64, 16)])
        t2.train([{"X": x, "Y": y}])
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_kvengine_standalone_matches_collective():
    gen = lambda: torch.Generator().manual_seed(3)  # noqa: E731
    m1 = FullConnectedNN.build_model(10, [8, 3], gen=gen(), softmax_temp=1.0, reference_backward=False)
    m2 = FullConnectedNN.build_model(10, [8, 3], gen=gen(), softmax_temp=1.0, reference_backward=False)
    t1 = Trainer(m1, KVEngine(m1, KVStore()))
    t2 = Trainer(m2, CollectiveEngine(m2))
    x, y = torch.randn(32, 10), torch.randint(0, 3, (32,))
    for _ in range(3):
        t1.train([{"X": x, "Y": y}])
        t2.train([{"X": x, "Y": y}])
    t1.engine.pull()
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-4, atol=1e-5)


def test_loss_surface_scan():
    gen = torch.Generator().manual_seed(0)
    m = FullConnectedNN.build_model(10, [8, 3], gen=gen, softmax_temp=1.0, reference_backward=False)
    w0 = {n: p.detach().clone() for n, p in m.named_parameters()}
    tr = Trainer(m, CollectiveEngine(m))
    b = {"X": torch.randn(64, 10), "Y": torch.randint(0, 3, (64,))}
    for _ in range(20):
        tr.train([b])
    final = {n: p.detach().clone() for n, p in m.named_parameters()}
    pts = LossSurface(b, m, w0).plot()
    assert len(pts) == 40 and pts[0][0] == -2.0
    by_s = dict(pts)
    assert by_s[0.0] < by_s[1.0]  # trained weights (s=0) beat the init (s=1)
    for n, p in m.named_parameters():
        assert torch.equal(p.detach(), final[n])  # restored


def test_auc_reference_fixture_and_bruteforce():
    rng = np.random.default_rng(0)
    p = rng.random(300)
    y = (rng.random(300) < p).astype(float)
    # brute force pairwise (strict) for tie-free scores
    pos, neg = p[y > 0], p[y <= 0]
    brute = (pos[:, None] > neg[None, :]).mean()
    assert abs(AUC(p, y).calculate() - brute) < 1e-12
    assert abs(auc_exact(p, y) - brute) < 1e-12
    # reference TestAuc-style vector with heavy ties at the 0.001 clamp
    pt = np.array([0.001, 0.917644, 0.905499, 0.001, 0.997438, 0.001259, 0.001, 0.003479, 0.001056, 0.998832])
    yt = np.array([0, 1, 1, 0, 1, 0, 1, 0, 0, 1])
    pos, neg = pt[yt > 0], pt[yt <= 0]
    tie_avg = ((pos[:, None] > neg[None, :]) + 0.5 * (pos[:, None] == neg[None, :])).mean()
    assert abs(auc_exact(pt, yt) - tie_avg) < 1e-12 and abs(tie_avg - 0.84) < 1e-12
    # reference algorithm: ties broken by input order (stable sort), not averaged -> 0.88 here
    assert abs(AUC(pt, yt).calculate() - 0.88) < 1e-12

