"""HIP kernel numerics vs the plain-torch fp32 reference of the same op (CPU path).

Every test builds inputs on the CPU, runs the reference implementation there, runs the HIP
kernel on cuda:0 and compares.  Shapes include non-multiple-of-8/16/64 tails (275 = the CTR
concat width the reference's jcublas smoke test used, 784, 1568).
"""
import pytest
import torch

from ps_amd import ops
from ps_amd.ops import compress as C
from ps_amd.ops import nn_ops as N
from ps_amd.ops import reduce as R
from ps_amd.ops import sparse as S

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_native_loaded():
    m = ops.native()
    assert m.ARCH == "gfx950"


@pytest.mark.parametrize("kind", [ops.SGD, ops.ADAM, ops.ADAGRAD, ops.FTRL])
@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [275, 4096, 150 * 784 + 3])
@pytest.mark.parametrize("wout", [None, torch.bfloat16, torch.float32])
def test_fused_opt(kind, gdt, n, wout):
    torch.manual_seed(kind * 31 + n)
    w = torch.randn(n)
    g = torch.randn(n).to(gdt)
    s0 = torch.rand(n) if kind != ops.SGD else torch.randn(n)
    s1 = torch.rand(n)
    hp = dict(lr=0.05, beta1=0.9, beta2=0.99, eps=1e-6, wd=0.01, momentum=0.9, nesterov=(n % 2 == 1),
              bc1=1.1, bc2=1.2, l1=0.01, l2=0.02, fbeta=1.0, ftrl_mode=n % 2, gscale=0.5)
    two = kind in (ops.ADAM, ops.FTRL)
    ref = [w.clone(), s0.clone(), s1.clone() if two else None]
    ops.fused_opt(kind, ref[0], ref[1], ref[2], g, **hp)
    gw, gs0, gs1 = w.to(DEV), s0.to(DEV), (s1.to(DEV) if two else None)
    wo = torch.empty(n, dtype=wout, device=DEV) if wout is not None else None
    ops.fused_opt(kind, gw, gs0, gs1, g.to(DEV), wout=wo, **hp)
    torch.cuda.synchronize()
    torch.testing.assert_close(gw.cpu(), ref[0], rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(gs0.cpu(), ref[1], rtol=2e-5, atol=2e-5)
    if two:
        torch.testing.assert_close(gs1.cpu(), ref[2], rtol=2e-5, atol=2e-5)
    if wo is not None:
        torch.testing.assert_close(wo.float().cpu(), ref[0].to(wout).float(), rtol=1e-2, atol=1e-2)


def test_fused_opt_gscale_tensor_and_unaligned():
    n = 1000
    w = torch.randn(n + 1)[1:]  # misaligned view -> scalar path
    g = torch.randn(n)
    ref = w.clone()
    ops.fused_opt(ops.SGD, ref, None, None, g * 0.25, lr=0.1)
    gw = torch.randn(n + 1, device=DEV)[1:]
    gw.copy_(w.to(DEV))
    ops.fused_opt(ops.SGD, gw, None, None, g.to(DEV), gscale_t=torch.tensor([0.25], device=DEV), lr=0.1)
    torch.testing.assert_close(gw.cpu(), ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("kind,rowwise", [(ops.ADAGRAD, True), (ops.ADAGRAD, False), (ops.ADAM, False),
                                          (ops.FTRL, False), (ops.SGD, False)])
def test_sparse_opt(kind, rowwise):
    torch.manual_seed(3)
    rows_total, dim = 500, 10
    table = torch.randn(rows_total, dim)
    rows = torch.randperm(rows_total)[:77]
    grad = torch.randn(77, dim)
    grad[5, 0] = 0.0
    st0 = torch.rand(rows_total) if rowwise else torch.rand(rows_total, dim)
    st1 = torch.rand(rows_total, dim) if kind in (ops.ADAM, ops.FTRL) else None
    hp = dict(lr=0.1, eps=1e-6, bc1=1.0, bc2=1.0, l1=0.01, l2=0.01, ftrl_mode=1)
    skip = kind == ops.FTRL
    rt, r0, r1 = table.clone(), st0.clone(), st1.clone() if st1 is not None else None
    ops.sparse_opt(kind, rt, r0, r1, rows, grad, rowwise=rowwise, skip_zero=skip, **hp)
    gt, g0, g1 = table.to(DEV), st0.to(DEV), st1.to(DEV) if st1 is not None else None
    ops.sparse_opt(kind, gt, g0, g1, rows.to(DEV), grad.to(DEV), rowwise=rowwise, skip_zero=skip, **hp)
    torch.testing.assert_close(gt.cpu(), rt, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(g0.cpu(), r0, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [1, 275, 1 << 20, (1 << 22) + 5])
def test_sumsq_clip(dt, n):
    x = torch.randn(n).to(dt)
    ref = x.double().pow(2).sum().item()
    out = R.sumsq(x.to(DEV))
    assert abs(out.item() - ref) <= 1e-4 * ref + 1e-6
    f = R.clip_factor(out, 1.0)
    assert abs(f.item() - min(1.0, 1.0 / (ref ** 0.5 + 1e-6))) < 1e-4
    out2 = R.sumsq(x.to(DEV))
    assert out2.item() == out.item()  # deterministic


@pytest.mark.parametrize("xd,yd", [(torch.float32, torch.bfloat16), (torch.bfloat16, torch.float32),
                                   (torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16)])
def test_cast_axpy_reduce(xd, yd):
    n = 12345
    x = torch.randn(n).to(xd)
    y = torch.randn(n).to(yd)
    gy = y.to(DEV)
    R.cast_(x.to(DEV), gy, 0.5)
    torch.testing.assert_close(gy.float().cpu(), (x.float() * 0.5).to(yd).float(), rtol=1e-2, atol=1e-2)
    gy = y.to(DEV)
    R.axpy_(0.3, x.to(DEV), gy)
    torch.testing.assert_close(gy.float().cpu(), (y.float() + 0.3 * x.float()).to(yd).float(), rtol=2e-2,
                               atol=2e-2)
    xs = torch.randn(4, n).to(xd)
    out = torch.empty(n, dtype=yd, device=DEV)
    R.reduce_n(xs.to(DEV), out, 0.25)
    torch.testing.assert_close(out.float().cpu(), (xs.float().sum(0) * 0.25).to(yd).float(), rtol=2e-2,
                               atol=2e-2)


def test_lerp():
    w0, w = torch.randn(1000), torch.randn(1000)
    out = torch.empty(1000, device=DEV)
    R.lerp(w0.to(DEV), w.to(DEV), 0.3, out)
    torch.testing.assert_close(out.cpu(), 0.3 * w0 + 0.7 * w)


@pytest.mark.parametrize("n", [64, 1024, 3000, 3001, 70000])
def test_onebit(n):
    torch.manual_seed(n)
    g = torch.randn(n)
    err = torch.randn(n) * 0.1
    nw, ns = C.packed_sizes(n)
    rw, rs, re = torch.zeros(nw, dtype=torch.int64), torch.zeros(ns), err.clone()
    C.onebit_pack(g, re, rw, rs)
    gw = torch.zeros(nw, dtype=torch.int64, device=DEV)
    gs = torch.zeros(ns, device=DEV)
    ge = err.to(DEV)
    C.onebit_pack(g.to(DEV), ge, gw, gs)
    assert torch.equal(gw.cpu(), rw)
    torch.testing.assert_close(gs.cpu(), rs, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ge.cpu(), re, rtol=1e-5, atol=1e-5)
    # unpack-reduce of 3 "workers"
    W = torch.stack([rw, rw, rw])
    Sc = torch.stack([rs, rs * 2, rs * 3])
    ref = torch.zeros(n)
    C.onebit_unpack_reduce(W, Sc, ref, 0.5)
    out = torch.zeros(n, device=DEV)
    C.onebit_unpack_reduce(W.to(DEV), Sc.to(DEV), out, 0.5)
    torch.testing.assert_close(out.cpu(), ref)


@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
def test_onebit_bf16_error_feedback(gdt):
    """The error-feedback buffer in bf16 (colocated.py ef_dtype): c = g + e is formed in fp32 and the
    new residual is rounded to bf16 -- the CPU oracle does the same."""
    n = 5000
    torch.manual_seed(7)
    g = torch.randn(n).to(gdt)
    err = (torch.randn(n) * 0.1).bfloat16()
    nw, ns = C.packed_sizes(n)
    rw, rs, re = torch.zeros(nw, dtype=torch.int64), torch.zeros(ns), err.clone()
    C.onebit_pack(g, re, rw, rs)
    gw, gs, ge = torch.zeros(nw, dtype=torch.int64, device=DEV), torch.zeros(ns, device=DEV), err.to(DEV)
    C.onebit_pack(g.to(DEV), ge, gw, gs)
    assert ge.dtype == torch.bfloat16
    assert torch.equal(gw.cpu(), rw)
    torch.testing.assert_close(gs.cpu(), rs, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ge.cpu().float(), re.float(), rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("n,mdt", [(3001, torch.float32), (5000, torch.bfloat16), (70000, torch.float32)])
def test_onebit_momentum_pack(n, mdt):
    """1-bit Adam's pack (colocated.py onebit_momentum): m = 0.9 m + 0.1 g stored back in m's dtype,
    then c = m + e packed -- vs the CPU oracle of the same op; and the warm-up momentum-only kernel."""
    torch.manual_seed(n)
    g = torch.randn(n).bfloat16()
    err = (torch.randn(n) * 0.1).to(mdt)
    mom = torch.randn(n).to(mdt)
    nw, ns = C.packed_sizes(n)
    rw, rs, re, rm = torch.zeros(nw, dtype=torch.int64), torch.zeros(ns), err.clone(), mom.clone()
    C.onebit_pack(g, re, rw, rs, rm, 0.9)
    gw, gs, ge, gm = torch.zeros(nw, dtype=torch.int64, device=DEV), torch.zeros(ns, device=DEV), err.to(DEV), mom.to(DEV)
    C.onebit_pack(g.to(DEV), ge, gw, gs, gm, 0.9)
    tol = dict(rtol=1e-2, atol=1e-3) if mdt == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gm.cpu().float(), rm.float(), **tol)
    assert (gw.cpu() != rw).sum() <= (0 if mdt == torch.float32 else nw // 50)  # bf16 m: rare sign ties differ
    torch.testing.assert_close(gs.cpu(), rs, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(ge.cpu().float(), re.float(), **tol)
    m2 = mom.to(DEV)
    C.onebit_momentum(g.to(DEV), m2, 0.5)
    torch.testing.assert_close(m2.cpu().float(), (0.5 * mom.float() + 0.5 * g.float()), **tol)


def test_sparse_rows():
    torch.manual_seed(1)
    table = torch.randn(1000, 16)
    rows = torch.randint(0, 1000, (300,))
    out_ref = torch.zeros(300, 40)
    S.gather_rows(table, rows, out_ref, 8, S.ACT_RELU)
    out = torch.zeros(300, 40, device=DEV)
    S.gather_rows(table.to(DEV), rows.to(DEV), out, 8, S.ACT_RELU)
    torch.testing.assert_close(out.cpu(), out_ref)
    ids = torch.randint(0, 50, (400,))
    grads = torch.randn(400, 10)
    u_ref, r_ref = S.dedup_rows(ids, grads, mean=True)
    u, r = S.dedup_rows(ids.to(DEV), grads.to(DEV), mean=True)
    assert torch.equal(u.cpu(), u_ref)
    torch.testing.assert_close(r.cpu(), r_ref, rtol=1e-5, atol=1e-5)
    t_ref = table[:, :10].contiguous()
    t_gpu = t_ref.to(DEV)
    S.scatter_add_rows(r_ref, u_ref, t_ref)
    S.scatter_add_rows(r, u, t_gpu)
    torch.testing.assert_close(t_gpu.cpu(), t_ref)


def test_embedding_bag_and_lr():
    torch.manual_seed(2)
    table = torch.randn(200, 10)
    ids = torch.randint(0, 200, (64, 23))
    out_ref = torch.zeros(64, 275)
    S.embedding_bag_fwd(table, ids, out_ref, 0, S.ACT_RELU)
    out = torch.zeros(64, 275, device=DEV)
    S.embedding_bag_fwd(table.to(DEV), ids.to(DEV), out, 0, S.ACT_RELU)
    torch.testing.assert_close(out.cpu(), out_ref)
    w = torch.randn(1000)
    bias = torch.randn(1)
    ids2 = torch.randint(-5000, 5000, (64, 23))
    z_ref = torch.empty(64)
    S.sparse_lr_fwd(w, ids2, bias, z_ref)
    z = torch.empty(64, device=DEV)
    S.sparse_lr_fwd(w.to(DEV), ids2.to(DEV), bias.to(DEV), z)
    torch.testing.assert_close(z.cpu(), z_ref, rtol=1e-5, atol=1e-5)


def test_lazy_init_rows():
    table = torch.zeros(100, 8, device=DEV)
    flags = torch.zeros(100, dtype=torch.uint8, device=DEV)
    rows = torch.tensor([3, 7, 7, 50], device=DEV)
    S.lazy_init_rows(table, rows, flags, 42, 1000, -0.5, 0.5)
    t1 = table.clone()
    assert flags.sum().item() == 3
    assert (t1[[3, 7, 50]].abs() > 0).all() and (t1[[0, 1, 99]] == 0).all()
    assert t1.max().item() < 0.5 and t1.min().item() >= -0.5
    table[3] += 1.0
    S.lazy_init_rows(table, rows, flags, 42, 1000, -0.5, 0.5)  # already initialised: untouched
    torch.testing.assert_close(table[3], t1[3] + 1.0)
    # same (seed, global row) -> same values on a different "rank" layout
    t2 = torch.zeros(10, 8, device=DEV)
    f2 = torch.zeros(10, dtype=torch.uint8, device=DEV)
    S.lazy_init_rows(t2, torch.tensor([3], device=DEV), f2, 42, 1000 + 4, -0.5, 0.5)  # global row 1007
    torch.testing.assert_close(t2[3], t1[7])


def test_softmax_losses():
    torch.manual_seed(4)
    x = torch.randn(100, 10) * 3000
    ref = N.softmax_temp(x)
    out = N.softmax_temp(x.to(DEV))
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-5, atol=1e-6)
    lab = torch.randint(0, 10, (100,))
    l_ref, g_ref = N.softmax_xent(ref, lab)
    l, g = N.softmax_xent(ref.to(DEV), lab.to(DEV))
    torch.testing.assert_close(l.cpu(), l_ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(g.cpu(), g_ref, rtol=1e-5, atol=1e-6)
    p = torch.rand(1000) * 0.98 + 0.01
    yy = (torch.rand(1000) > 0.5).float()
    l_ref, g_ref = N.bce(p, yy)
    l, g = N.bce(p.to(DEV), yy.to(DEV))
    torch.testing.assert_close(l.cpu(), l_ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(g.cpu(), g_ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("k,s,p", [(2, 2, 0), (3, 2, 1), (2, 1, 0)])
def test_maxpool(k, s, p):
    torch.manual_seed(5)
    x = torch.randn(2, 3, 28, 28)
    y_ref, a_ref = N.maxpool2d_fwd(x, k, s, p)
    y, a = N.maxpool2d_fwd(x.to(DEV), k, s, p)
    torch.testing.assert_close(y.cpu(), y_ref)
    dy = torch.randn_like(y_ref)
    dx_ref = N.maxpool2d_bwd(dy, a_ref, x.shape, k, s, p)
    dx = N.maxpool2d_bwd(dy.to(DEV), a, x.shape, k, s, p)
    torch.testing.assert_close(dx.cpu(), dx_ref, rtol=1e-5, atol=1e-5)


def test_im2col_col2im():
    torch.manual_seed(6)
    x = torch.randn(2, 3, 9, 7)
    col_ref = N.im2col(x, 3, 2, 1)
    col = N.im2col(x.to(DEV), 3, 2, 1)
    torch.testing.assert_close(col.cpu(), col_ref)
    back_ref = N.col2im(col_ref, x.shape, 3, 2, 1)
    back = N.col2im(col, x.shape, 3, 2, 1)
    torch.testing.assert_close(back.cpu(), back_ref, rtol=1e-5, atol=1e-5)


def test_dropout_and_init():
    x = torch.ones(1 << 16, device=DEV)
    y = N.dropout(x, 0.3, 7, 0)
    keep = (y != 0).float().mean().item()
    assert abs(keep - 0.7) < 0.01
    torch.testing.assert_close(y[y != 0], torch.full_like(y[y != 0], 1 / 0.7))
    dy = torch.randn(1 << 16, device=DEV)
    dx = N.dropout(dy, 0.3, 7, 0)
    assert torch.equal(dx != 0, y != 0)
    w = torch.empty(100000, device=DEV)
    N.uniform_init_(w, 3, -0.2, 0.2)
    assert w.min().item() >= -0.2 and w.max().item() < 0.2 and abs(w.mean().item()) < 0.01


@pytest.mark.parametrize("M,N,K", [(1000, 150, 784), (1000, 150, 275), (100, 10, 50), (64, 64, 32), (257, 33, 70),
                                   (1000, 1, 10)])
@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_mfma_linear_fwd_bwd(M, N, K, act):
    from ps_amd.ops import dense as D

    torch.manual_seed(M + N + K)
    x = (torch.randn(M, K) * 0.5).bfloat16()
    w = (torch.randn(N, K) * 0.1).bfloat16()
    b = torch.randn(N) * 0.1
    dy = torch.randn(M, N).bfloat16()
    # fp32 reference on the same bf16-rounded inputs
    xr, wr, br = x.float().requires_grad_(), w.float().requires_grad_(), b.clone().requires_grad_()
    yr = D._act_ref(xr @ wr.t() + br, act)
    yr.backward(dy.float())
    xg, wg, bg = x.cuda().requires_grad_(), w.cuda().requires_grad_(), b.cuda().requires_grad_()
    yg = D.linear_act(xg, wg, bg, act)
    yg.backward(dy.cuda())
    torch.cuda.synchronize()
    tol = dict(rtol=2e-2, atol=2e-2 * max(1.0, (K ** 0.5) * 0.1))
    torch.testing.assert_close(yg.float().cpu(), yr.detach(), **tol)
    torch.testing.assert_close(xg.grad.float().cpu(), xr.grad, rtol=3e-2, atol=3e-2 * max(1.0, N ** 0.5 * 0.1))
    torch.testing.assert_close(wg.grad.float().cpu(), wr.grad, rtol=3e-2, atol=5e-2 * max(1.0, M ** 0.5 * 0.1))
    torch.testing.assert_close(bg.grad.cpu(), br.grad, rtol=3e-2, atol=5e-2 * max(1.0, M ** 0.5 * 0.1))


def test_mfma_gemm_asymmetric_identity():
    """A = I with an asymmetric B catches a transposed C-write (cdna guide §3)."""
    from ps_amd.ops import dense as D

    n = 48
    eye = torch.eye(n).bfloat16().cuda()
    b = torch.arange(n * n, dtype=torch.float32).view(n, n).remainder(97).bfloat16().cuda()
    c = D.gemm_nt(eye, b, out_dtype=torch.float32)  # I @ B^T = B^T
    torch.testing.assert_close(c, b.float().t())


@pytest.mark.gpu
@pytest.mark.parametrize("B,T,D", [(37, 26, 128), (8, 3, 64), (5, 31, 32)])
def test_dlrm_interact_fwd_bwd(B, T, D):
    from ps_amd.ops.dense import _interact_ref, dlrm_interact

    torch.manual_seed(0)
    x = torch.randn(B, D, device="cuda").bfloat16().requires_grad_(True)
    e = torch.randn(B, T, D, device="cuda").bfloat16().requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    er = e.detach().float().requires_grad_(True)
    y = dlrm_interact(x, e)
    yr = _interact_ref(xr, er)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=5e-2 * (D ** 0.5) / 4)
    g = torch.randn_like(yr).bfloat16()
    y.backward(g)
    yr.backward(g.float())
    cos = torch.nn.functional.cosine_similarity
    assert cos(x.grad.float().flatten(), xr.grad.flatten(), dim=0) > 0.999
    assert cos(e.grad.float().flatten(), er.grad.flatten(), dim=0) > 0.999
    torch.testing.assert_close(e.grad.float(), er.grad, rtol=3e-2, atol=0.15 * (D ** 0.5) / 4)


@pytest.mark.parametrize("scale", [1.0, 1e-4])
def test_softmax_temp_bwd(scale):
    torch.manual_seed(5)
    p = torch.softmax(torch.randn(1000, 10), dim=1)
    dy = torch.randn(1000, 10)
    ref = N.softmax_temp_bwd(p, dy, scale)
    out = N.softmax_temp_bwd(p.to(DEV), dy.to(DEV), scale)
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-5, atol=1e-7)
