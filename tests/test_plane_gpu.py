"""The xGMI plane on the MI355X: W real PROCESSES on cuda:0, each mapping the others' device
arenas through CUDA-IPC handles, the native engine issuing the fused multi-source optimizer
and the owner-dealt pull kernels, pushes fired from autograd hooks (overlap=True, the
production configuration).  Compared with single-process fp32 oracles: BSP at W = 2 and 4,
SSP(1), global-norm clipping, per-prefix updaters, 1-bit pushes (vs the CPU oracle of the
same compression), and a bf16 ResNet-tiny trajectory at W = 4 (fp32 sum of the pushes on
the owner) against fp32 torch.  The control plane (handle exchange, barriers) is gloo."""
import copy

import pytest
import torch
import torch.nn.functional as F

from ps_amd.parallel.transport import run_loopback
from tests import dist_util

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(40, 64), torch.nn.Tanh(), torch.nn.Linear(64, 5))


def _data(n=64, dev=DEV):
    g = torch.Generator().manual_seed(3)
    return torch.randn(n, 40, generator=g).to(dev), torch.randint(0, 5, (n,), generator=g).to(dev)


def _body(tp, kw, steps, upd="momentum", models=None):
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdamUpdater, MomentumUpdater, SimpleUpdater

    torch.cuda.set_device(0)
    m = (models[tp.rank] if models is not None else _model(seed=tp.rank)).to(DEV)
    u = {"momentum": lambda: MomentumUpdater(0.1, 0.9, 1e-4), "sgd": lambda: SimpleUpdater(0.2),
         "mixed": lambda: {"0.": AdamUpdater(0.01), "default": MomentumUpdater(0.1, 0.9)}}[upd]()
    ps = ColocatedPS(m, u, tp, bucket_mb=0.004, last_bucket_mb=0.002, plane="xgmi", timeout_s=60, **kw)
    x, y = _data()
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    losses = []
    for _ in range(steps):
        loss = F.cross_entropy(m(xs), ys)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    ps.synchronize()
    torch.cuda.synchronize()
    out = {n: p.detach().float().cpu().clone() for n, p in m.named_parameters()}
    st = ps.plane_stats()
    kind = ps.plane_kind
    ps.close()
    return out, losses, kind, st


def _oracle(world, steps, opt_factory, clip=None):
    ref = _model(0).to(DEV)
    opt = opt_factory(ref.parameters())
    x, y = _data()
    for _ in range(steps):
        opt.zero_grad()
        (sum(F.cross_entropy(ref(x[r::world]), y[r::world]) for r in range(world)) / world).backward()
        if clip is not None:
            torch.nn.utils.clip_grad_norm_(ref.parameters(), clip)
        opt.step()
    return {n: p.detach().cpu() for n, p in ref.named_parameters()}


@pytest.mark.parametrize("world", [2, 4])
def test_plane_processes_bsp_equals_single_process(world):
    res = dist_util.run(_body, world, ({}, 5))
    assert res[0][2] == "xgmi"
    for r in range(1, world):
        for k in res[0][0]:
            assert torch.equal(res[0][0][k], res[r][0][k])
    ref = _oracle(world, 5, lambda p: torch.optim.SGD(p, lr=0.1, momentum=0.9, weight_decay=1e-4))
    for k, v in ref.items():
        torch.testing.assert_close(res[0][0][k], v, rtol=1e-5, atol=1e-5)
    st = res[0][3]
    assert st["rounds"] >= 1 and st["serve_ms"] > 0 and st["pull_ms"] > 0


def test_plane_processes_ssp1_matches_delayed_sgd():
    world, steps, lr, s = 2, 6, 0.2, 1
    res = dist_util.run(_body, world, ({"staleness": s}, steps, "sgd", [_model(0), _model(0)]))
    ref = _model(0).to(DEV)
    x, y = _data()
    versions = [{n: p.detach().clone() for n, p in ref.named_parameters()}]
    for t in range(steps):
        probe = copy.deepcopy(ref)
        with torch.no_grad():
            for n, p in probe.named_parameters():
                p.copy_(versions[max(0, t - s)][n])
        loss = sum(F.cross_entropy(probe(x[r::world]), y[r::world]) for r in range(world)) / world
        grads = torch.autograd.grad(loss, list(probe.parameters()))
        versions.append({n: versions[-1][n] - lr * g for (n, _), g in zip(probe.named_parameters(), grads)})
    want = versions[max(0, steps - s)]
    for k in want:
        torch.testing.assert_close(res[0][0][k], want[k].cpu(), rtol=1e-5, atol=1e-5)


def test_plane_processes_clip_norm():
    res = dist_util.run(_body, 2, ({"clip_norm": 0.05}, 4, "sgd"))
    ref = _oracle(2, 4, lambda p: torch.optim.SGD(p, lr=0.2), clip=0.05)
    for k, v in ref.items():
        torch.testing.assert_close(res[0][0][k], v, rtol=1e-5, atol=1e-5)


def test_plane_processes_mixed_updaters():
    res = dist_util.run(_body, 2, ({}, 5, "mixed"))
    ref = _model(0).to(DEV)
    opts = [torch.optim.Adam(ref[0].parameters(), lr=0.01, eps=1e-8),
            torch.optim.SGD(ref[2].parameters(), lr=0.1, momentum=0.9)]
    x, y = _data()
    for _ in range(5):
        for o in opts:
            o.zero_grad()
        (sum(F.cross_entropy(ref(x[r::2]), y[r::2]) for r in range(2)) / 2).backward()
        for o in opts:
            o.step()
    for n, p in ref.named_parameters():
        torch.testing.assert_close(res[0][0][n], p.detach().cpu(), rtol=1e-4, atol=1e-5)


def _cpu_onebit(tp, steps):
    # the same 1-bit training on CPU thread-ranks (python oracles of pack / unpack-reduce)
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import MomentumUpdater

    m = copy.deepcopy(_CPU_MODELS[tp.rank])
    ps = ColocatedPS(m, MomentumUpdater(0.1, 0.9, 1e-4), tp, bucket_mb=0.004, last_bucket_mb=0.002,
                     plane="collective", compress="onebit", compress_warmup=1)
    x, y = _data(dev="cpu")
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    for _ in range(steps):
        F.cross_entropy(m(xs), ys).backward()
        ps.finish_step()
    ps.synchronize()
    return {n: p.detach().clone() for n, p in m.named_parameters()}


_CPU_MODELS = None


def test_plane_processes_onebit_matches_cpu_oracle():
    global _CPU_MODELS
    res = dist_util.run(_body, 2, ({"compress": "onebit", "compress_warmup": 1}, 6, "momentum",
                                   [_model(0), _model(0)]))
    _CPU_MODELS = [_model(0), _model(0)]
    want = run_loopback(_cpu_onebit, 2, 6)[0]
    for k in want:
        assert torch.equal(res[0][0][k], res[1][0][k])
        torch.testing.assert_close(res[0][0][k], want[k], rtol=1e-4, atol=1e-4)


def test_plane_thread_ranks_gpu():
    # thread-ranks of one process share raw device pointers instead of IPC handles
    models = [_model(0).to(DEV) for _ in range(3)]
    res = run_loopback(_body, 3, {}, 4, "momentum", models)
    ref = _oracle(3, 4, lambda p: torch.optim.SGD(p, lr=0.1, momentum=0.9, weight_decay=1e-4))
    for k, v in ref.items():
        torch.testing.assert_close(res[0][0][k], v, rtol=1e-5, atol=1e-5)


def _resnet_body(tp, steps):
    from ps_amd.models.resnet import prepare_for_mi355x, resnet_tiny
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import MomentumUpdater

    torch.cuda.set_device(0)
    torch.manual_seed(0)
    net = prepare_for_mi355x(resnet_tiny(num_classes=10, fused_bn=True).cuda())
    ps = ColocatedPS(net, MomentumUpdater(0.05, 0.9, 0.0), tp, bucket_mb=0.25, plane="xgmi", timeout_s=60)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(64, 3, 64, 64, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (64,), device="cuda", generator=g)
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    losses = []
    for _ in range(steps):
        loss = F.cross_entropy(net(xs.bfloat16()).float(), ys)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    ps.synchronize()
    torch.cuda.synchronize()
    out = {n: p.detach().float().cpu().clone() for n, p in net.named_parameters() if p.requires_grad}
    ps.close()
    return losses, out


def _bf16_oracle(world, steps, lr=0.05, mom=0.9):
    """The same bf16 ResNet-tiny (same kernels, per-rank BN batches) in ONE process: every
    rank's shard is run in turn with THAT rank's BN buffers (the fused BN kernels shift their
    statistic sums by the running mean, so sharing one set of buffers would perturb the batch
    statistics at the rounding level), the bf16 gradients are summed in fp32 in rank order, and
    the same fused momentum kernel the owners run (step_flat, gscale 1/W) updates an fp32 master
    whose bf16 copy is the next replica -- the plane's arithmetic without the plane (no arenas,
    no IPC, no owner chunks)."""
    from ps_amd.models.resnet import prepare_for_mi355x, resnet_tiny
    from ps_amd.parallel.updaters import MomentumUpdater

    torch.manual_seed(0)
    net = prepare_for_mi355x(resnet_tiny(num_classes=10, fused_bn=True).cuda())
    params = [(n, p) for n, p in net.named_parameters() if p.requires_grad]
    # flat contiguous fp32 masters (conv weights are channels_last; the update is elementwise)
    master = {n: p.detach().float().contiguous() for n, p in params}
    u = MomentumUpdater(lr, mom, 0.0)
    states = {n: u.new_states(v) for n, v in master.items()}
    bufs = [{n: b.detach().clone() for n, b in net.named_buffers()} for _ in range(world)]
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(64, 3, 64, 64, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (64,), device="cuda", generator=g)
    for step in range(steps):
        gsum = {n: torch.zeros_like(v) for n, v in master.items()}
        for r in range(world):
            with torch.no_grad():
                for n, b in net.named_buffers():
                    b.copy_(bufs[r][n])
            for _, p in params:
                p.grad = None
            F.cross_entropy(net(x[r::world].bfloat16()).float(), y[r::world]).backward()
            for n, p in params:
                gsum[n] += p.grad.float()
            with torch.no_grad():
                for n, b in net.named_buffers():
                    bufs[r][n].copy_(b)
        with torch.no_grad():
            for n, p in params:
                out = torch.empty(p.shape, dtype=p.dtype, device=p.device)
                u.step_flat(master[n].view(-1), [s.view(-1) for s in states[n]], gsum[n].view(-1),
                            wout=out.view(-1), gscale=1.0 / world, step=step + 1)
                p.copy_(out)
    return {n: p.detach().float().cpu() for n, p in params}


def _check_weights_tight(res, world, steps):
    """every rank's final weights are bitwise equal, and equal to the
    single-process bf16 oracle up to bf16 rounding of the replica (2 bf16 ulps of |w|, plus an
    absolute floor for weights near 0): a wrong owner chunk or a stale pull moves a whole chunk
    by a learning-rate-sized step and fails this."""
    want = _bf16_oracle(world, steps)
    w0 = res[0][1]
    for r in range(1, world):
        for k in w0:
            assert torch.equal(w0[k], res[r][1][k]), (r, k)
    for k, v in want.items():
        err = (w0[k] - v).abs()
        bound = 2.0 ** -7 * v.abs() + 2e-3
        assert bool((err <= bound).all()), (k, err.max().item(), (err / (v.abs() + 1e-3)).max().item())


def test_plane_processes_resnet_tiny_bf16_trajectory_vs_fp32():
    from ps_amd.models.resnet import resnet_tiny

    world, steps = 4, 6
    res = dist_util.run(_resnet_body, world, (steps,))
    torch.manual_seed(0)
    ref = resnet_tiny(num_classes=10, fused_bn=True)
    for mod in ref.modules():
        if hasattr(mod, "fuse_block"):
            mod.fuse_block = False
    ref = ref.cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(64, 3, 64, 64, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (64,), device="cuda", generator=g)
    lref = []
    for _ in range(steps):
        opt.zero_grad()
        ls = [F.cross_entropy(ref(x[r::world]), y[r::world]) for r in range(world)]
        (sum(ls) / world).backward()
        opt.step()
        lref.append(ls[0].item())
    la = res[0][0]
    for a, b in zip(la, lref):
        assert abs(a - b) < 0.05 * max(1.0, abs(b)), (la, lref)
    assert la[-1] < la[0], la
    _check_weights_tight(res, world, steps)


def _resnet8_body(tp, steps):
    import copy as _copy

    from ps_amd.models.resnet import prepare_for_mi355x, resnet_tiny
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import MomentumUpdater

    torch.cuda.set_device(0)
    torch.manual_seed(0)
    net = prepare_for_mi355x(resnet_tiny(num_classes=10, fused_bn=True).cuda())
    ps = ColocatedPS(net, MomentumUpdater(0.05, 0.9, 0.0), tp, bucket_mb=0.25, plane="xgmi", timeout_s=120)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(64, 3, 64, 64, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (64,), device="cuda", generator=g)
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    losses = []
    for _ in range(steps):
        loss = F.cross_entropy(net(xs.bfloat16()).float(), ys)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    ps.synchronize()
    torch.cuda.synchronize()
    out = {n: p.detach().float().cpu().clone() for n, p in net.named_parameters() if p.requires_grad}
    ps.close()
    return losses, out


def test_world8_processes_bf16_resnet_tiny_tracks_fp32_oracle():
    """W = 8 processes, bf16 ResNet-tiny; the xGMI plane sums the 8 bf16
    pushes in fp32 on the owner -- the trajectory tracks fp32 torch (per-rank BN batches)."""
    from ps_amd.models.resnet import resnet_tiny

    world, steps = 8, 5
    res = dist_util.run(_resnet8_body, world, (steps,), timeout=400)
    torch.manual_seed(0)
    ref = resnet_tiny(num_classes=10, fused_bn=True)
    for mod in ref.modules():
        if hasattr(mod, "fuse_block"):
            mod.fuse_block = False
    ref = ref.cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(64, 3, 64, 64, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (64,), device="cuda", generator=g)
    lref = []
    for _ in range(steps):
        opt.zero_grad()
        ls = [F.cross_entropy(ref(x[r::world]), y[r::world]) for r in range(world)]
        (sum(ls) / world).backward()
        opt.step()
        lref.append(ls[0].item())
    la = res[0][0]
    for a, b in zip(la, lref):
        assert abs(a - b) < 0.05 * max(1.0, abs(b)), (la, lref)
    _check_weights_tight(res, world, steps)


def _mlp8_body(tp, models, steps, reduce_fp32):
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import SimpleUpdater

    m = models[tp.rank]
    ps = ColocatedPS(m, SimpleUpdater(0.5), tp, bucket_mb=0.05, plane="collective", overlap=False,
                     reduce_fp32=reduce_fp32)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(256, 64, generator=g).to(DEV)
    y = torch.randint(0, 8, (256,), generator=g).to(DEV)
    for _ in range(steps):
        F.cross_entropy(m(x[tp.rank::tp.world].bfloat16()).float(), y[tp.rank::tp.world]).backward()
        ps.finish_step()
    ps.synchronize()
    torch.cuda.synchronize()
    return {n: p.detach().float().cpu() for n, p in m.named_parameters()}


def test_world8_collective_fp32_reduction_closer_to_fp32_oracle():
    """The collective plane's reduce_fp32 option: the 8-way reduce-scatter of bf16 buckets runs
    in fp32 (thread-ranks); the bf16 replicas track the fp32 oracle."""
    world, steps = 8, 6

    def mk():
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.Tanh(), torch.nn.Linear(256, 8))

    errs = {}
    ref = mk().to(DEV)
    opt = torch.optim.SGD(ref.parameters(), lr=0.5)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(256, 64, generator=g).to(DEV)
    y = torch.randint(0, 8, (256,), generator=g).to(DEV)
    for _ in range(steps):
        opt.zero_grad()
        (sum(F.cross_entropy(ref(x[r::world]), y[r::world]) for r in range(world)) / world).backward()
        opt.step()
    for fp32 in (False, True):
        models = [mk().to(DEV).bfloat16() for _ in range(world)]
        res = run_loopback(_mlp8_body, world, models, steps, fp32, timeout_s=300)
        errs[fp32] = max((res[0][n] - p.detach().cpu()).abs().max().item() for n, p in ref.named_parameters())
    print("max |w - w_fp32| after 6 steps, bf16 vs fp32 reduction:", errs)
    assert errs[True] < 0.05, errs


def _llama_body(tp, steps, ef_dtype=None, adam1bit=False):
    from ps_amd.models.transformer import LlamaConfig, LlamaForCausalLM
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdamUpdater, OneBitAdamUpdater

    torch.cuda.set_device(0)
    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    model = LlamaForCausalLM(cfg).cuda().to(torch.bfloat16)
    upd = (OneBitAdamUpdater(3e-3, 0.9, 0.95, 1e-8, bias_correction="step", warmup=2) if adam1bit
           else AdamUpdater(3e-3, 0.9, 0.95, 1e-8, bias_correction="step"))
    ps = ColocatedPS(model, upd, tp, bucket_mb=0.05, compress="onebit", compress_warmup=2, plane="xgmi", timeout_s=60,
                     ef_dtype=ef_dtype, onebit_momentum=0.9 if adam1bit else None)
    assert ps.pack_stream is not None  # the pack runs off the backward's stream
    g = torch.Generator(device="cuda").manual_seed(tp.rank)
    ids = torch.randint(0, 64, (4, 64), device="cuda", generator=g)  # a small learnable vocabulary
    losses = []
    for _ in range(steps):
        loss = model(ids, ids)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    ps.synchronize()
    torch.cuda.synchronize()
    out = {n: p.detach().float().cpu().clone() for n, p in model.named_parameters()}
    ps.close()
    return out, losses


@pytest.mark.parametrize("ef_dtype", [None, torch.bfloat16])
def test_tiny_llama_onebit_two_processes_on_the_plane(ef_dtype):
    """the Llama config's 1-bit push (owner decodes the W packed pushes inside
    the fused Adam kernel) with 2 processes: replicas stay identical, the loss falls -- with the
    error feedback in fp32 and in bf16 (the 8B bench's choice), packed on the pack stream."""
    res = dist_util.run(_llama_body, 2, (25, ef_dtype))
    for k in res[0][0]:
        assert torch.equal(res[0][0][k], res[1][0][k])
    for _, losses in res:
        assert sum(losses[-5:]) / 5 < 0.8 * sum(losses[:5]) / 5, losses


def test_tiny_llama_onebit_adam_two_processes_on_the_plane():
    """1-bit Adam on the plane (worker momentum packed on the pack stream, owners' Adam with beta1 = 0
    and a frozen variance after 2 warm-up rounds): replicas identical, the loss falls."""
    res = dist_util.run(_llama_body, 2, (25, torch.bfloat16, True))
    for k in res[0][0]:
        assert torch.equal(res[0][0][k], res[1][0][k])
    for _, losses in res:
        assert sum(losses[-5:]) / 5 < 0.8 * sum(losses[:5]) / 5, losses


def test_plane_processes_ipc_event_round_end_matches_oracle(monkeypatch):
    """PS_AMD_PLANE_IPC_EVENTS=1: owners publish a serve when it is ENQUEUED and every peer's pull
    waits on the owner's inter-process event on the device (csrc/plane.cpp enable_ipc_events).
    BSP at W = 2 and 4 and SSP(1) still match the fp32 oracles exactly as the host-observed
    round end does."""
    monkeypatch.setenv("PS_AMD_PLANE_IPC_EVENTS", "1")
    for world in (2, 4):
        res = dist_util.run(_body, world, ({}, 5))
        ref = _oracle(world, 5, lambda p: torch.optim.SGD(p, lr=0.1, momentum=0.9, weight_decay=1e-4))
        for k, v in ref.items():
            torch.testing.assert_close(res[0][0][k], v, rtol=1e-5, atol=1e-5)
            for r in range(1, world):
                assert torch.equal(res[0][0][k], res[r][0][k])
