"""Co-located PS on one MI355X: the fused HIP server path must reproduce torch.optim exactly
(fp32 model) and train a bf16 model (fp32 master) to the same loss trajectory."""
import copy

import pytest
import torch
import torch.nn.functional as F

from ps_amd.parallel.colocated import ColocatedPS
from ps_amd.parallel.updaters import AdamUpdater, MomentumUpdater

pytestmark = pytest.mark.gpu


def _mlp():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(784, 150), torch.nn.ReLU(), torch.nn.Linear(150, 50),
                               torch.nn.ReLU(), torch.nn.Linear(50, 10)).cuda()


@pytest.mark.parametrize("upd", ["momentum", "adam"])
@pytest.mark.parametrize("staleness", [0, 1])
def test_ps_matches_torch_fp32(upd, staleness):
    m = _mlp()
    ref = copy.deepcopy(m)
    if upd == "momentum":
        u = MomentumUpdater(0.05, 0.9, 1e-4)
        opt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    else:
        u = AdamUpdater(1e-3, 0.9, 0.999, 1e-8, bias_correction="step")
        opt = torch.optim.Adam(ref.parameters(), lr=1e-3, betas=(0.9, 0.999), eps=1e-8)
    ps = ColocatedPS(m, u, bucket_mb=0.05, last_bucket_mb=0.01, staleness=staleness)
    x = torch.randn(256, 784, device="cuda")
    y = torch.randint(0, 10, (256,), device="cuda")
    if staleness == 0:
        for _ in range(5):
            F.cross_entropy(m(x), y).backward()
            ps.finish_step()
            opt.zero_grad()
            F.cross_entropy(ref(x), y).backward()
            opt.step()
        ps.synchronize()
        torch.cuda.synchronize()
        for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
            torch.testing.assert_close(p, q, rtol=1e-4, atol=1e-5)
    else:
        # SSP(1): step t uses weights version t-1 -> the loss still decreases
        losses = []
        for _ in range(20):
            l = F.cross_entropy(m(x), y)
            l.backward()
            ps.finish_step()
            losses.append(l.item())
        assert losses[-1] < losses[0]


def test_ps_bf16_replica_fp32_master():
    m = _mlp()
    ref = copy.deepcopy(m)
    mb = copy.deepcopy(m).to(torch.bfloat16)
    ps = ColocatedPS(mb, MomentumUpdater(0.05, 0.9), bucket_mb=0.1)
    opt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    x = torch.randn(256, 784, device="cuda")
    y = torch.randint(0, 10, (256,), device="cuda")
    for _ in range(10):
        F.cross_entropy(mb(x.bfloat16()).float(), y).backward()
        ps.finish_step()
        opt.zero_grad()
        F.cross_entropy(ref(x), y).backward()
        opt.step()
    torch.cuda.synchronize()
    lb = F.cross_entropy(mb(x.bfloat16()).float(), y).item()
    lr_ = F.cross_entropy(ref(x), y).item()
    assert abs(lb - lr_) < 0.05
    # master shard stays fp32 and matches the replica after rounding
    for b, bk in enumerate(ps.reg.buckets):
        lo, hi = bk.owner_range(0)
        rep = ps.wbuf[bk.group][ps.wslot][lo:hi].float()
        torch.testing.assert_close(rep, ps.master[b].bfloat16().float())


def test_ps_clip_norm():
    m = _mlp()
    ref = copy.deepcopy(m)
    ps = ColocatedPS(m, MomentumUpdater(0.1, 0.0), clip_norm=0.5, bucket_mb=0.05)
    opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    x = torch.randn(64, 784, device="cuda") * 10
    y = torch.randint(0, 10, (64,), device="cuda")
    for _ in range(3):
        F.cross_entropy(m(x), y).backward()
        ps.finish_step()
        opt.zero_grad()
        F.cross_entropy(ref(x), y).backward()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 0.5)
        opt.step()
    torch.cuda.synchronize()
    for p, q in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-4, atol=1e-5)


def test_ps_linear_grads_land_in_bucket_and_match():
    """Tiny Llama on the colocated PS: with PsLinear (ops/linear.py) the projection weights'
    gradients are written into the bound gradient slot (p.grad IS the bucket view, nothing left
    for the landing to copy) and the trained weights track an nn.Linear-only twin step for step."""
    from ps_amd.models.transformer import LlamaConfig, LlamaForCausalLM
    from ps_amd.ops.linear import PsLinear

    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    a = LlamaForCausalLM(cfg).cuda()
    b = copy.deepcopy(a)
    for mod in b.modules():  # the twin: plain nn.Linear forwards
        if isinstance(mod, PsLinear):
            mod.forward = lambda x, _m=mod: F.linear(x, _m.weight, _m.bias)
    pa = ColocatedPS(a, AdamUpdater(1e-3, 0.9, 0.95, 1e-8, bias_correction="step"), bucket_mb=0.05)
    pb = ColocatedPS(b, AdamUpdater(1e-3, 0.9, 0.95, 1e-8, bias_correction="step"), bucket_mb=0.05)
    ids = torch.randint(0, cfg.vocab, (2, 64), device="cuda")
    in_place = []
    for step in range(4):
        la = a(ids, ids)
        la.backward()
        if step == 0:
            for n, p in a.named_parameters():
                if n.endswith(("wqkv.weight", "wo.weight", "w13.weight", "w2.weight", "lm_head.weight")):
                    v = pa._view(pa.gbuf, pa.gslot, n)
                    in_place.append(p.grad is not None and p.grad.data_ptr() == v.data_ptr())
        pa.finish_step()
        lb = b(ids, ids)
        lb.backward()
        pb.finish_step()
        torch.testing.assert_close(la.float(), lb.float(), rtol=2e-2, atol=2e-2)
    assert in_place and all(in_place), in_place
    pa.synchronize()
    pb.synchronize()
    torch.cuda.synchronize()
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        torch.testing.assert_close(p.float(), q.float(), rtol=2e-2, atol=2e-3)
