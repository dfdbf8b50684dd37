"""Gradient landing in the co-located PS (parallel/colocated.py): adopted gradients copied into
the flat buckets with one multi-tensor copy, channels_last conv keys, zero-fill of keys that got
no gradient, micro-batch accumulation -- checked against plain SGD on a copy of the model."""
import copy

import torch
import torch.nn as nn
import torch.nn.functional as F


class _Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.c3 = nn.Conv2d(8, 16, 3, padding=1, bias=False)
        self.c1 = nn.Conv2d(16, 8, 1)
        self.fc = nn.Linear(8, 5)
        self.unused = nn.Linear(3, 3)  # never in the graph: its bucket region must be zero

    def forward(self, x):
        x = F.relu(self.c1(F.relu(self.c3(x))))
        return self.fc(x.mean((2, 3)))


def _setup():
    torch.manual_seed(0)
    m = _Net().to(memory_format=torch.channels_last)
    ref = copy.deepcopy(m)
    x = torch.randn(6, 8, 5, 5).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 5, (6,))
    return m, ref, x, y


def test_landing_matches_sgd_and_keeps_channels_last():
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import SimpleUpdater

    m, ref, x, y = _setup()
    ps = ColocatedPS(m, SimpleUpdater(0.05), bucket_mb=0.002, last_bucket_mb=0.001)
    assert "c3.weight" in ps.cl_keys and "c1.weight" not in ps.cl_keys
    assert m.c3.weight.is_contiguous(memory_format=torch.channels_last)
    opt = torch.optim.SGD(ref.parameters(), lr=0.05)
    for step in range(3):
        F.cross_entropy(m(x), y).backward()
        ps.finish_step()
        opt.zero_grad()
        F.cross_entropy(ref(x), y).backward()
        opt.step()
        for (n, p), q in zip(m.named_parameters(), ref.parameters()):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6, msg=n)
    # the unused key's gradient region is zero in every slot
    for slot in range(ps.nslots):
        assert torch.count_nonzero(ps._view(ps.gbuf, slot, "unused.weight")) == 0


def test_landing_with_microbatch_accumulation():
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import SimpleUpdater

    m, ref, x, y = _setup()
    ps = ColocatedPS(m, SimpleUpdater(0.05), bucket_mb=0.002, last_bucket_mb=0.001, average=True)
    opt = torch.optim.SGD(ref.parameters(), lr=0.05)
    for _ in range(2):
        ps.accumulating = True
        F.cross_entropy(m(x[:3]), y[:3]).backward()
        ps.accumulating = False
        F.cross_entropy(m(x[3:]), y[3:]).backward()
        ps.finish_step()
        opt.zero_grad()
        F.cross_entropy(ref(x[:3]), y[:3]).backward()
        F.cross_entropy(ref(x[3:]), y[3:]).backward()
        opt.step()
    for (n, p), q in zip(m.named_parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6, msg=n)


def test_stride2_phase_weights_gather_matches_indexing():
    """ops/convgemm._phase_weights (one cached gather) == per-phase advanced indexing."""
    import torch

    from ps_amd.ops.convgemm import _phase_weights

    w = torch.randn(16, 8, 3, 3).contiguous(memory_format=torch.channels_last)
    got = _phase_weights(w)
    i = 0
    for a in (0, 1):
        for b in (0, 1):
            kh = [1] if a == 0 else [2, 0]
            kw = [1] if b == 0 else [2, 0]
            ref = w[:, :, kh][:, :, :, kw].permute(1, 2, 3, 0).reshape(w.shape[1], -1)
            assert torch.equal(got[i], ref) and got[i].is_contiguous()
            i += 1
