"""Weight gradients on the side stream (ps_amd/ops/side_stream.py) vs everything on the compute
stream: same gradients for a fused ResNet, same trajectory through the co-located PS (whose
bucket landing moves onto the side stream), and the micro-batch accumulation fallback."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(seed=0):
    from ps_amd.models.resnet import prepare_for_mi355x, resnet_tiny

    torch.manual_seed(seed)
    m = resnet_tiny(num_classes=10)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
    return prepare_for_mi355x(m.to(DEV))


def _batch(n=16, s=64, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(n, 3, s, s, device=DEV, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    return x, torch.randint(0, 10, (n,), device=DEV, generator=g)


def _deterministic(monkeypatch):
    """Every weight gradient on the in-house kernels (fixed-order split-K reductions): the
    side-stream run must then be BITWISE equal to the single-stream run."""
    from ps_amd.ops import convgemm as cg

    monkeypatch.setattr(cg, "WGRAD3X3_MIN_C", 64)


def test_side_stream_grads_match_single_stream(monkeypatch):
    from ps_amd.ops import side_stream as side

    _deterministic(monkeypatch)
    base = _model()
    x, y = _batch()
    grads = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PS_AMD_WGRAD_STREAM", flag)
        m = copy.deepcopy(base)
        F.cross_entropy(m(x).float(), y).backward()
        # no explicit synchronize / join here: the end-of-backward callback must order the reads
        grads[flag] = {n: p.grad.clone() for n, p in m.named_parameters()}
    assert side.active(torch.device(DEV)) is not None
    for n, g in grads["0"].items():
        assert torch.equal(grads["1"][n], g), n


def test_colocated_ps_trajectory_with_side_stream(monkeypatch):
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import MomentumUpdater

    _deterministic(monkeypatch)
    base = _model(1)
    batches = [_batch(seed=i) for i in range(4)]
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PS_AMD_WGRAD_STREAM", flag)
        m = copy.deepcopy(base)
        ps = ColocatedPS(m, MomentumUpdater(lr=0.05, momentum=0.9), bucket_mb=0.5, last_bucket_mb=0.1)
        losses = []
        for x, y in batches:
            loss = F.cross_entropy(m(x).float(), y)
            loss.backward()
            ps.finish_step()
            losses.append(loss.item())
        ps.synchronize()
        out[flag] = (losses, {n: ps.weight(n).float().clone() for n in ps.params})
        ps.close()
    la, wa = out["1"]
    lb, wb = out["0"]
    assert la == lb
    for n in wb:
        assert torch.equal(wa[n], wb[n]), n


def test_accumulation_falls_back_to_compute_stream(monkeypatch):
    """A second backward into existing .grad must not run on the side stream (AccumulateGrad
    adds on the compute stream); the two-micro-batch sum matches one backward of both."""
    _deterministic(monkeypatch)
    monkeypatch.setenv("PS_AMD_WGRAD_STREAM", "1")
    base = _model(2)
    x, y = _batch(seed=5)
    m = copy.deepcopy(base)
    for i in range(2):
        F.cross_entropy(m(x[i * 8:(i + 1) * 8]).float(), y[i * 8:(i + 1) * 8], reduction="sum").backward()
    acc = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    monkeypatch.setenv("PS_AMD_WGRAD_STREAM", "0")
    r = copy.deepcopy(base)
    for i in range(2):
        F.cross_entropy(r(x[i * 8:(i + 1) * 8]).float(), y[i * 8:(i + 1) * 8], reduction="sum").backward()
    for n, p in r.named_parameters():
        assert torch.equal(acc[n], p.grad.float()), n
