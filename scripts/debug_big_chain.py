"""Two layer-3 bottlenecks (the test_conv_big_gpu chain) run once per process; saves the forward
output and every gradient to OUT so runs under different PS_AMD_CONV_BIG* settings compare.
usage: python scripts/debug_big_chain.py OUT.pt  |  python scripts/debug_big_chain.py --cmp A.pt B.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(out):
    import torch.nn as nn

    from ps_amd.models.resnet import Bottleneck, prepare_for_mi355x
    from ps_amd.ops import convgemm as cg

    torch.manual_seed(4)
    n, h = 400, 14
    a = nn.Sequential(Bottleneck(1024, 256), Bottleneck(1024, 256))
    for m in a.modules():
        if isinstance(m, nn.BatchNorm2d):
            nn.init.uniform_(m.weight, 0.5, 1.5)
            nn.init.uniform_(m.bias, -0.2, 0.2)
    fp32 = os.environ.get("FP32") == "1"
    a = a.cuda() if fp32 else prepare_for_mi355x(a.cuda())
    if fp32 or os.environ.get("UNFUSED") == "1":
        for blk in a:
            blk.fuse_block = False
    x = torch.randn(n, 1024, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    if fp32:
        x = x.float()
    xa = x.clone().requires_grad_()
    with cg.deferred_bn_counters():
        a[0]._defer_out = os.environ.get("DEFER", "1") == "1"
        y = a(xa)
    g = torch.randn(y.shape, device="cuda", generator=torch.Generator(device="cuda").manual_seed(9)).bfloat16()
    y.backward(g.to(y.dtype).contiguous(memory_format=torch.channels_last))
    d = {"y": y.detach().float().cpu(), "dx": xa.grad.float().cpu()}
    for name, p in a.named_parameters():
        d[name] = p.grad.float().cpu()
    torch.save(d, out)
    print("saved", out, dict(cg.FOLD_STATS))


def cmp(pa, pb):
    a, b = torch.load(pa), torch.load(pb)
    for k in a:
        e = ((a[k] - b[k]).norm() / b[k].norm().clamp_min(1e-12)).item()
        print(f"{k:40s} {e:.4f}")


if __name__ == "__main__":
    if sys.argv[1] == "--cmp":
        cmp(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
