"""Is the whole-network gradient gap of the bf16 production ResNet-50 vs fp32 (~22 % relative per
conv weight at bn3.weight = 0.1, tests/test_resnet_routes_gpu.py) the kernels or the problem's
conditioning?  Control: a DIFFERENT bf16 implementation -- the plain torch module path in bf16
(MIOpen convolutions, torch BatchNorm) -- against the same fp32 oracle, and a perturbation control:
the fp32 oracle against itself with the input perturbed by 2^-9 relative noise (one bf16 rounding).
usage: python scripts/diag_resnet_control.py [B S G3]"""
import os
import sys
import types

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from ps_amd.models.resnet import prepare_for_mi355x, resnet50
    from tests.test_resnet_routes_gpu import _gemm_conv, _rel, _warm_bn3

    B, S, G3 = (int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (256, 224, 0.1)
    torch.manual_seed(0)
    base = resnet50(num_classes=1000, fused_bn=True)
    _warm_bn3(base, G3)
    with torch.no_grad():
        for n, p in base.named_parameters():
            if ".bn" not in n and "downsample.1" not in n and not n.startswith("bn1"):
                p.copy_(p.bfloat16().float())
    sd = base.state_dict()

    def oracle():
        r = resnet50(num_classes=1000, fused_bn=False)
        r.load_state_dict(sd)
        r = r.cuda()
        for mod in r.modules():
            if isinstance(mod, torch.nn.Conv2d):
                mod.forward = types.MethodType(_gemm_conv, mod)
        return r

    gen = torch.Generator(device="cuda").manual_seed(1)
    xr = torch.randn(B, 3, S, S, device="cuda", generator=gen)
    y = torch.randint(0, 1000, (B,), device="cuda", generator=gen)
    grads = {}
    # fp32 oracle
    ref = oracle()
    F.cross_entropy(ref(xr), y).backward()
    grads["fp32"] = {n: p.grad.detach().float().clone() for n, p in ref.named_parameters()}
    del ref
    # fp32 oracle, input perturbed by one bf16 rounding's worth of noise
    ref = oracle()
    xp = xr * (1 + 2 ** -9 * torch.randn(xr.shape, device="cuda", generator=gen))
    F.cross_entropy(ref(xp), y).backward()
    grads["fp32_perturbed"] = {n: p.grad.detach().float().clone() for n, p in ref.named_parameters()}
    del ref
    # bf16 plain module path (MIOpen + torch BN)
    mod = resnet50(num_classes=1000, fused_bn=False)
    mod.load_state_dict(sd)
    mod = prepare_for_mi355x(mod.cuda())
    F.cross_entropy(mod(xr.contiguous(memory_format=torch.channels_last).bfloat16()).float(), y).backward()
    grads["bf16_modules"] = {n: p.grad.detach().float().clone() for n, p in mod.named_parameters()}
    del mod
    # bf16 production path
    net = resnet50(num_classes=1000, fused_bn=True)
    net.load_state_dict(sd)
    net = prepare_for_mi355x(net.cuda())
    F.cross_entropy(net(xr.contiguous(memory_format=torch.channels_last).bfloat16()).float(), y).backward()
    grads["bf16_production"] = {n: p.grad.detach().float().clone() for n, p in net.named_parameters()}
    del net
    torch.cuda.empty_cache()

    def summary(a, b):
        out = {}
        for n in grads[b]:
            cat = "fc" if n.startswith("fc") else ("bn" if ("bn" in n or "downsample.1" in n) else "conv")
            out.setdefault(cat, []).append(_rel(grads[a][n], grads[b][n]))
        return "  ".join(f"{c} mean {sum(v) / len(v):.4f} max {max(v):.4f}" for c, v in out.items())

    print(f"B={B} S={S} bn3.weight={G3}; relative gradient error per parameter vs the reference:", flush=True)
    for a, b in (("fp32_perturbed", "fp32"), ("bf16_modules", "fp32"), ("bf16_production", "fp32"),
                 ("bf16_production", "bf16_modules")):
        print(f"  {a:16s} vs {b:13s} {summary(a, b)}", flush=True)


if __name__ == "__main__":
    main()
