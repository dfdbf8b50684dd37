"""Localise a gap between the bf16 production ResNet-50 and the fp32 oracle
(tests/test_resnet_routes_gpu.py): per-block forward outputs, logits, loss, then per-parameter
gradient errors grouped by block, at the batch / image sizes given.
usage: python scripts/diag_resnet_vs_fp32.py B S G3 [B S G3 ...]   (G3 < 0: random BN affine everywhere;
else default BN init with bn3.weight = G3)"""
import os
import sys
import types

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from ps_amd.models.resnet import prepare_for_mi355x, resnet50
    from tests.test_resnet_routes_gpu import _gemm_conv, _randomise_bn, _rel

    args = [float(a) for a in sys.argv[1:]] or [1024, 224, -1]
    for B, S, G3 in zip(args[0::3], args[1::3], args[2::3]):
        B, S = int(B), int(S)
        torch.manual_seed(0)
        base = resnet50(num_classes=1000, fused_bn=True)
        if G3 < 0:
            _randomise_bn(base)
        else:
            with torch.no_grad():
                for n, p in base.named_parameters():
                    if n.endswith("bn3.weight"):
                        p.fill_(G3)
        with torch.no_grad():
            for n, p in base.named_parameters():
                if ".bn" not in n and "downsample.1" not in n and not n.startswith("bn1"):
                    p.copy_(p.bfloat16().float())
        ref = resnet50(num_classes=1000, fused_bn=False)
        ref.load_state_dict(base.state_dict())
        ref = ref.cuda()
        for mod in ref.modules():
            if isinstance(mod, torch.nn.Conv2d):
                mod.forward = types.MethodType(_gemm_conv, mod)
        net = prepare_for_mi355x(base.cuda())
        gen = torch.Generator(device="cuda").manual_seed(1)
        xr = torch.randn(B, 3, S, S, device="cuda", generator=gen)
        x = xr.contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (B,), device="cuda", generator=gen)
        outs = {}

        def hook(tag, name):
            def f(mod, inp, out):
                outs[(tag, name)] = out.detach().float().clone()
            return f

        hs = []
        lp = net(x.bfloat16()).float()
        lr = ref(xr)
        print(f"=== B={B} S={S} G3={G3}: logits rel err {_rel(lp, lr):.4f} loss {F.cross_entropy(lp, y).item():.5f} "
              f"vs {F.cross_entropy(lr, y).item():.5f}", flush=True)
        for h in hs:
            h.remove()
        F.cross_entropy(lp, y).backward()
        F.cross_entropy(lr, y).backward()
        rp = dict(ref.named_parameters())
        rows = {}
        for n, p in net.named_parameters():
            blk = ".".join(n.split(".")[:2]) if n.startswith("layer") else n.split(".")[0]
            rows.setdefault(blk, []).append((round(_rel(p.grad, rp[n].grad), 4), n.split(".", 2)[-1]))
        for blk, es in rows.items():
            conv = [e for e, n in es if "conv" in n or "downsample.0" in n]
            bnw = [e for e, n in es if n.endswith("weight") and ("bn" in n or "downsample.1" in n)]
            bnb = [e for e, n in es if n.endswith("bias")]
            f = lambda v: f"{max(v):.3f}" if v else "-"
            print(f"  grad {blk:10s} conv max {f(conv)}  bn.w max {f(bnw)}  bn.b max {f(bnb)}", flush=True)
        del net, ref, base, x, xr, lp, lr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
