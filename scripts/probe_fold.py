"""Chained fused bottlenecks: input/param gradient error vs the module path, fold on / off."""
import copy
import os

import torch
import torch.nn as nn

from ps_amd.models.resnet import Bottleneck, prepare_for_mi355x
from ps_amd.ops import convgemm as cg
from ps_amd.ops.bn import BatchNormAct2d

torch.manual_seed(1)
ds = nn.Sequential(nn.Conv2d(128, 256, 1, stride=2, bias=False), BatchNormAct2d(256, act="none"))
a = nn.Sequential(Bottleneck(128, 64, 2, ds), Bottleneck(256, 64), Bottleneck(256, 64))
for m in a.modules():
    if isinstance(m, nn.BatchNorm2d):
        nn.init.uniform_(m.weight, 0.5, 1.5)
        nn.init.uniform_(m.bias, -0.2, 0.2)
b = copy.deepcopy(a)
for blk in b:
    blk.fuse_block = False
a, b = prepare_for_mi355x(a.cuda()), prepare_for_mi355x(b.cuda())
x = torch.randn(4, 128, 17, 17, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
gw = torch.randn(4, 256, 9, 9, device="cuda")


def run(model, ctx=True):
    model.zero_grad()
    xi = x.clone().requires_grad_()
    if ctx:
        with cg.deferred_bn_counters():
            y = model[2](model[1](model[0](xi)))
    else:
        y = model[2](model[1](model[0](xi)))
    (y.float() * gw).sum().backward()
    return xi.grad.float().clone(), {n: p.grad.float().clone() for n, p in model.named_parameters()}


def rel(u, v):
    return ((u - v).norm() / v.norm().clamp_min(1e-12)).item()


c = copy.deepcopy(b).float()  # fp32 module path: the arbiter


def run32():
    c.zero_grad()
    xi = x.float().clone().requires_grad_()
    y = c[2](c[1](c[0](xi)))
    (y * gw).sum().backward()
    return xi.grad.clone(), {n: p.grad.float().clone() for n, p in c.named_parameters()}


g32, p32 = run32()
gb, pb = run(b)
print("module-bf16 vs fp32: xgrad rel", round(rel(gb, g32), 4), "worst",
      [(k, round(e, 4)) for e, k in sorted(((rel(pb[k], p32[k]), k) for k in p32), reverse=True)[:3]], flush=True)
for label, env, ctx in [("fold", "1", True), ("nofold", "0", True), ("noctx", "1", False)]:
    os.environ["PS_AMD_FOLD_BN3"] = env
    u0 = cg.FOLD_STATS["used"]
    ga, pa = run(a, ctx)
    worst = sorted(((rel(pa[k], pb[k]), k) for k in pb), reverse=True)[:4]
    print(label, "vs fp32: xgrad rel", round(rel(ga, g32), 4), "worst",
          [(k, round(e, 4)) for e, k in sorted(((rel(pa[k], p32[k]), k) for k in p32), reverse=True)[:3]])
    print(label, "used", cg.FOLD_STATS["used"] - u0, "xgrad rel", round(rel(ga, gb), 4), "worst params",
          [(k, round(e, 4)) for e, k in worst], flush=True)
