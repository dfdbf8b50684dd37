"""GPU probe: ResNet-50 step time under different configurations (one JSON line each).

  baseline   plain torch: bf16 model + torch.optim.SGD(foreach) -- no PS
  ps         ColocatedPS (fused HIP momentum SGD on the fp32 master shard)
"""
import argparse
import json
import time

import torch
import torch.nn.functional as F

from ps_amd.models.resnet import resnet50, prepare_for_mi355x
from ps_amd.parallel.colocated import ColocatedPS
from ps_amd.parallel.updaters import MomentumUpdater


def run(mode, batch, bn_fp32, steps, warmup, cl=True):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = resnet50().to(dev)
    if cl:
        m = prepare_for_mi355x(m, bn_fp32=bn_fp32)
    else:
        m = m.to(torch.bfloat16)
    x = torch.randn(batch, 3, 224, 224, device=dev).to(torch.bfloat16)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device=dev)
    if mode == "ps":
        ps = ColocatedPS(m, MomentumUpdater(0.1, 0.9, 5e-5), bucket_mb=25, last_bucket_mb=2)

        def step():
            F.cross_entropy(m(x).float(), y).backward()
            ps.finish_step()
    else:
        opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5, foreach=True)

        def step():
            opt.zero_grad(set_to_none=True)
            F.cross_entropy(m(x).float(), y).backward()
            opt.step()
    t0 = time.perf_counter()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    rec = dict(mode=mode, batch=batch, bn_fp32=bn_fp32, channels_last=cl, ms=el / steps * 1e3,
               img_s=batch * steps / el, warmup_s=round(tw, 1))
    print(json.dumps(rec), flush=True)
    del m, x
    torch.cuda.empty_cache()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="ps:256:1,baseline:256:1,ps:256:0,ps:128:1,ps:512:1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--benchmark", type=int, default=1)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    for c in a.configs.split(","):
        mode, b, bn = c.split(":")
        try:
            run(mode, int(b), bool(int(bn)), a.steps, a.warmup)
        except Exception as e:  # keep probing other configs
            print(json.dumps(dict(config=c, error=repr(e)[:300])), flush=True)
