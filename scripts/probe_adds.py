"""GPU probe: where do the per-step fp32 elementwise adds of the ResNet-50 PS step come from?

Runs a few steps of the bench configuration (smaller batch; the op count per step does not depend
on it), profiles one step with torch.profiler and prints every aten add-like op with its count,
input shapes and the Python stack that issued it.
"""
import sys

import torch
import torch.nn.functional as F
from torch.profiler import ProfilerActivity, profile

from ps_amd.models.resnet import prepare_for_mi355x, resnet50
from ps_amd.parallel.colocated import ColocatedPS
from ps_amd.parallel.updaters import MomentumUpdater


def main(batch=64):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = prepare_for_mi355x(resnet50().to(dev))
    x = torch.randn(batch, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device=dev)
    ps = ColocatedPS(m, MomentumUpdater(0.1, 0.9, 5e-5), bucket_mb=25, last_bucket_mb=2)

    def step():
        F.cross_entropy(m(x).float(), y).backward()
        ps.finish_step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True, group_by_stack_n=6)
    rows = [e for e in ka if "add" in e.key and e.key.startswith("aten::")]
    rows.sort(key=lambda e: -e.count)
    for e in rows:
        print(f"{e.count:5d}  {e.key}  shapes={e.input_shapes}")
        for fr in (e.stack or [])[:6]:
            print(f"         {fr}")
    print("--- device kernels with 'add' in the name")
    kern = {}
    for e in prof.events():
        if e.device_type == torch.autograd.DeviceType.CUDA and "add" in e.name.lower():
            kern[e.name[:120]] = kern.get(e.name[:120], 0) + 1
    for k, v in sorted(kern.items(), key=lambda kv: -kv[1]):
        print(f"{v:5d}  {k}")
    sys.stdout.flush()


if __name__ == "__main__":
    main()
