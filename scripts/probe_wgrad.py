"""Weight-gradient kernels (csrc/kernels/convgemm.hip conv_wgrad) on every ResNet-50 1x1 / 3x3
shape at the bench batch vs MIOpen (convolution_backward, weight only): time, TF/s and the
bandwidth of the minimum HBM traffic (dz + x read once, dW written once).

    python scripts/probe_wgrad.py [--batch 1024] [--it 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402
from ps_amd.ops.convgemm import geo  # noqa: E402

SHAPES = [  # H (input), Cin, Cout, ks, stride, calls per step
    (56, 64, 64, 1, 1, 1), (56, 256, 64, 1, 1, 2), (56, 64, 256, 1, 1, 4), (56, 64, 64, 3, 1, 3),
    (56, 256, 128, 1, 1, 1), (28, 512, 128, 1, 1, 3), (28, 128, 512, 1, 1, 4), (56, 256, 512, 1, 2, 1),
    (56, 128, 128, 3, 2, 1), (28, 128, 128, 3, 1, 3),
    (28, 512, 256, 1, 1, 1), (14, 1024, 256, 1, 1, 5), (14, 256, 1024, 1, 1, 6), (28, 512, 1024, 1, 2, 1),
    (28, 256, 256, 3, 2, 1), (14, 256, 256, 3, 1, 5),
    (14, 1024, 512, 1, 1, 1), (7, 2048, 512, 1, 1, 2), (7, 512, 2048, 1, 1, 3), (14, 1024, 2048, 1, 2, 1),
    (14, 512, 512, 3, 2, 1), (7, 512, 512, 3, 1, 2)]


def bench(fn, it):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--it", type=int, default=5)
    ap.add_argument("--miopen", type=int, default=1)
    ap.add_argument("--only", default="", help="comma list of shape substrings, e.g. '3x3 56x56,3x3 28x28'")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    nat = native()
    n = a.batch
    tot = {"ours": 0.0, "miopen": 0.0}
    for h, ci, co, ks, s, calls in SHAPES:
        name = f"{ks}x{ks} {h}x{h} {ci}->{co} s{s}"
        if a.only and not any(o in name for o in a.only.split(",")):
            continue
        g = geo(h, h, ks, s, ks // 2)
        oh = g[2]
        M = n * oh * oh
        x = torch.randn(n, ci, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        dz = torch.randn(n, co, oh, oh, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, ci)
        dz2 = dz.permute(0, 2, 3, 1).reshape(-1, co)
        flops = 2.0 * M * co * ks * ks * ci
        byts = 2.0 * (x.numel() + dz.numel()) + 2.0 * co * ci * ks * ks
        rec = {"shape": f"{ks}x{ks} {h}x{h} {ci}->{co} s{s}", "calls": calls}
        t = bench(lambda: nat.conv_wgrad(dz2, x2, g), a.it)
        rec.update(us=round(t, 1), tflops=round(flops / t / 1e6, 1), hbm_tbps=round(byts / t / 1e6, 2))
        tot["ours"] += calls * t
        if a.miopen:
            w = torch.empty(co, ci, ks, ks, device="cuda", dtype=torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            tm = bench(lambda: torch.ops.aten.convolution_backward(dz, x, w, None, [s, s], [ks // 2] * 2, [1, 1], False,
                                                                   [0, 0], 1, [False, True, False]), a.it)
            rec.update(miopen_us=round(tm, 1), miopen_tflops=round(flops / tm / 1e6, 1))
            tot["miopen"] += calls * tm
        print(json.dumps(rec), flush=True)
        del x, dz, x2, dz2
        torch.cuda.empty_cache()
    print(json.dumps({"step_total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
