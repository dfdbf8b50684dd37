"""3x3 convolutions of the ResNet-50 bottleneck: the in-house implicit-GEMM kernels
(csrc/kernels/convgemm.hip) vs MIOpen (torch conv2d / convolution_backward, channels_last bf16)
at the bench batch, per direction.  Data gradient of a stride-1 3x3 conv = the same forward GEMM
over dz with the spatially flipped, channel-transposed weight.

    python scripts/probe_conv3x3.py [--batch 1024] [--it 10]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402
from ps_amd.ops.convgemm import geo  # noqa: E402

SHAPES = [  # H (input), C, stride
    (56, 64, 1), (56, 128, 2), (28, 128, 1), (28, 256, 2), (14, 256, 1), (14, 512, 2), (7, 512, 1)]


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
    ap.add_argument("--it", type=int, default=10)
    ap.add_argument("--miopen", type=int, default=1)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True  # as bench.py: MIOpen find picks its best solver
    nat = native()
    n = a.batch
    tot = {"miopen": 0.0, "ours": 0.0}
    for h, c, s in SHAPES:
        g = geo(h, h, 3, s, 1)
        oh = g[2]
        M = n * oh * oh
        flops = 2.0 * M * c * 9 * c
        x = torch.randn(n, c, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(c, c, 3, 3, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        dz = torch.randn(n, c, oh, oh, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        rec = {"shape": f"3x3 {h}x{h} {c} s{s}", "M": M}
        if a.miopen:
            rec["miopen_fwd_us"] = bench(lambda: F.conv2d(x, w, None, s, 1), a.it)
            rec["miopen_dgrad_us"] = bench(lambda: torch.ops.aten.convolution_backward(
                dz, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]), a.it)
            rec["miopen_wgrad_us"] = bench(lambda: torch.ops.aten.convolution_backward(
                dz, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]), a.it)
        else:
            rec["miopen_fwd_us"] = rec["miopen_dgrad_us"] = rec["miopen_wgrad_us"] = 0.0
        x2 = x.permute(0, 2, 3, 1).reshape(-1, c)
        dz2 = dz.permute(0, 2, 3, 1).reshape(-1, c)
        wm = w.permute(0, 2, 3, 1).reshape(c, 9 * c)
        coef = torch.cat([torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda")])
        ksh = torch.zeros(c, device="cuda")
        rec["ours_fwd_us"] = bench(lambda: nat.conv_gemm(x2, wm, g, coef, 1, None, ksh), a.it)
        rec["ours_fwd_nopro_us"] = bench(lambda: nat.conv_gemm(x2, wm, g, None, 0), a.it)
        if s == 1:
            wt = w.flip(2, 3).transpose(0, 1).permute(0, 2, 3, 1).reshape(c, 9 * c).contiguous()
            rec["ours_dgrad_us"] = bench(lambda: nat.conv_gemm(dz2, wt, g), a.it)
            mean, invstd = torch.randn(c, device="cuda"), torch.rand(c, device="cuda") + 0.5
            rec["ours_dgrad_bnsums_us"] = bench(lambda: nat.conv_gemm(dz2, wt, g, None, 3, x2, None, coef, mean,
                                                                      invstd), a.it)
        rec["ours_wgrad_us"] = bench(lambda: nat.conv_wgrad(dz2, x2, g, coef), a.it)
        rec["ours_wgrad_nopro_us"] = bench(lambda: nat.conv_wgrad(dz2, x2, g), a.it)
        for k in list(rec):
            if k.endswith("_us"):
                rec[k] = round(rec[k], 1)
                d = k.split("_")[1]
                rec[k.replace("_us", "_tf")] = round(flops / rec[k] / 1e6, 1) if rec[k] > 0 else None
        tot["miopen"] += rec["miopen_fwd_us"] + rec["miopen_dgrad_us"] + rec["miopen_wgrad_us"]
        tot["ours"] += rec["ours_fwd_us"] + rec.get("ours_dgrad_us", rec["miopen_dgrad_us"]) + rec["ours_wgrad_us"]
        print(json.dumps(rec), flush=True)
        del x, w, dz
        torch.cuda.empty_cache()
    print(json.dumps({"total_us_one_conv_per_shape": tot}), flush=True)


if __name__ == "__main__":
    main()
