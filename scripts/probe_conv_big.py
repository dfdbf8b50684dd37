"""Deep-K 1x1 convolution GEMMs of ResNet-50 (layers 2-4 at batch 1024 / 256) through conv_gemm:
time per call and TF/s.  Run once with PS_AMD_CONV_BIG=1 (256 x 256 tiles, conv_big.hip) and once
with PS_AMD_CONV_BIG=0 (the 128 x 128 conv_fwd_kernel) -- the switch is read once per process.
One JSON line per shape and batch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402
from ps_amd.ops.convgemm import geo  # noqa: E402

# name, H (input map), K (input channels), N (output channels), stride, epilogue
SHAPES = [
    ("l3 conv1 14x14 1024->256", 14, 1024, 256, 1, 1),
    ("l3 conv3 dgrad 14x14 1024->256", 14, 1024, 256, 1, 3),
    ("l3 conv3 14x14 256->1024", 14, 256, 1024, 1, 1),
    ("l3b0 conv1 28x28 512->256", 28, 512, 256, 1, 1),
    ("l4 conv1 7x7 2048->512", 7, 2048, 512, 1, 1),
    ("l4 conv3 dgrad 7x7 2048->512", 7, 2048, 512, 1, 3),
    ("l4 conv3 7x7 512->2048", 7, 512, 2048, 1, 1),
    ("l4b0 conv1 14x14 1024->512", 14, 1024, 512, 1, 1),
    ("ds l2 56->28 256->512", 56, 256, 512, 2, 1),
    ("ds l3 28->14 512->1024", 28, 512, 1024, 2, 1),
    ("ds l4 14->7 1024->2048", 14, 1024, 2048, 2, 1),
]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    return sorted(ts)[1]


def main():
    nat = native()
    mode = os.environ.get("PS_AMD_CONV_BIG", "1")
    for n in (1024, 256):
        for name, h, k, co, s, epi in SHAPES:
            gg = geo(h, h, 1, s)
            M = n * gg[2] * gg[3]
            a = (torch.randn(n * h * h, k, device="cuda") * 0.5).bfloat16()
            b = (torch.randn(co, k, device="cuda") * k ** -0.5).bfloat16()
            ks = torch.zeros(co, device="cuda")
            if epi == 1:
                fn = lambda: nat.conv_gemm(a, b, gg, None, 1, None, ks)  # noqa: E731
            else:
                z = torch.randn(M, co, device="cuda").bfloat16()
                mc = torch.cat([torch.ones(co, device="cuda"), torch.zeros(co, device="cuda")])
                mean, inv = torch.zeros(co, device="cuda"), torch.ones(co, device="cuda")
                fn = lambda: nat.conv_gemm(a, b, gg, None, 3, z, None, mc, mean, inv)  # noqa: E731
            t = timeit(fn)
            plan = nat.conv_gemm_plan(M, co, k, gg, False, epi)
            flops = 2.0 * M * k * co
            byts = 2.0 * (M * k + M * co * (2 if epi == 3 else 1))
            print(json.dumps({"big": mode, "batch": n, "shape": name, "tile": plan[:2], "ms": round(t, 4),
                              "TFs": round(flops / t / 1e9, 1), "TBs": round(byts / t / 1e9, 2)}), flush=True)
            del a, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
