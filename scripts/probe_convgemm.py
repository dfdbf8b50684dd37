"""Micro-benchmark of the implicit-GEMM conv kernels (csrc/kernels/convgemm.hip) on ResNet-50
shapes at batch 512 vs hipBLASLt (torch.matmul) on the same [pixels, C] rows.

Prints one JSON line per shape: time (us), TF/s and HBM-side GB/s of ours and of the library
GEMM.  ``--quick``: only the first two shapes (for rocprofv3 --pmc passes)."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402
from ps_amd.ops.convgemm import geo  # noqa: E402

SHAPES = [  # name, images, H, Cin, Cout, ks, stride, pro
    ("1x1 14x14 1024->256", 512, 14, 1024, 256, 1, 1, False),
    ("1x1 56x56 64->256 +bn", 512, 56, 64, 256, 1, 1, True),
    ("1x1 56x56 256->64", 512, 56, 256, 64, 1, 1, False),
    ("1x1 28x28 128->512 +bn", 512, 28, 128, 512, 1, 1, True),
    ("1x1 7x7 2048->512", 512, 7, 2048, 512, 1, 1, False),
    ("1x1 7x7 512->2048 +bn", 512, 7, 512, 2048, 1, 1, True),
    ("3x3 56x56 64->64", 512, 56, 64, 64, 3, 1, True),
    ("3x3 14x14 256->256", 512, 14, 256, 256, 3, 1, True),
]


def bench(fn, it=20):
    for _ in range(3):
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
    quick = "--quick" in sys.argv
    nat = native()
    for name, n, h, ci, co, ks, s, pro in SHAPES[:2] if quick else SHAPES:
        g = geo(h, h, ks, s, ks // 2)
        M = n * g[2] * g[3]
        a = torch.randn(n * h * h, ci, device="cuda").bfloat16()
        b = (torch.randn(co, ks * ks * ci, device="cuda") * 0.05).bfloat16()
        coef = torch.cat([torch.rand(ci, device="cuda") + 0.5, torch.randn(ci, device="cuda")]) if pro else None
        ks_ = torch.zeros(co, device="cuda")
        t = bench(lambda: nat.conv_gemm(a, b, g, coef, 1, None, ks_))
        flops = 2.0 * M * co * ks * ks * ci
        byts = 2.0 * (a.numel() + M * co)
        rec = {"shape": name, "us": round(t, 1), "tflops": round(flops / t / 1e6, 1), "gbps": round(byts / t / 1e3, 1)}
        if ks == 1:
            tb = bench(lambda: a @ b.t())
            rec.update(blas_us=round(tb, 1), blas_tflops=round(flops / tb / 1e6, 1))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
