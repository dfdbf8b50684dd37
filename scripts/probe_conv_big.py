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


if __name__ == "__main__" and "--pro" not in sys.argv:
    main()


PRO_SHAPES = [  # name, M (batch 1024), K, N, kind
    ("l3 BWD conv3 dgrad (g,z -> dz) 1024->256", 200704, 1024, 256, "bwd"),
    ("l4 BWD conv3 dgrad 2048->512", 50176, 2048, 512, "bwd"),
    ("l3 RESP conv1 1024->256", 200704, 1024, 256, "resp"),
    ("l3b0 RESP conv1 512->256 (28x28)", 802816, 512, 256, "resp"),
    ("l4 RESP conv1 2048->512", 50176, 2048, 512, "resp"),
    ("l4b0 RESP conv1 1024->512 (14x14)", 200704, 1024, 512, "resp"),
    ("l3 PRO1 conv3 256->1024", 200704, 256, 1024, "pro1"),
]


def main_pro():
    """The prologue variants at their ResNet-50 bs1024 shapes: ms, TF/s and the HBM rate over every
    tensor they move (A and a2 read, aout (+ bits) written, C written, epilogue rows read)."""
    nat = native()
    for name, M, K, N, kind in PRO_SHAPES:
        a = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
        b = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
        gg = [M, 1, M, 1, 1, 1, 0]
        ks = torch.zeros(N, device="cuda")
        coef = torch.cat([torch.ones(K, device="cuda"), torch.zeros(K, device="cuda")])
        if kind == "bwd":
            z = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
            cb = torch.cat([torch.ones(K, device="cuda"), torch.zeros(2 * K, device="cuda")])
            z2 = torch.randn(M, N, device="cuda").bfloat16()
            mc = torch.cat([torch.ones(N, device="cuda"), torch.zeros(N, device="cuda")])
            mean, inv = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
            fn = lambda: nat.conv_gemm(a, b, gg, None, 3, z2, None, mc, mean, inv, a2=z, bwd=cb)  # noqa: E731
            byts = 2.0 * (3 * M * K + 2 * M * N)
            src2 = 2
        elif kind == "resp":
            r = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
            out = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
            bits = torch.empty(M * K // 8, device="cuda", dtype=torch.uint8)
            fn = lambda: nat.conv_gemm(a, b, gg, coef, 1, None, ks, a2=r, aout=out, abits=bits)  # noqa: E731
            byts = 2.0 * (3 * M * K + M * N) + M * K / 8
            src2 = 1
        else:
            fn = lambda: nat.conv_gemm(a, b, gg, coef, 1, None, ks)  # noqa: E731
            byts = 2.0 * (M * K + M * N)
            src2 = 0
        t = timeit(fn)
        plan = nat.conv_gemm_plan(M, N, K, gg, True, 3 if kind == "bwd" else 1, src2)
        print(json.dumps({"big": os.environ.get("PS_AMD_CONV_BIG", "1"), "pro_big": os.environ.get("PS_AMD_CONV_BIG_PRO", "1"),
                          "shape": name, "tile": plan[:2], "ms": round(t, 4),
                          "TFs": round(2.0 * M * K * N / t / 1e9, 1), "TBs": round(byts / t / 1e9, 2)}), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__" and "--pro" in sys.argv:
    main_pro()
