"""conv3 backward at the ResNet-50 layer-1 shape: the fused one-pass kernel
(csrc/kernels/conv_bwd_fused.hip) vs the chain it replaces (BN-backward-prologue data gradient that
stores dz3 + the weight-gradient GEMM re-reading dz3 and z2).  Prints one JSON line per shape."""
import json
import sys

import torch

sys.path.insert(0, ".")
from ps_amd.ops import native  # noqa: E402


def timeit(fn, reps=10, rounds=3):
    fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        best.append(a.elapsed_time(b) / reps)
    return sorted(best)[len(best) // 2]


def main():
    dev = "cuda"
    for M, CI, CO in [(1024 * 56 * 56, 64, 256), (256 * 56 * 56, 64, 256), (1024 * 28 * 28, 128, 512)]:
        g = torch.Generator(device=dev).manual_seed(0)
        d = torch.randn(M, CO, device=dev, generator=g).bfloat16()
        z3 = torch.randn(M, CO, device=dev, generator=g).bfloat16()
        z2 = torch.randn(M, CI, device=dev, generator=g).bfloat16()
        coef = torch.randn(3 * CO, device=dev, generator=g) * 0.1
        w3t = (torch.randn(CI, CO, device=dev, generator=g) * CO ** -0.5).bfloat16()
        cf2 = torch.cat([torch.rand(CI, device=dev, generator=g) + 0.5, torch.randn(CI, device=dev, generator=g)])
        m2, i2 = torch.zeros(CI, device=dev), torch.ones(CI, device=dev)
        geo = [M, 1, M, 1, 1, 1, 0]

        def fused():
            return native().conv11_bwd_fused(d, z3, coef, w3t, z2, cf2, m2, i2)

        def chain():
            c, p, dz = native().conv_gemm(d, w3t, geo, None, 3, z2, None, cf2, m2, i2, a2=z3, bwd=coef)
            return native().conv_wgrad(dz, z2, geo, cf2)

        def chain_dgrad():
            return native().conv_gemm(d, w3t, geo, None, 3, z2, None, cf2, m2, i2, a2=z3, bwd=coef)

        tf, tc, td = timeit(fused), timeit(chain), timeit(chain_dgrad)
        gb = (2 * M * CO + 2 * M * CI) * 2 / 1e9  # fused: g, z3, z2 read; gy written
        print(json.dumps({"M": M, "CI": CI, "CO": CO, "fused_ms": round(tf, 4), "chain_ms": round(tc, 4),
                          "chain_dgrad_ms": round(td, 4), "fused_GB": round(gb, 3),
                          "fused_TBps": round(gb / tf, 2)}), flush=True)


if __name__ == "__main__":
    main()
