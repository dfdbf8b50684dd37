"""ResNet-50 layer-1 3x3 (56 x 56, 64 -> 64) forward (epilogue 1) and data gradient (epilogue 3)
at batch 1024 / 256: time per launch.  Run under PS_AMD_CONV_C64=0 (tall im2col tile), 1 (round-4
resident-weight kernel) or 2 (planar kernel, csrc/kernels/conv3x3_c64.hip)."""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from ps_amd.ops import native  # noqa: E402
from ps_amd.ops.convgemm import geo  # noqa: E402


def timeit(fn, reps=20):
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
    dev = "cuda"
    for n in (1024, 256):
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(n * 56 * 56, 64, device=dev, generator=g).bfloat16()
        w = (torch.randn(64, 576, device=dev, generator=g) * 0.04).bfloat16()
        ks = torch.zeros(64, device=dev)
        z1 = torch.randn(n * 56 * 56, 64, device=dev, generator=g).bfloat16()
        coef = torch.cat([torch.ones(64, device=dev), torch.zeros(64, device=dev)])
        mean, inv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
        gg = geo(56, 56, 3, 1, 1)
        tf = timeit(lambda: native().conv_gemm(x, w, gg, None, 1, None, ks))
        td = timeit(lambda: native().conv_gemm(x, w, gg, None, 3, z1, None, coef, mean, inv))
        fl = 2 * n * 56 * 56 * 64 * 576 / 1e9
        print(json.dumps({"mode": os.environ.get("PS_AMD_CONV_C64", "0"), "lookahead": os.environ.get("PS_AMD_C64_LOOKAHEAD", "2"), "batch": n, "fwd_ms": round(tf, 4),
                          "dgrad_ms": round(td, 4), "fwd_TFs": round(fl / tf, 1), "dgrad_TFs": round(fl / td, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
