"""One conv_big GEMM shape, run 20 times, for rocprofv3 --pmc passes (scripts/runs/gpu_round5_bigpmc.sh).
usage: python scripts/probe_big_pmc.py {deep|fold}
  deep: layer-3 conv1 forward 1024 -> 256 (M 200704, epilogue 1; K loop dominated)
  fold: layer-3 conv1 data gradient 256 -> 1024 (M 200704, epilogue 6; epilogue dominated)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "deep"
    nat = native()
    M = 200704
    K, N = (1024, 256) if kind == "deep" else (256, 1024)
    gg = [M, 1, M, 1, 1, 1, 0]
    a = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
    if kind == "deep":
        pos, kw, epi = (None, torch.zeros(N, device="cuda")), {}, 1
    else:
        bits = torch.randint(0, 256, (M * N // 8,), device="cuda", dtype=torch.uint8)
        pos = (torch.randn(M, N, device="cuda").bfloat16(),)
        kw = dict(bits=bits, aux2=torch.randn(M, N, device="cuda").bfloat16(), bits2=bits,
                  mean=torch.zeros(N, device="cuda"), invstd=torch.ones(N, device="cuda"))
        epi = 6
    for _ in range(20):
        nat.conv_gemm(a, w, gg, None, epi, *pos, **kw)
    torch.cuda.synchronize()
    print("done", kind, nat.conv_gemm_plan(M, N, K, gg, False, epi))


if __name__ == "__main__":
    main()
