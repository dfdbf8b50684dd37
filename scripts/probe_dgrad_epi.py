"""Data-gradient conv GEMMs with read-heavy epilogues (ResNet-50 bs1024 shapes): time / TB/s of
conv_gemm at epilogue 3 (ReLU mask + BN sums), 5 (masked identity gradient) and 6 (5 + the previous
block's bn3 reduce).  One JSON line per shape (profiles/r2_probe_dgrad_epi.jsonl: a persistent grid
and issuing the epilogue reads before the K loop were both measured here and not kept)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402
from ps_amd.ops.convgemm import geo  # noqa: E402

SHAPES = [  # name, pixels M, K, N, epi
    ("L3 conv1 dgrad epi6", 1024 * 14 * 14, 256, 1024, 6),
    ("L4 conv1 dgrad epi6", 1024 * 7 * 7, 512, 2048, 6),
    ("L2 conv1 dgrad epi6", 1024 * 28 * 28, 128, 512, 6),
    ("L3 conv3 dgrad epi3", 1024 * 14 * 14, 1024, 256, 3),
    ("L2 conv3 dgrad epi3", 1024 * 28 * 28, 512, 128, 3),
    ("L3 conv1 dgrad epi5", 1024 * 14 * 14, 256, 1024, 5),
]


def main():
    nat = native()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for name, M, K, N, epi in SHAPES:
        h = int(round((M / 1024) ** 0.5))
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        b = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        aux = torch.randn(M, N, device=dev).to(torch.bfloat16)
        bits = torch.randint(0, 256, (M * N // 8,), device=dev, dtype=torch.uint8)
        mean = torch.zeros(N, device=dev)
        inv = torch.ones(N, device=dev)
        mc = torch.cat([torch.ones(N, device=dev), torch.zeros(N, device=dev)])
        g = geo(h, h)
        if epi == 3:
            fn = lambda: nat.conv_gemm(a, b, g, None, 3, aux, None, mc, mean, inv)  # noqa: E731
            nbytes = 2 * (M * K + 2 * M * N)
        elif epi == 5:
            fn = lambda: nat.conv_gemm(a, b, g, None, 5, aux, bits=bits)  # noqa: E731
            nbytes = 2 * (M * K + 2 * M * N) + M * N // 8
        else:
            aux2 = torch.randn(M, N, device=dev).to(torch.bfloat16)
            fn = lambda: nat.conv_gemm(a, b, g, None, 6, aux, bits=bits, mean=mean, invstd=inv, aux2=aux2,  # noqa: E731
                                       bits2=bits)
            nbytes = 2 * (M * K + 3 * M * N) + M * N // 4
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / it * 1e3
        print(json.dumps({"shape": name, "us": round(us, 1),
                          "tbps": round(nbytes / us / 1e6, 2), "tflops": round(2 * M * N * K / us / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
