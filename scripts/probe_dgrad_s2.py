"""Stride-2 3x3 data gradients of ResNet-50 (bs1024): the four phase GEMMs (conv_dgrad_s2, epilogue
3) vs MIOpen's convolution_backward (data only) + the separate bn1 backward reduce it needs."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402
from ps_amd.ops.convgemm import _phase_weights  # noqa: E402

torch.backends.cudnn.benchmark = True


def timed(fn, it=10):
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
    nat = native()
    dev = "cuda"
    for h, c in ((56, 128), (28, 256), (14, 512)):
        n, oh = 1024, h // 2
        w = (torch.randn(c, c, 3, 3, device=dev) * 0.02).bfloat16().contiguous(memory_format=torch.channels_last)
        dz = torch.randn(n, c, oh, oh, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        y1 = torch.randn(n, c, h, h, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        z1 = torch.randn(n * h * h, c, device=dev).bfloat16()
        mc = torch.cat([torch.ones(c, device=dev), torch.zeros(c, device=dev)])
        mean, inv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        dzr = dz.permute(0, 2, 3, 1).reshape(-1, c)
        wph = _phase_weights(w)
        ours = timed(lambda: nat.conv_dgrad_s2(dzr, wph, h, h, 3, z1, mc, mean, inv))
        mio = timed(lambda: torch.ops.aten.convolution_backward(dz, y1, w, None, [2, 2], [1, 1], [1, 1], False,
                                                                 [0, 0], 1, [True, False, False]))
        fl = 2 * n * oh * oh * 9 * c * c
        print(json.dumps({"shape": f"3x3 s2 {h}x{h} {c}", "ours_us": round(ours, 1), "ours_tf": round(fl / ours / 1e6, 1),
                          "miopen_us": round(mio, 1), "miopen_tf": round(fl / mio / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
