"""SwiGLU kernels alone on the Llama-3-8B MLP shape (4 x 4096 tokens, F 14336): fwd / bwd us and the
HBM rate over what they must move (fwd: gu in, h out; bwd: dh + gu in, dgu out)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402


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
    R, F = 16384, 14336
    nat = native()
    gu = torch.randn(R, 2 * F, device="cuda").bfloat16()
    dh = torch.randn(R, F, device="cuda").bfloat16()
    tf = bench(lambda: nat.swiglu_fwd(gu))
    tb = bench(lambda: nat.swiglu_bwd(dh, gu))
    fb, bb = 3 * R * F * 2, 5 * R * F * 2
    print(json.dumps({"shape": f"R{R} F{F}", "fwd_us": round(tf, 1), "fwd_TBs": round(fb / tf / 1e6, 2),
                      "bwd_us": round(tb, 1), "bwd_TBs": round(bb / tb / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
