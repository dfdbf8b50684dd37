"""BERT-base attention (B 1024, S 128, H 12, d 64; dropout 0.1) alone: fwd / bwd ms and the HBM rate
over qkv + out (+ dout, dqkv) -- to tell kernel headroom from in-step contention."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops.transformer import attention_qkv  # noqa: E402


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    B, S, H, D = 1024, 128, 12, 64
    for p in (0.1, 0.0):
        qkv = (torch.randn(B, S, 3 * H * D, device="cuda") * 0.5).bfloat16().requires_grad_(True)
        out = attention_qkv(qkv, H, p, None)
        g = torch.randn_like(out)
        tf = t(lambda: attention_qkv(qkv, H, p, None))
        tfb = t(lambda: torch.autograd.grad(attention_qkv(qkv, H, p, None), qkv, g))
        nb = qkv.numel() * 2
        print(json.dumps({"dropout": p, "fwd_ms": round(tf, 4), "fwd_TBs": round((nb + out.numel() * 2) / tf / 1e9, 2),
                          "fwd_bwd_ms": round(tfb, 4), "bwd_ms": round(tfb - tf, 4),
                          "bwd_TBs": round((2 * nb + 2 * out.numel() * 2) / (tfb - tf) / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
