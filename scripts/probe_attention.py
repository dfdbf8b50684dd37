"""Fused attention kernels (csrc/kernels/attention.hip) vs torch SDPA on the BERT-base bench shape
(B 256, S 128, 12 heads x 64), forward and backward, with / without probability dropout."""
import json
import os
import sys

import torch
import torch.nn.functional as F

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
    B, S, H = 256, 128, 12
    qkv = torch.randn(B, S, 3 * H * 64, device="cuda").bfloat16()
    dout = torch.randn(B, S, H * 64, device="cuda").bfloat16()
    nat = native()
    by_f = 2 * (qkv.numel() + dout.numel())
    by_b = 2 * (qkv.numel() * 2 + dout.numel() * 2)
    for p in (0.0, 0.1):
        out, lse = nat.attn_fwd(qkv, H, p, 7)
        tf = bench(lambda: nat.attn_fwd(qkv, H, p, 7))
        tb = bench(lambda: nat.attn_bwd(qkv, out, dout, lse, H, p, 7))
        q, k, v = qkv.view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
        qs, ks, vs = (t.detach().clone().requires_grad_() for t in (q, k, v))
        o = F.scaled_dot_product_attention(qs, ks, vs, dropout_p=p)
        go = torch.randn_like(o)
        sf = bench(lambda: F.scaled_dot_product_attention(qs, ks, vs, dropout_p=p))
        sb = bench(lambda: torch.autograd.grad(o, (qs, ks, vs), go, retain_graph=True))
        print(json.dumps({"p": p, "fused_fwd_us": round(tf, 1), "fused_bwd_us": round(tb, 1),
                          "fused_fwd_TBps": round(by_f / tf / 1e6, 2), "fused_bwd_TBps": round(by_b / tb / 1e6, 2),
                          "sdpa_fwd_us": round(sf, 1), "sdpa_bwd_us": round(sb, 1)}), flush=True)


if __name__ == "__main__":
    main()
