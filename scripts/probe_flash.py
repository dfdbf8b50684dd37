"""Causal GQA flash attention (csrc/kernels/flash_attn.hip) vs torch SDPA on the Llama-3-8B bench
shape (1 x 4096 tokens, 32 q / 8 kv heads x 128): forward and backward times and TF/s (causal
FLOPs: 4 S^2 D H / 2 forward, 2.5x that backward)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402


def bench(fn, it=10):
    for _ in range(2):
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    H, KV, S, D = 32, 8, 4096, 128
    q = torch.randn(B, H, S, D, device="cuda").bfloat16()
    k = torch.randn(B, KV, S, D, device="cuda").bfloat16()
    v = torch.randn(B, KV, S, D, device="cuda").bfloat16()
    dout = torch.randn(B, S, H * D, device="cuda").bfloat16()
    nat = native()
    out, lse = nat.fa_fwd(q, k, v)
    fl = 4.0 * S * S * D * H / 2 * B
    tf = bench(lambda: nat.fa_fwd(q, k, v))
    tb = bench(lambda: nat.fa_bwd(q, k, v, out, dout, lse))
    qs, ks, vs = (t.detach().clone().requires_grad_() for t in (q, k, v))
    o = F.scaled_dot_product_attention(qs, ks, vs, is_causal=True, enable_gqa=True)
    go = torch.randn_like(o)
    sf = bench(lambda: F.scaled_dot_product_attention(qs, ks, vs, is_causal=True, enable_gqa=True))
    sb = bench(lambda: torch.autograd.grad(o, (qs, ks, vs), go, retain_graph=True))
    print(json.dumps({"shape": f"B{B} H{H} KV{KV} S{S} D{D} causal", "fused_fwd_us": round(tf, 1),
                      "fused_fwd_tf": round(fl / tf / 1e6, 1), "fused_bwd_us": round(tb, 1),
                      "fused_bwd_tf": round(2.5 * fl / tb / 1e6, 1), "sdpa_fwd_us": round(sf, 1),
                      "sdpa_fwd_tf": round(fl / sf / 1e6, 1), "sdpa_bwd_us": round(sb, 1),
                      "sdpa_bwd_tf": round(2.5 * fl / sb / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
