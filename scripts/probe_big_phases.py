"""Per-block phase timing of the 256 x 256-tile conv GEMM (conv_big.hip, tbuf stamps, 100 MHz wall
clock): first stage landed, K loop, accumulators -> LDS, row pass issued, stores drained, on the
layer-3 conv1 data-gradient shape (M 200704, K 256, N 1024) with epilogue 0 and 6 and the layer-3
conv3 data gradient (K 1024, N 256, epilogue 3).  Prints mean / p10 / p90 per phase in us, the
kernel span and the number of blocks resident per CU over time.
usage: python scripts/probe_big_phases.py -> gpurun_out/big_phases.txt"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402
from ps_amd.ops.convgemm import geo  # noqa: E402

TICK_US = 0.01  # wall_clock64 runs at 100 MHz


def phases(tb, nblk):
    t = tb.view(nblk, 8).cpu().double()
    t0 = t[:, 0].min()
    d = {"first_stage": t[:, 1] - t[:, 0], "k_loop": t[:, 2] - t[:, 1], "acc_to_lds": t[:, 3] - t[:, 2],
         "row_pass": t[:, 4] - t[:, 3], "store_drain": t[:, 5] - t[:, 4], "block_total": t[:, 5] - t[:, 0]}
    out = {}
    for k, v in d.items():
        v = v * TICK_US
        out[k] = [round(v.mean().item(), 2), round(v.quantile(0.1).item(), 2), round(v.quantile(0.9).item(), 2)]
    out["span_us"] = round(((t[:, 5].max() - t0) * TICK_US).item(), 1)
    # average blocks in flight = sum of block durations / span
    out["avg_blocks_in_flight"] = round((d["block_total"].sum() / (t[:, 5].max() - t0)).item(), 1)
    return out


def main():
    nat = native()
    lines = []
    n, h = 1024, 14
    gg = geo(h, h)
    M = n * h * h
    for name, k, cin, epi in [("l3 conv1 dgrad epi0", 256, 1024, 0), ("l3 conv1 dgrad epi6", 256, 1024, 6),
                              ("l3 conv3 dgrad epi3 K1024", 1024, 256, 3), ("l4-like K512 N2048 epi0", 512, 2048, 0)]:
        a = (torch.randn(M, k, device="cuda") * 0.5).bfloat16()
        w = (torch.randn(cin, k, device="cuda") * k ** -0.5).bfloat16()
        pos, kw = (), {}
        if epi == 6:
            bits = torch.randint(0, 256, (M * cin // 8,), device="cuda", dtype=torch.uint8)
            pos = (torch.randn(M, cin, device="cuda").bfloat16(),)
            kw = dict(bits=bits, aux2=torch.randn(M, cin, device="cuda").bfloat16(), bits2=bits,
                      mean=torch.zeros(cin, device="cuda"), invstd=torch.ones(cin, device="cuda"))
        elif epi == 3:
            pos = (torch.randn(M, cin, device="cuda").bfloat16(), None,
                   torch.cat([torch.ones(cin, device="cuda"), torch.zeros(cin, device="cuda")]),
                   torch.zeros(cin, device="cuda"), torch.ones(cin, device="cuda"))
        bm, bn, gm = nat.conv_gemm_plan(M, cin, k, gg, False, epi)
        assert bm == 256, (bm, bn)
        nblk = gm * (cin // bn)
        tb = torch.zeros(nblk * 8, dtype=torch.int64, device="cuda")
        for _ in range(3):
            nat.conv_gemm(a, w, gg, None, epi, *pos, **kw)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        nat.conv_gemm(a, w, gg, None, epi, *pos, **kw, tbuf=tb)
        ev[1].record()
        torch.cuda.synchronize()
        rec = {"shape": name, "tile": [bm, bn], "blocks": nblk, "event_ms": round(ev[0].elapsed_time(ev[1]), 4)}
        rec.update(phases(tb, nblk))
        lines.append(json.dumps(rec))
        print(lines[-1], flush=True)
        del a, w, pos, kw
        torch.cuda.empty_cache()
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/big_phases.txt", "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
