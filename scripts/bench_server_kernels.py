"""Server hot-path kernels vs the measured HBM roofline.

For every parameter-server kernel: bytes it must move (each operand read once, each result
written once), device time (HIP events over ``--iters`` launches after a warm-up), achieved
TB/s, and the fraction of the measured device-to-device copy bandwidth (the practical HBM
roofline of this box).  Shapes: Adam on a 1B-element shard (Llama-3-8B / 8 ranks), AdamW on
BERT-base (110M), momentum on ResNet-50 (25.6M), and the DLRM sparse path (26 x 1M x 128 rows
table slice, 400K touched rows).

    python scripts/bench_server_kernels.py [--iters 20] [--json gpurun_out/server_kernels.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ps_amd import ops  # noqa: E402
from ps_amd.ops import compress as C  # noqa: E402
from ps_amd.ops import sparse as S  # noqa: E402

DEV = "cuda"


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters * 1e-3  # seconds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default="gpurun_out/server_kernels.json")
    ap.add_argument("--big", type=int, default=1, help="include the 1B-element Adam shard (16 GB)")
    a = ap.parse_args()
    it = a.iters
    rows = []

    def rec(name, nbytes, sec, **kw):
        r = {"kernel": name, "bytes": nbytes, "us": round(sec * 1e6, 1), "TB/s": round(nbytes / sec / 1e12, 3), **kw}
        rows.append(r)
        print(json.dumps(r), flush=True)

    # ---- roofline: device-to-device copy (read + write) of 2 GiB
    src = torch.empty(2**29, dtype=torch.float32, device=DEV).uniform_()
    dst = torch.empty_like(src)
    t = timed(lambda: dst.copy_(src), it)
    peak = 2 * src.numel() * 4 / t
    rec("d2d_copy_2GiB (roofline)", 2 * src.numel() * 4, t)
    del src, dst

    # ---- fused optimizers on flat shards: (kind, n, grad dtype, wout dtype, hp)
    cfgs = [("momentum_resnet50", ops.SGD, 25_557_032, torch.bfloat16, torch.bfloat16,
             dict(lr=0.1, momentum=0.9, wd=5e-5)),
            ("adamw_bert_base", ops.ADAM, 110_000_000, torch.bfloat16, torch.bfloat16,
             dict(lr=1e-4, wd=0.01, adamw=True, bc1=1.1, bc2=1.01))]
    if a.big:
        cfgs.append(("adamw_llama8b_shard_1B", ops.ADAM, 1_003_782_656, torch.bfloat16, torch.bfloat16,
                     dict(lr=3e-4, wd=0.1, adamw=True, bc1=1.1, bc2=1.01)))
    for name, kind, n, gdt, wdt, hp in cfgs:
        w = torch.randn(n, device=DEV)
        g = torch.randn(n, device=DEV).to(gdt)
        st0 = torch.zeros(n, device=DEV)
        st1 = torch.zeros(n, device=DEV) if kind == ops.ADAM else None
        wout = torch.empty(n, device=DEV, dtype=wdt)
        ns = 1 if st1 is None else 2
        nbytes = n * (4 * 2 + 4 * 2 * ns + g.element_size() + wout.element_size())
        t = timed(lambda: ops.fused_opt(kind, w, st0, st1, g, wout=wout, **hp), it)
        rec(f"fused_opt:{name}", nbytes, t, n=n, frac_of_copy_roofline=round(nbytes / t / peak, 3))
        del w, g, st0, st1, wout
        torch.cuda.empty_cache()

    # ---- DLRM sparse path (one rank's shard of 26 x 1M x 128 over 8 ranks)
    R, D, U = 3_250_000, 128, 400_000
    table = torch.randn(R, D, device=DEV) * 0.01
    hstate = torch.zeros(R, device=DEV)
    rows_u = torch.randperm(R, device=DEV)[:U]
    grads = torch.randn(U, D, device=DEV)
    t = timed(lambda: ops.sparse_opt(ops.ADAGRAD, table, hstate, None, rows_u, grads, rowwise=True, lr=0.01,
                                     eps=1e-8), it)
    nb = U * D * 4 * 3 + U * 8 * 2
    rec("sparse_opt:rowwise_adagrad_400Kx128", nb, t, frac_of_copy_roofline=round(nb / t / peak, 3))
    # merged form: 2 workers pushed overlapping rows -> sorted runs
    dup = torch.cat([rows_u, rows_u[: U // 2]])
    srt, perm = torch.sort(dup)
    g2 = torch.randn(dup.numel(), D, device=DEV)
    t = timed(lambda: ops.sparse_opt(ops.ADAGRAD, table, hstate, None, srt, g2, rowwise=True, perm=perm, lr=0.01,
                                     eps=1e-8), it)
    nb = dup.numel() * D * 4 + U * D * 4 * 2 + dup.numel() * 16
    rec("sparse_opt:rowwise_adagrad_sorted_runs_600K", nb, t, frac_of_copy_roofline=round(nb / t / peak, 3))
    out = torch.empty(U, D, device=DEV)
    t = timed(lambda: S.gather_rows(table, rows_u, out), it)
    nb = U * D * 4 * 2 + U * 8
    rec("gather_rows:400Kx128", nb, t, frac_of_copy_roofline=round(nb / t / peak, 3))
    occ = torch.randint(0, U, (2 * U,), device=DEV)
    src = torch.randn(2 * U, D, device=DEV)
    srt, perm = torch.sort(occ)
    cnt = torch.bincount(srt, minlength=U)
    seg = torch.zeros(U + 1, dtype=torch.int64, device=DEV)
    seg[1:] = torch.cumsum(cnt, 0)
    red = torch.empty(U, D, device=DEV)
    t = timed(lambda: S.segment_reduce_rows(src, perm, seg, red), it)
    nb = 2 * U * D * 4 + U * D * 4 + 2 * U * 8
    rec("segment_reduce_rows:800K->400Kx128", nb, t, frac_of_copy_roofline=round(nb / t / peak, 3))
    flags = torch.zeros(R, dtype=torch.uint8, device=DEV)

    def init_fresh():
        flags.zero_()
        S.lazy_init_rows(table, rows_u, flags, 7, 0, -0.01, 0.01)

    t = timed(init_fresh, it)
    nb = U * D * 4 + U * 8 + R  # rows written + ids + flags reset
    rec("lazy_init_rows:400Kx128 (+flags reset)", nb, t, frac_of_copy_roofline=round(nb / t / peak, 3))
    hk = torch.full((1 << 23,), -1, dtype=torch.int64, device=DEV)
    st = torch.zeros(1, dtype=torch.int32, device=DEV)
    ids = torch.randint(0, 1 << 40, (U,), device=DEV)
    S.hash_slots(hk, ids, True, st)
    t = timed(lambda: S.hash_slots(hk, ids, False, st), it)
    rec("hash_slots:lookup_400K_in_8M", U * 16 + U * 8, t, note="latency-bound probe loads")
    del table, hstate, grads, g2, src, red, out, flags, hk
    torch.cuda.empty_cache()

    # ---- 1-bit compression (256M-element bucket, 8 workers' payloads on the owner)
    n = 1 << 28
    g = torch.randn(n, device=DEV).to(torch.bfloat16)
    err = torch.zeros(n, device=DEV)
    nw, nsc = C.packed_sizes(n)
    words = torch.empty(nw, dtype=torch.int64, device=DEV)
    scales = torch.empty(nsc, dtype=torch.float32, device=DEV)
    t = timed(lambda: C.onebit_pack(g, err, words, scales), it)
    nb = n * (2 + 4 + 4) + nw * 8 + nsc * 4
    rec("onebit_pack:256M_bf16", nb, t, frac_of_copy_roofline=round(nb / t / peak, 3))
    W = 8
    chunk = n // W
    wv = words[: W * (chunk // 64)].view(W, chunk // 64)
    sv = scales[: W * (chunk // C.CHUNK)].view(W, chunk // C.CHUNK)
    outp = torch.empty(chunk, device=DEV, dtype=torch.bfloat16)
    t = timed(lambda: C.onebit_unpack_reduce(wv, sv, outp, 1.0, False), it)
    nb = wv.numel() * 8 + sv.numel() * 4 + chunk * 2
    rec("onebit_unpack_reduce:8x32M", nb, t, frac_of_copy_roofline=round(nb / t / peak, 3))
    os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
    with open(a.json, "w") as f:
        json.dump({"copy_roofline_TBps": round(peak / 1e12, 3), "kernels": rows}, f, indent=1)


if __name__ == "__main__":
    main()
