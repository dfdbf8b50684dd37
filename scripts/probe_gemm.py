"""Our MFMA NT GEMM (ps_amd._C.gemm_nt) vs torch.matmul (hipBLASLt) on ResNet-50 1x1-conv
GEMM shapes at batch 512: C[M, N] = A[M, K] . B[N, K]^T."""
import json

import torch

from ps_amd.ops import native

SHAPES = [(512 * 3136, 256, 64), (512 * 3136, 64, 256), (512 * 784, 512, 128), (512 * 196, 256, 1024),
          (512 * 196, 1024, 256), (512 * 49, 512, 2048), (8192, 8192, 8192)]


def bench(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(N, K, device="cuda").bfloat16()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    t_ours = bench(lambda: native().gemm_nt(a, b, c, None, 0, 1.0, False))
    t_blas = bench(lambda: a @ b.t())
    err = ((c.float() - (a @ b.t()).float()).abs().max() / (a @ b.t()).float().abs().max()).item()
    fl = 2 * M * N * K
    print(json.dumps({"M": M, "N": N, "K": K, "ours_us": round(t_ours, 1), "blas_us": round(t_blas, 1),
                      "ours_tflops": round(fl / t_ours / 1e6), "blas_tflops": round(fl / t_blas / 1e6),
                      "rel_err": err}), flush=True)
