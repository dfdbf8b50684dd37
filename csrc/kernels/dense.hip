// MFMA fused linear layer (K1/K2 in SURVEY §2.5): Y = act(X W^T + b) in bf16 with fp32
// accumulation, for the reference-scale FC layers (layer/FcLayer.java:74-110: MNIST
// 784->150->50->10, CTR 275->150->10->1) whose GEMMs are too small for library GEMMs to
// reach a good fraction of the chip, and whose bias + activation would otherwise be two
// more passes over the output.
//
// "NT" GEMM: C[M, N] = A[M, K] . B[N, K]^T -- both operands K-contiguous (row-major X and
// the [out, in] weight), which is exactly the operand layout of v_mfma_f32_16x16x32_bf16:
// lane l holds A[l&15][8*(l>>4) .. +7] and B[l&15][8*(l>>4) .. +7], i.e. one 16-byte
// ds_read_b128 per operand per MFMA.  Backward reuses the same kernel on transposed copies.
//
// Tiling: 256 threads = 4 waves, block tile 64x64, BK = 32; each wave owns a 32x32 sub-tile
// = 2x2 MFMA 16x16x32 accumulators.  Global -> LDS staging: one 16-byte load per thread per
// operand per K-step (64 rows x 32 k x 2 B = 4 KiB), double-buffered in LDS; LDS rows are
// padded to 80 B so the 16 lanes reading one k-slice of 16 rows hit distinct banks.  M/N/K
// tails are zero-filled on load and masked on store.  Epilogue: + bias, activation
// (0 none, 1 relu, 2 leaky 0.01, 3 the reference clipped sigmoid), bf16 store.
#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int kBM = 64, kBN = 64, kBK = 32;
constexpr int kLdsRow = 40;  // 32 bf16 + 8 pad (80 B)

__device__ __forceinline__ float act_fwd(float v, int act) {
  if (act == 1) return v > 0.f ? v : 0.f;
  if (act == 2) return v > 0.f ? v : 0.01f * v;
  if (act == 3) return 0.001f + 0.998f / (1.f + __expf(-v));
  return v;
}

// load 8 consecutive bf16 of row `row` starting at k0 (zero-filled outside [0,rows)x[0,K))
__device__ __forceinline__ u16x8 load_row8(const uint16_t* __restrict__ p, int64_t ld, int row, int rows, int k0,
                                           int K, bool vec_ok) {
  u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
  if (row < rows) {
    const uint16_t* src = p + static_cast<int64_t>(row) * ld + k0;
    if (vec_ok && k0 + 8 <= K) {
      v = *reinterpret_cast<const u16x8*>(src);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (k0 + j < K) v[j] = src[j];
    }
  }
  return v;
}

template <int ACT, bool BIAS, bool OUT_F32>
__global__ __launch_bounds__(256) void gemm_nt_bf16_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                           const uint16_t* __restrict__ B, int64_t ldb,
                                                           void* __restrict__ C, int64_t ldc,
                                                           const float* __restrict__ bias, int M, int N, int K,
                                                           float alpha, int accumulate) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2][2][kBM * kLdsRow];  // [buf][A/B][row*40 + k]
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int m0 = blockIdx.y * kBM, n0 = blockIdx.x * kBN;
  // staging coordinates: thread t loads row t/4, k-chunk (t%4)*8 of both tiles
  const int srow = t >> 2, sk = (t & 3) * 8;
  const bool vec_a = ((reinterpret_cast<uintptr_t>(A) | (lda * 2)) & 15) == 0;
  const bool vec_b = ((reinterpret_cast<uintptr_t>(B) | (ldb * 2)) & 15) == 0;

  f32x4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + kBK - 1) / kBK;
  u16x8 ra = load_row8(A, lda, m0 + srow, M, sk, K, vec_a);
  u16x8 rb = load_row8(B, ldb, n0 + srow, N, sk, K, vec_b);
  *reinterpret_cast<u16x8*>(&lds[0][0][srow * kLdsRow + sk]) = ra;
  *reinterpret_cast<u16x8*>(&lds[0][1][srow * kLdsRow + sk]) = rb;
  __syncthreads();
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // issue the next tile's global loads before the MFMAs (latency hidden under compute)
    if (kt + 1 < nk) {
      ra = load_row8(A, lda, m0 + srow, M, (kt + 1) * kBK + sk, K, vec_a);
      rb = load_row8(B, ldb, n0 + srow, N, (kt + 1) * kBK + sk, K, vec_b);
    }
    bf16x8_t af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      af[i] = *reinterpret_cast<const bf16x8_t*>(&lds[cur][0][(wm + i * 16 + fr) * kLdsRow + fk]);
      bfr[i] = *reinterpret_cast<const bf16x8_t*>(&lds[cur][1][(wn + i * 16 + fr) * kLdsRow + fk]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) {
      *reinterpret_cast<u16x8*>(&lds[cur ^ 1][0][srow * kLdsRow + sk]) = ra;
      *reinterpret_cast<u16x8*>(&lds[cur ^ 1][1][srow * kLdsRow + sk]) = rb;
    }
    __syncthreads();
  }
  // epilogue: C/D layout of 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn + j * 16 + (lane & 15);
      if (col >= N) continue;
      const float bv = BIAS ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
        if (row >= M) continue;
        float v = alpha * acc[i][j][r];
        if constexpr (OUT_F32) {
          float* cp = static_cast<float*>(C) + static_cast<int64_t>(row) * ldc + col;
          if (accumulate) v += *cp;
          *cp = act_fwd(v + bv, ACT);
        } else {
          uint16_t* cp = static_cast<uint16_t*>(C) + static_cast<int64_t>(row) * ldc + col;
          if (accumulate) v += bf16_to_f32(*cp);
          *cp = f32_to_bf16(act_fwd(v + bv, ACT));
        }
      }
    }
}

void launch_gemm_nt_bf16(const uint16_t* a, int64_t lda, const uint16_t* b, int64_t ldb, void* c, int c_f32,
                         int64_t ldc, int M, int N, int K, float alpha, int accumulate, const float* bias, int act,
                         hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  dim3 grid((N + kBN - 1) / kBN, (M + kBM - 1) / kBM);
#define PSAMD_GEMM(ACT, BIAS, F32)                                                                            \
  hipLaunchKernelGGL((gemm_nt_bf16_kernel<ACT, BIAS, F32>), grid, dim3(256), 0, s, a, lda, b, ldb, c, ldc, bias, \
                     M, N, K, alpha, accumulate)
#define PSAMD_GEMM_ACT(BIAS, F32)          \
  switch (act) {                           \
    case 1: PSAMD_GEMM(1, BIAS, F32); break; \
    case 2: PSAMD_GEMM(2, BIAS, F32); break; \
    case 3: PSAMD_GEMM(3, BIAS, F32); break; \
    default: PSAMD_GEMM(0, BIAS, F32); break; \
  }
  if (bias) {
    if (c_f32) { PSAMD_GEMM_ACT(true, true) } else { PSAMD_GEMM_ACT(true, false) }
  } else {
    if (c_f32) { PSAMD_GEMM_ACT(false, true) } else { PSAMD_GEMM_ACT(false, false) }
  }
#undef PSAMD_GEMM_ACT
#undef PSAMD_GEMM
}

// dZ = dY * act'(Y) (Y = activation output), bf16 -- the reference activation backwards
// (Relu.java, LeakyRelu.java, Sigmoid.java: dy * y * (1 - y))
__global__ __launch_bounds__(256) void act_bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                                                      uint16_t* __restrict__ dz, int64_t n, int act) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float g = bf16_to_f32(dy[i]), yv = bf16_to_f32(y[i]);
    float d = g;
    if (act == 1) d = yv > 0.f ? g : 0.f;
    else if (act == 2) d = yv > 0.f ? g : 0.01f * g;
    else if (act == 3) d = g * yv * (1.f - yv);
    dz[i] = f32_to_bf16(d);
  }
}

void launch_act_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dz, int64_t n, int act, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(act_bwd_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, s, dy, y, dz, n, act);
}

}  // namespace psamd
