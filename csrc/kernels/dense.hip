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



// ------------------------------------------------------------------------------ DLRM interaction
// out[b] = [ x[b] | triu_{i<j}( z_i . z_j ) ] with z = [x[b]; e[b, 0..T)] (n = T + 1 <= 32
// vectors of D bf16), i.e. torch.cat + bmm + triu gather + cat in ONE pass: one wave per sample,
// Z = z z^T on v_mfma_f32_32x32x16_bf16 (the A and B fragments of z z^T are the same registers),
// only the n(n-1)/2 upper-triangle dots are written.  Backward: dz = (G + G^T) z, G the
// scattered triangle gradient, as a second 32x32 MFMA product per sample; dx adds the
// pass-through gradient.  SURVEY K16 (dense.hip, "DLRM interaction").
namespace {
typedef float f32x16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int tri_index(int i, int j, int n) { return i * (2 * n - i - 1) / 2 + (j - i - 1); }
}  // namespace

__global__ __launch_bounds__(256) void dlrm_interact_fwd_kernel(const uint16_t* __restrict__ x,
                                                                const uint16_t* __restrict__ e,
                                                                uint16_t* __restrict__ out, int B, int T, int D) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // wave-uniform; no block barriers below
  const int n = T + 1, P = n * (n - 1) / 2;
  const int r = lane & 31, h = lane >> 5;
  const uint16_t* row = r == 0 ? x + static_cast<int64_t>(b) * D
                               : e + (static_cast<int64_t>(b) * T + (r - 1)) * D;
  f32x16v acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  for (int k0 = 0; k0 < D; k0 += 16) {
    bf16x8_t f = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r < n) f = *reinterpret_cast<const bf16x8_t*>(row + k0 + 8 * h);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f, f, acc, 0, 0, 0);
  }
  uint16_t* o = out + static_cast<int64_t>(b) * (D + P);
  for (int c = lane; c < D / 8; c += 64)  // dense pass-through
    *reinterpret_cast<u16x8*>(o + 8 * c) = *reinterpret_cast<const u16x8*>(x + static_cast<int64_t>(b) * D + 8 * c);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int i = (q & 3) + 8 * (q >> 2) + 4 * h, j = r;  // C layout of 32x32x16
    if (i < j && j < n) o[D + tri_index(i, j, n)] = f32_to_bf16(acc[q]);
  }
}

// 4 waves (samples) per block; LDS z tile per wave: [32][D + 8] bf16
__global__ __launch_bounds__(256) void dlrm_interact_bwd_kernel(const uint16_t* __restrict__ x,
                                                                const uint16_t* __restrict__ e,
                                                                const uint16_t* __restrict__ dout,
                                                                uint16_t* __restrict__ dx, uint16_t* __restrict__ de,
                                                                int B, int T, int D) {
  extern __shared__ __attribute__((aligned(16))) uint16_t zl[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x * 4 + w;
  const bool live = b < B;  // dead waves still pass the barrier
  const int n = T + 1, P = n * (n - 1) / 2, ld = D + 8;
  uint16_t* z = zl + w * 32 * ld;
  if (live) {
    for (int c = lane; c < 32 * (D / 8); c += 64) {
      const int rr = c / (D / 8), k = (c % (D / 8)) * 8;
      u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (rr == 0) v = *reinterpret_cast<const u16x8*>(x + static_cast<int64_t>(b) * D + k);
      else if (rr < n) v = *reinterpret_cast<const u16x8*>(e + (static_cast<int64_t>(b) * T + (rr - 1)) * D + k);
      *reinterpret_cast<u16x8*>(z + rr * ld + k) = v;
    }
  }
  __syncthreads();
  if (!live) return;
  const int r = lane & 31, h = lane >> 5;
  const uint16_t* gi = dout + static_cast<int64_t>(b) * (D + P) + D;
  // G fragments (A operand): lane holds Gs[i = r][j = 16 s + 8 h + t], Gs symmetric, zero diagonal
  bf16x8_t ga[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int i = r, j = 16 * s + 8 * h + t;
      uint16_t v = 0;
      if (i < n && j < n && i != j) v = gi[i < j ? tri_index(i, j, n) : tri_index(j, i, n)];
      ga[s][t] = static_cast<short>(v);
    }
  for (int c0 = 0; c0 < D; c0 += 32) {
    f32x16v acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t bz;  // B operand: lane holds z[j = 16 s + 8 h + t][c0 + r]
#pragma unroll
      for (int t = 0; t < 8; ++t) bz[t] = static_cast<short>(z[(16 * s + 8 * h + t) * ld + c0 + r]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[s], bz, acc, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = (q & 3) + 8 * (q >> 2) + 4 * h, col = c0 + r;
      if (i == 0) {
        const float pass = bf16_to_f32(dout[static_cast<int64_t>(b) * (D + P) + col]);
        dx[static_cast<int64_t>(b) * D + col] = f32_to_bf16(acc[q] + pass);
      } else if (i < n) {
        de[(static_cast<int64_t>(b) * T + (i - 1)) * D + col] = f32_to_bf16(acc[q]);
      }
    }
  }
}

void launch_dlrm_interact_fwd(const uint16_t* x, const uint16_t* e, uint16_t* out, int B, int T, int D,
                              hipStream_t s) {
  if (B <= 0) return;
  hipLaunchKernelGGL(dlrm_interact_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, s, x, e, out, B, T, D);
}

void launch_dlrm_interact_bwd(const uint16_t* x, const uint16_t* e, const uint16_t* dout, uint16_t* dx, uint16_t* de,
                              int B, int T, int D, hipStream_t s) {
  if (B <= 0) return;
  const size_t lds = static_cast<size_t>(4) * 32 * (D + 8) * sizeof(uint16_t);
  hipLaunchKernelGGL(dlrm_interact_bwd_kernel, dim3((B + 3) / 4), dim3(256), lds, s, x, e, dout, dx, de, B, T, D);
}

}  // namespace psamd
