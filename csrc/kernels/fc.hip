// Fused FC-layer backward (K2 in SURVEY §2.5), bf16 and fp32, on MFMA.
//
// Reference: layer/FcLayer.java:93-110 -- delta = act'(delta); db = rowMean(delta);
// dW = delta . A^T / N; delta_prev = W^T . delta.  The activation backward is folded into the
// PROLOGUE of both GEMMs (dz = act'(y) * dy is formed while the dy tile is staged, it is never
// written), the bias gradient is reduced from the same staged tile (the "rowMean fused into the
// dW epilogue"), and the operands are used where they lie: dy [M, N], x [M, K] and W [N, K]
// are all row-major, the reduction index of both GEMMs is their SLOW index for one operand,
// so that operand is transposed while it is staged into LDS (no transposed copy in HBM).
//
//   fc_bwd_dw :  dW[N, K] = sum_m dz[m, n] x[m, k]   (+ db[n] = sum_m dz[m, n])
//   fc_bwd_dx :  dX[M, K] = sum_n dz[m, n] W[n, k]
//
// Tiles: 256 threads = 4 waves, C tile 64x64, reduction 32 per stage, each wave a 32x32 quarter
// = 2x2 16x16 MFMA tiles; bf16 operands use v_mfma_f32_16x16x32_bf16 (one 16-B LDS read per
// operand per MFMA), fp32 operands v_mfma_f32_16x16x4_f32 (fp32 end to end for the
// reference-parity fp32 models).  Operand pieces move as 16-B vector loads (8 contiguous
// elements per thread, in either staging layout) into registers one stage ahead, and land in a
// double-buffered LDS tile after the current stage's MFMAs (one barrier per stage).
// Activation codes as dense.hip: 0 none, 1 relu, 2 leaky 0.01, 3 reference clipped sigmoid
// (backward dy * y * (1 - y) on the clipped output, Sigmoid.java).
#include <algorithm>

#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {
namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr int kT = 64;   // C tile rows / cols
constexpr int kR = 32;   // reduction per stage
constexpr int kPad = 8;  // LDS row padding (elements)
constexpr int kTile = (kT * (kR + kPad) > kR * (kT + kPad)) ? kT * (kR + kPad) : kR * (kT + kPad);  // either layout

template <typename T> struct Ld;
template <> struct Ld<float> {
  __device__ __forceinline__ static float get(const float* p, int64_t i) { return p[i]; }
};
template <> struct Ld<uint16_t> {
  __device__ __forceinline__ static float get(const uint16_t* p, int64_t i) { return bf16_to_f32(p[i]); }
};

__device__ __forceinline__ float act_grad(float g, float y, int act) {
  if (act == 1) return y > 0.f ? g : 0.f;
  if (act == 2) return y > 0.f ? g : 0.01f * g;
  if (act == 3) return g * y * (1.f - y);
  return g;
}

// One thread's share of a 64 x 32 operand stage: 8 consecutive elements of ONE memory row -- 8
// reduction elements of one C-row (k contiguous) or, TRANS (element (row, k) at src[k * ld +
// row]), 8 C-rows of one reduction row.  Either way they are contiguous in memory, so an aligned
// in-range piece is one 16-B load (bf16) or two (fp32); tails and odd strides go element-wise.
// GRAD also loads y at the same offsets for the act' prologue.
template <typename T>
__device__ __forceinline__ void load8(const T* __restrict__ p, int64_t o, int nvalid, bool vec, float (&v)[8]) {
  if (vec) {
    if constexpr (sizeof(T) == 2) {
      const u16x8 q = *reinterpret_cast<const u16x8*>(p + o);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf16_to_f32(q[j]);
    } else {
      const f32x4v a = *reinterpret_cast<const f32x4v*>(p + o), b = *reinterpret_cast<const f32x4v*>(p + o + 4);
      v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
      v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = j < nvalid ? Ld<T>::get(p, o + j) : 0.f;
  }
}

template <typename T, bool TRANS, bool GRAD>
struct StageRegs8 {
  float v[8];
  float y[GRAD ? 8 : 1];
  // global -> registers (issued a stage ahead of its use)
  __device__ __forceinline__ void load(const T* __restrict__ src, const T* __restrict__ ysrc, int64_t ld, int rows,
                                       int kdim, int r0, int k0) {
    const int t = threadIdx.x;
    int64_t o;
    int nvalid;
    if constexpr (TRANS) {
      const int gk = k0 + (t >> 3), row = r0 + (t & 7) * 8;  // 32 reduction rows x 8 chunks of 8 C-rows
      nvalid = gk < kdim ? min(8, rows - row) : 0;
      o = static_cast<int64_t>(gk) * ld + row;
    } else {
      const int grow = r0 + (t >> 2), gk = k0 + (t & 3) * 8;  // 64 C-rows x 4 chunks of 8 reduction elements
      nvalid = grow < rows ? min(8, kdim - gk) : 0;
      o = static_cast<int64_t>(grow) * ld + gk;
    }
    nvalid = nvalid < 0 ? 0 : nvalid;
    const bool vec = nvalid == 8 && (o & (16 / sizeof(T) - 1)) == 0;
    load8<T>(src, o, nvalid, vec, v);
    if constexpr (GRAD) load8<T>(ysrc, o, nvalid, vec, y);
  }
  // registers -> LDS with one 16-B store per 8 elements (bf16) or two (fp32): the tile keeps the
  // memory layout -- [row][k] (ld kR + kPad) or, TRANS, [k][row] (ld kT + kPad) -- and the MFMA
  // fragments of a TRANS tile are read transposed (mma_stage).  act' applied, bias-gradient
  // partials accumulated (DB) on the way.
  template <bool DB>
  __device__ __forceinline__ void store(T* lds, int act, float (&dbacc)[8]) {
    const int t = threadIdx.x;
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x[j] = v[j];
      if constexpr (GRAD) x[j] = act_grad(x[j], y[j], act);
      if constexpr (TRANS && DB) dbacc[j] += x[j];
    }
    T* dst = TRANS ? lds + (t >> 3) * (kT + kPad) + (t & 7) * 8 : lds + (t >> 2) * (kR + kPad) + (t & 3) * 8;
    if constexpr (sizeof(T) == 2) {
      u16x8 q;
#pragma unroll
      for (int j = 0; j < 8; ++j) q[j] = f32_to_bf16(x[j]);
      *reinterpret_cast<u16x8*>(dst) = q;
    } else {
      *reinterpret_cast<f32x4v*>(dst) = f32x4v{x[0], x[1], x[2], x[3]};
      *reinterpret_cast<f32x4v*>(dst + 4) = f32x4v{x[4], x[5], x[6], x[7]};
    }
  }
};

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// 16x16x32 bf16 operand of C-rows r0 .. r0+15: lane l takes (row r0 + (l & 15), k = 8 (l >> 4) + e).
// [row][k] tile: one 16-B row read.  [k][row] tile (TRANS): two ds_read_b64_tr_b16, each over a
// 16-lane group reading a 4 (k) x 16 (row) block and handing every lane one row's 4 values.
template <bool TRANS>
__device__ __forceinline__ bf16x8_t frag16(const uint16_t* T, int r0, int lane) {
  if constexpr (!TRANS) {
    return *reinterpret_cast<const bf16x8_t*>(&T[(r0 + (lane & 15)) * (kR + kPad) + (lane >> 4) * 8]);
  } else {
    const int g = lane >> 4, i = lane & 15;
    const uint16_t* a0 = T + (8 * g + (i >> 2)) * (kT + kPad) + r0 + 4 * (i & 3);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * (kT + kPad)));
    return __builtin_bit_cast(bf16x8_t, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
  }
}

// 16x16x4 f32 operand: lane l takes (row r0 + (l & 15), k = 4 s + (l >> 4)); a [k][row] tile gives
// 16 consecutive rows of one k per 16-lane group (conflict-free), a [row][k] tile a strided read.
template <bool TRANS>
__device__ __forceinline__ float frag4(const float* T, int r0, int s, int lane) {
  if constexpr (TRANS) return T[(4 * s + (lane >> 4)) * (kT + kPad) + r0 + (lane & 15)];
  else return T[(r0 + (lane & 15)) * (kR + kPad) + 4 * s + (lane >> 4)];
}

template <typename T, bool TA, bool TB>
__device__ __forceinline__ void mma_stage(const T* la, const T* lb, int wm, int wn, int lane, f32x4v (&acc)[2][2]) {
  if constexpr (sizeof(T) == 2) {
    bf16x8_t af[2], bf[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      af[i] = frag16<TA>(reinterpret_cast<const uint16_t*>(la), wm + i * 16, lane);
      bf[i] = frag16<TB>(reinterpret_cast<const uint16_t*>(lb), wn + i * 16, lane);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
  } else {
#pragma unroll
    for (int s = 0; s < kR / 4; ++s) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = frag4<TA>(reinterpret_cast<const float*>(la), wm + i * 16, s, lane);
        b[i] = frag4<TB>(reinterpret_cast<const float*>(lb), wn + i * 16, s, lane);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
}

// C[R, Cc] = sum_k A'[r][k] B'[c][k]; A' from (a, ay) with the act' prologue, TA / TB select
// the transposed staging of A' / B'.  DB: blocks of column tile 0 also write dbias[r] = sum_k A'[r][k].
template <typename T, bool TA, bool TB, bool DB, typename OT = T>
__device__ __forceinline__ void fc_bwd_body(const T* __restrict__ a, const T* __restrict__ ay, int64_t lda,
                                            const T* __restrict__ b, int64_t ldb, OT* __restrict__ c, int64_t ldc,
                                            float* __restrict__ dbias, int R, int Cc, int K, int act,
                                            T (*lds)[2][kTile], float (*dbl)[9], int kbeg = 0, int kend = -1) {
  if (kend < 0) kend = K;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int r0 = blockIdx.y * kT, c0 = blockIdx.x * kT;
  const bool db_here = DB && blockIdx.x == 0;
  f32x4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
  float dbacc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // register-staged double buffer: stage q + 1's global loads are in flight during stage q's
  // MFMAs, written to the idle LDS buffer after them -- one barrier per stage
  StageRegs8<T, TA, true> ra;
  StageRegs8<T, TB, false> rb;
  ra.load(a, ay, lda, R, kend, r0, kbeg);
  rb.load(b, nullptr, ldb, Cc, kend, c0, kbeg);
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += kR) {
    if (db_here) ra.template store<TA>(lds[buf][0], act, dbacc);
    else ra.template store<false>(lds[buf][0], act, dbacc);
    rb.template store<false>(lds[buf][1], 0, dbacc);
    __syncthreads();
    if (k0 + kR < kend) {
      ra.load(a, ay, lda, R, kend, r0, k0 + kR);
      rb.load(b, nullptr, ldb, Cc, kend, c0, k0 + kR);
    }
    mma_stage<T, TA, TB>(lds[buf][0], lds[buf][1], wm, wn, lane, acc);
    buf ^= 1;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = c0 + wn + j * 16 + (lane & 15);
      if (col >= Cc) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = r0 + wm + i * 16 + (lane >> 4) * 4 + q;
        if (row < R) Elem<OT>::store(c, static_cast<int64_t>(row) * ldc + col, acc[i][j][q]);
      }
    }
  if constexpr (DB && TA) {
    if (!db_here) return;
    // thread t staged C-rows (t & 7) * 8 .. +7 at reduction rows t >> 3 (+ 32 s): sum the 32
    // reduction-row partials of each C-row
#pragma unroll
    for (int j = 0; j < 8; ++j) dbl[threadIdx.x][j] = dbacc[j];
    __syncthreads();
    if (threadIdx.x < kT) {
      const int rc = threadIdx.x >> 3, j = threadIdx.x & 7;
      float s = 0.f;
      for (int k = 0; k < 32; ++k) s += dbl[k * 8 + rc][j];
      const int row = r0 + rc * 8 + j;
      if (row < R) dbias[row] = s;
    }
  }
}

// dW and dX are independent: ONE launch runs both (grid z = job), so a small layer's two GEMMs
// share the machine instead of running back to back.
struct FcJob {
  const void* a;
  const void* ay;
  int64_t lda;
  const void* b;
  int64_t ldb;
  void* c;
  int64_t ldc;
  float* dbias;
  int R, Cc, K;
};

// dW's reduction runs over the batch (M): a small layer at a large batch has few output tiles
// and a long serial K loop, so the reduction splits over grid z into fp32 slabs (plus bias-
// gradient slabs) that a fixed-order reduce sums -- deterministic, no atomics.
template <typename T, bool DB>
__global__ __launch_bounds__(256) void fc_bwd_kernel(FcJob dw, FcJob dx, int zoff, int nsplit, int kchunk,
                                                     float* __restrict__ ws, int act) {
  __shared__ __attribute__((aligned(16))) T lds[2][2][kTile];  // [buffer][operand]
  __shared__ float dbl[256][9];
  const int z = static_cast<int>(blockIdx.z) + zoff;
  if (z < nsplit) {  // dW[N, K] (split z): A' = dz^T (reduction m = slow index of dy), B' = x^T
    if (static_cast<int>(blockIdx.x) * kT >= dw.Cc || static_cast<int>(blockIdx.y) * kT >= dw.R) return;
    const int kb = z * kchunk, ke = std::min(dw.K, kb + kchunk);
    if (nsplit == 1)
      fc_bwd_body<T, true, true, DB>(static_cast<const T*>(dw.a), static_cast<const T*>(dw.ay), dw.lda,
                                     static_cast<const T*>(dw.b), dw.ldb, static_cast<T*>(dw.c), dw.ldc, dw.dbias,
                                     dw.R, dw.Cc, dw.K, act, lds, dbl);
    else
      fc_bwd_body<T, true, true, DB, float>(static_cast<const T*>(dw.a), static_cast<const T*>(dw.ay), dw.lda,
                                            static_cast<const T*>(dw.b), dw.ldb,
                                            ws + static_cast<int64_t>(z) * dw.R * dw.Cc, dw.ldc,
                                            DB ? ws + static_cast<int64_t>(nsplit) * dw.R * dw.Cc + z * dw.R : nullptr,
                                            dw.R, dw.Cc, dw.K, act, lds, dbl, kb, ke);
  } else {  // dX[M, K]: A' = dz (reduction n contiguous), B' = W^T (reduction n = slow index of W)
    if (static_cast<int>(blockIdx.x) * kT >= dx.Cc || static_cast<int>(blockIdx.y) * kT >= dx.R) return;
    fc_bwd_body<T, false, true, false>(static_cast<const T*>(dx.a), static_cast<const T*>(dx.ay), dx.lda,
                                       static_cast<const T*>(dx.b), dx.ldb, static_cast<T*>(dx.c), dx.ldc, nullptr,
                                       dx.R, dx.Cc, dx.K, act, lds, dbl);
  }
}

// out[e] = sum_s slab[s][e] in split order (e < n), the bias slabs into db
template <typename T>
__global__ __launch_bounds__(256) void fc_slab_reduce_kernel(const float* __restrict__ ws, int nsplit, int64_t n,
                                                             T* __restrict__ out, int nb, float* __restrict__ db) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) {
    float acc = 0.f;
    for (int z = 0; z < nsplit; ++z) acc += ws[z * n + i];
    Elem<T>::store(out, i, acc);
  } else if (db != nullptr && i < n + nb) {
    const float* b = ws + static_cast<int64_t>(nsplit) * n;
    float acc = 0.f;
    for (int z = 0; z < nsplit; ++z) acc += b[z * nb + (i - n)];
    db[i - n] = acc;
  }
}

}  // namespace

// dW reduction splits: fill ~256 blocks, each split >= 4 stages of 32
int fc_dw_splits(int M, int N, int K) {
  const int tiles = ((N + kT - 1) / kT) * ((K + kT - 1) / kT);
  const int stages = (M + kR - 1) / kR;
  if (tiles >= 256 || stages < 8) return 1;
  int s = std::min((256 + tiles - 1) / tiles, stages / 4);
  return std::max(1, std::min(s, 16));
}

int64_t fc_bwd_ws_floats(int M, int N, int K) {
  const int s = fc_dw_splits(M, N, K);
  return s > 1 ? static_cast<int64_t>(s) * (static_cast<int64_t>(N) * K + N) : 0;
}

namespace {

template <typename T>
void launch_fc(const void* dy, const void* y, const void* x, const void* w, void* dw, float* db, void* dx, int M,
               int N, int K, int act, float* ws, hipStream_t s) {
  if (dw == nullptr && dx == nullptr) return;
  const FcJob jw{dy, y, static_cast<int64_t>(N), x, static_cast<int64_t>(K), dw, static_cast<int64_t>(K), db, N, K, M};
  const FcJob jx{dy, y, static_cast<int64_t>(N), w, static_cast<int64_t>(K), dx, static_cast<int64_t>(K), nullptr, M, K,
                 N};
  const int nsplit = dw != nullptr && ws != nullptr ? fc_dw_splits(M, N, K) : 1;
  const int kchunk = ((M + nsplit - 1) / nsplit + kR - 1) / kR * kR;
  const int zoff = dw != nullptr ? 0 : nsplit, nz = (dw != nullptr ? nsplit : 0) + (dx != nullptr);
  const int gx = (K + kT - 1) / kT;
  int gy = 0;
  if (dw != nullptr) gy = std::max(gy, (N + kT - 1) / kT);
  if (dx != nullptr) gy = std::max(gy, (M + kT - 1) / kT);
  const dim3 grid(gx, gy, nz);
  if (db != nullptr && dw != nullptr)
    hipLaunchKernelGGL((fc_bwd_kernel<T, true>), grid, dim3(256), 0, s, jw, jx, zoff, nsplit, kchunk, ws, act);
  else
    hipLaunchKernelGGL((fc_bwd_kernel<T, false>), grid, dim3(256), 0, s, jw, jx, zoff, nsplit, kchunk, ws, act);
  if (nsplit > 1) {
    const int64_t n = static_cast<int64_t>(N) * K;
    const int nb = db != nullptr ? N : 0;
    hipLaunchKernelGGL((fc_slab_reduce_kernel<T>), dim3(static_cast<unsigned>((n + nb + 255) / 256)), dim3(256), 0, s,
                       ws, nsplit, n, static_cast<T*>(dw), nb, db);
  }
}

// Forward for fp32 operands: Y = act(X W^T + b) on v_mfma_f32_16x16x4_f32 (the bf16 forward is
// dense.hip's gemm_nt).  Both operands are K-contiguous: no transposed staging.
__global__ __launch_bounds__(256) void fc_fwd_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ bias, float* __restrict__ y, int M,
                                                          int N, int K, int act) {
  __shared__ __attribute__((aligned(16))) float lds[2][2][kTile];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int r0 = blockIdx.y * kT, c0 = blockIdx.x * kT;
  f32x4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
  float unused[8];
  StageRegs8<float, false, false> ra, rb;
  ra.load(x, nullptr, K, M, K, r0, 0);
  rb.load(w, nullptr, K, N, K, c0, 0);
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += kR) {
    ra.template store<false>(lds[buf][0], 0, unused);
    rb.template store<false>(lds[buf][1], 0, unused);
    __syncthreads();
    if (k0 + kR < K) {
      ra.load(x, nullptr, K, M, K, r0, k0 + kR);
      rb.load(w, nullptr, K, N, K, c0, k0 + kR);
    }
    mma_stage<float, false, false>(lds[buf][0], lds[buf][1], wm, wn, lane, acc);
    buf ^= 1;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = c0 + wn + j * 16 + (lane & 15);
      if (col >= N) continue;
      const float bv = bias ? bias[col] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = r0 + wm + i * 16 + (lane >> 4) * 4 + q;
        if (row >= M) continue;
        float v = acc[i][j][q] + bv;
        if (act == 1) v = v > 0.f ? v : 0.f;
        else if (act == 2) v = v > 0.f ? v : 0.01f * v;
        else if (act == 3) v = 0.001f + 0.998f / (1.f + __expf(-v));
        y[static_cast<int64_t>(row) * N + col] = v;
      }
    }
}

}  // namespace

void launch_fc_bwd(const void* dy, const void* y, const void* x, const void* w, void* dw, float* db, void* dx,
                   int dtype, int M, int N, int K, int act, float* ws, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return;
  if (dtype == 1) launch_fc<uint16_t>(dy, y, x, w, dw, db, dx, M, N, K, act, ws, s);
  else launch_fc<float>(dy, y, x, w, dw, db, dx, M, N, K, act, ws, s);
}

void launch_fc_fwd_f32(const float* x, const float* w, const float* b, float* y, int M, int N, int K, int act,
                       hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  dim3 grid((N + kT - 1) / kT, (M + kT - 1) / kT);
  hipLaunchKernelGGL(fc_fwd_f32_kernel, grid, dim3(256), 0, s, x, w, b, y, M, N, K, act);
}

}  // namespace psamd
