// Causal grouped-query flash attention (Llama-3: head dim 128, S a multiple of 128), forward and
// backward on v_mfma_f32_32x32x16_bf16 -- replaces SDPA's library kernels, whose backward ran
// at ~180 TF/s on the Llama-3-8B bench shape (profiles/r2_llama_rocprof_kernel_stats.txt).
//
// Forward / dQ (grid: query blocks of 128 x heads x batch, 4 waves of 32 queries): the block's
// keys stream through LDS 64 at a time; S^T = K Q^T is held in registers with ONE query per lane
// column, so the online softmax (running max / sum) is in-register plus one cross-half
// shuffle, P^T goes straight from the accumulators into the O^T = V^T P^T MFMAs (acc_to_b), and
// O leaves as 8-B row pieces in the [B, S, H, D] layout the output projection reads.  The dQ
// kernel recomputes P^T from the forward's log-sum-exp, forms dS^T = P^T (dO V^T - D), and
// accumulates dQ^T = K^T dS^T; it also stores D = rowsum(dO * O).
// dK / dV (grid: key blocks of 128 x KV heads x batch, 4 waves of 32 keys): every query head
// of the GQA group streams through LDS 64 queries at a time (prefetched one stage ahead); S =
// Q K^T and dP = dO V^T with ONE key per lane column, so P and dS feed dV^T += dO^T P and
// dK^T += Q^T dS straight from the accumulators, which sum the whole group in registers -- the
// backward is deterministic (no atomics, no partials).
// Forward: 8 waves (256 queries) share each K / V tile, prefetched into registers one tile ahead;
// forward and dQ grids run their heaviest (latest) query blocks first.
#include "psamd_launch.h"
#include "psamd_mfma.h"

namespace psamd {
namespace {

using namespace mfma;

constexpr int kD = 128;   // head dim
constexpr int kBQ = 128;  // queries per block (4 waves x 32)
constexpr int kBK = 64;   // keys per forward / dQ iteration
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNeg = -3.0e38f;

// [rows][128] swizzled tile from rows of stride rs elements
__device__ __forceinline__ void stage_rows(uint16_t* T, const uint16_t* src, int64_t rs, int rows) {
  for (int id = threadIdx.x; id < rows * 16; id += blockDim.x) {
    const int r = id >> 4, ch = id & 15;
    *reinterpret_cast<u16x8*>(T + off<128>(r, ch * 8)) = *reinterpret_cast<const u16x8*>(src + r * rs + ch * 8);
  }
}

__device__ __forceinline__ void store_t(const f32x16 (&acc)[4], uint16_t* row, float mul, int hl) {
  // acc^T layout: lane column = the output row, register rows d = db*32 + (e & 3) + 8 (e >> 2) + 4 hl
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const u16x4 v = {f32_to_bf16(acc[db][4 * g] * mul), f32_to_bf16(acc[db][4 * g + 1] * mul),
                       f32_to_bf16(acc[db][4 * g + 2] * mul), f32_to_bf16(acc[db][4 * g + 3] * mul)};
      *reinterpret_cast<u16x4*>(row + db * 32 + 8 * g + 4 * hl) = v;
    }
}

// ------------------------------------------------------------------------------ forward
// S^T for one 64-key block from the LDS tile (asm reads: a DMA into the other buffer is in flight)
__device__ __forceinline__ void st_block(const uint16_t* Ks, const bf16x8_t (&qf)[8], int c, int hl, f32x16 (&st)[2]) {
  zero(st[0]);
  zero(st[1]);
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    bf16x8_t a[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 4; ++j) a[ks][j] = frag_a<128>(Ks, ks * 32 + c, 2 * (4 * g + j) + hl);
    lds_wait();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 4; ++j) tie(a[ks][j]);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) st[ks] = mma(a[ks][j], qf[4 * g + j], st[ks]);
  }
}

// acc^T[d][n] += T^T[d][key] P^T[key][n] over the 64 keys of the tile (P^T in accumulator layout)
__device__ __forceinline__ void pv_block(const uint16_t* T, const f32x16 (&pt)[2], int lane, int hl, f32x16 (&acc)[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const bf16x8_t pb = acc_to_b(pt[s >> 1], s, hl);
    bf16x8_t a[4];
#pragma unroll
    for (int db = 0; db < 4; ++db) a[db] = tfrag_a<128>(T, s, db * 32, lane);
    lds_wait();
#pragma unroll
    for (int db = 0; db < 4; ++db) tie(a[db]);
#pragma unroll
    for (int db = 0; db < 4; ++db) acc[db] = mma(a[db], pb, acc[db]);
  }
}

// NW waves x 32 queries per block share each 64-key K / V tile; the tiles are prefetched into
// registers one tile ahead (issued right after the tile in LDS is published, written to LDS
// after the next barrier), so the global loads overlap the whole QK^T / softmax / PV of the
// current tile.  Query blocks run latest-first: under the causal mask the last blocks carry the
// most keys, and starting them first keeps the tail short.
template <int NW>
__global__ __launch_bounds__(NW * 64) void fa_fwd_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                                                         const uint16_t* __restrict__ v, uint16_t* __restrict__ out,
                                                         float* __restrict__ lse, int S, int H, int KV, float scale) {
  constexpr int BQ = NW * 32, NT = NW * 64;
  constexpr int CH = kBK * 16 / NT;  // 16-B chunks per thread per tensor per tile
  static_assert(CH >= 1 && kBK * 16 % NT == 0, "tile / block shape");
  __shared__ __attribute__((aligned(16))) uint16_t Ks[kBK * kD];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[kBK * kD];
  const int qb = gridDim.x - 1 - blockIdx.x, h = blockIdx.y, b = blockIdx.z, kvh = h / (H / KV);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, c = lane & 31;
  const uint16_t* qp = q + static_cast<int64_t>(b * H + h) * S * kD;
  const uint16_t* kp = k + static_cast<int64_t>(b * KV + kvh) * S * kD;
  const uint16_t* vp = v + static_cast<int64_t>(b * KV + kvh) * S * kD;
  const int q0 = qb * BQ + w * 32, qi = q0 + c;
  bf16x8_t qf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8_t*>(qp + static_cast<int64_t>(qi) * kD + 16 * s + 8 * hl);
  const int nkb = (qb * BQ + BQ - 1) / kBK + 1;
  const float k2 = scale * kLog2e;
  u16x8 kr[CH], vr[CH];
  auto gload = [&](int kb) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int id = threadIdx.x + i * NT, r = id >> 4, ch = id & 15;
      const int64_t o = static_cast<int64_t>(kb * kBK + r) * kD + ch * 8;
      kr[i] = *reinterpret_cast<const u16x8*>(kp + o);
      vr[i] = *reinterpret_cast<const u16x8*>(vp + o);
    }
  };
  auto swrite = [&]() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int id = threadIdx.x + i * NT, r = id >> 4, ch = id & 15;
      *reinterpret_cast<u16x8*>(Ks + off<128>(r, ch * 8)) = kr[i];
      *reinterpret_cast<u16x8*>(Vs + off<128>(r, ch * 8)) = vr[i];
    }
  };
  float m = kNeg, l = 0.f;
  f32x16 o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) zero(o[db]);
  gload(0);
  for (int kb = 0; kb < nkb; ++kb) {
    __syncthreads();  // the previous tile is read out
    swrite();
    __syncthreads();
    if (kb + 1 < nkb) gload(kb + 1);  // in flight behind this tile's math
    if (kb * kBK > q0 + 31) continue;  // wave-uniform: every key is in this wave's future
    f32x16 st[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      zero(st[ks]);
#pragma unroll
      for (int s = 0; s < 8; ++s) st[ks] = mma(frag<128>(Ks, ks * 32 + c, 2 * s + hl), qf[s], st[ks]);
    }
    float mb = kNeg;
    if (kb * kBK + kBK - 1 > q0) {  // the diagonal tile: mask the future keys
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int key = kb * kBK + ks * 32 + (e & 3) + 8 * (e >> 2) + 4 * hl;
          if (key > qi) st[ks][e] = kNeg;
        }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 16; ++e) mb = fmaxf(mb, st[ks][e]);
    mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
    const float mn = fmaxf(m, mb);
    const float alpha = exp2f((m - mn) * k2);
    const float mk = mn * k2;
    float ls = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float p = exp2f(st[ks][e] * k2 - mk);
        st[ks][e] = p;
        ls += p;
      }
    ls += __shfl_xor(ls, 32, 64);
    l = l * alpha + ls;
    m = mn;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int e = 0; e < 16; ++e) o[db][e] *= alpha;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8_t pb = acc_to_b(st[s >> 1], s, hl);
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db] = mma(tfrag<128>(Vs, s, db * 32, lane), pb, o[db]);
    }
  }
  store_t(o, out + (static_cast<int64_t>(b) * S + qi) * H * kD + h * kD, 1.f / l, hl);
  if (hl == 0) lse[static_cast<int64_t>(b * H + h) * S + qi] = m * scale + __logf(l);
}

// ------------------------------------------------------------------------------ backward: dQ (+ D)
__global__ __launch_bounds__(256) void fa_bwd_dq_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                                                        const uint16_t* __restrict__ v, const uint16_t* __restrict__ o,
                                                        const uint16_t* __restrict__ dout,
                                                        const float* __restrict__ lse, float* __restrict__ dsum,
                                                        uint16_t* __restrict__ dq, int S, int H, int KV, float scale) {
  __shared__ __attribute__((aligned(16))) uint16_t Ks[2][kBK * kD];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[2][kBK * kD];
  const int qb = gridDim.x - 1 - blockIdx.x, h = blockIdx.y, b = blockIdx.z, kvh = h / (H / KV);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, c = lane & 31;
  const uint16_t* qp = q + static_cast<int64_t>(b * H + h) * S * kD;
  const uint16_t* kp = k + static_cast<int64_t>(b * KV + kvh) * S * kD;
  const uint16_t* vp = v + static_cast<int64_t>(b * KV + kvh) * S * kD;
  const int q0 = qb * kBQ + w * 32, qi = q0 + c;
  const int nkb = (qb * kBQ + kBQ - 1) / kBK + 1;
  auto issue = [&](int kb) {
    dma_tile128(Ks[kb & 1], kp + static_cast<int64_t>(kb) * kBK * kD, kD, kBK, w, 4, lane);
    dma_tile128(Vs[kb & 1], vp + static_cast<int64_t>(kb) * kBK * kD, kD, kBK, w, 4, lane);
  };
  issue(0);
  const int64_t orow = (static_cast<int64_t>(b) * S + qi) * H * kD + h * kD;
  bf16x8_t qf[8], df[8];
  float dd = 0.f;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    qf[s] = *reinterpret_cast<const bf16x8_t*>(qp + static_cast<int64_t>(qi) * kD + 16 * s + 8 * hl);
    df[s] = *reinterpret_cast<const bf16x8_t*>(dout + orow + 16 * s + 8 * hl);
    const u16x8 ov = *reinterpret_cast<const u16x8*>(o + orow + 16 * s + 8 * hl);
    const u16x8 dv = __builtin_bit_cast(u16x8, df[s]);
#pragma unroll
    for (int e = 0; e < 8; ++e) dd += bf16_to_f32(ov[e]) * bf16_to_f32(dv[e]);
  }
  dd += __shfl_xor(dd, 32, 64);
  const int64_t li = static_cast<int64_t>(b * H + h) * S + qi;
  if (hl == 0) dsum[li] = dd;
  const float l2 = lse[li] * kLog2e, k2 = scale * kLog2e;
  f32x16 acc[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) zero(acc[db]);
  for (int kb = 0; kb < nkb; ++kb) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kb + 1 < nkb) issue(kb + 1);
    if (kb * kBK > q0 + 31) continue;
    f32x16 st[2], dp[2];
    st_block(Ks[kb & 1], qf, c, hl, st);
    st_block(Vs[kb & 1], df, c, hl, dp);  // dP^T = V dO^T: same shape as S^T = K Q^T
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int key = kb * kBK + ks * 32 + (e & 3) + 8 * (e >> 2) + 4 * hl;
        const float p = key > qi ? 0.f : exp2f(st[ks][e] * k2 - l2);
        st[ks][e] = p * (dp[ks][e] - dd);  // dS^T
      }
    pv_block(Ks[kb & 1], st, lane, hl, acc);  // dQ^T += K^T dS^T
  }
  store_t(acc, dq + static_cast<int64_t>(b * H + h) * S * kD + static_cast<int64_t>(qi) * kD, scale, hl);
}

// ------------------------------------------------------------------------------ backward: dK / dV
// One block per (128-key block, KV head): the block sweeps EVERY query head of its GQA group, so
// dK / dV of its keys accumulate over the group in registers and leave once, in bf16 (no per-q-
// head fp32 partials, no group-sum pass).  Queries stream through LDS 64 at a time, prefetched
// into registers one stage ahead.  Key blocks with the most queries (the first ones) run first.
constexpr int kBQS = 64;  // queries per dK / dV stage

__global__ __launch_bounds__(256) void fa_bwd_dkdv_kernel(const uint16_t* __restrict__ q,
                                                          const uint16_t* __restrict__ k,
                                                          const uint16_t* __restrict__ v,
                                                          const uint16_t* __restrict__ dout,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ dsum, uint16_t* __restrict__ dko,
                                                          uint16_t* __restrict__ dvo, int S, int H, int KV, float scale) {
  constexpr int CH = kBQS * 16 / 256;  // 16-B chunks per thread per tensor per stage
  __shared__ __attribute__((aligned(16))) uint16_t Qs[kBQS * kD];
  __shared__ __attribute__((aligned(16))) uint16_t dOs[kBQS * kD];
  __shared__ float Ls[kBQS], Ds[kBQS];
  const int kblk = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z, G = H / KV;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, c = lane & 31;
  const uint16_t* kp = k + static_cast<int64_t>(b * KV + kvh) * S * kD;
  const uint16_t* vp = v + static_cast<int64_t>(b * KV + kvh) * S * kD;
  const int k0 = kblk * kBQ + w * 32, key = k0 + c;
  bf16x8_t kf[8], vf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8_t*>(kp + static_cast<int64_t>(key) * kD + 16 * s + 8 * hl);
    vf[s] = *reinterpret_cast<const bf16x8_t*>(vp + static_cast<int64_t>(key) * kD + 16 * s + 8 * hl);
  }
  const float k2 = scale * kLog2e;
  f32x16 dk[4], dv[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    zero(dk[db]);
    zero(dv[db]);
  }
  // stages: (q head g, query stage qs) for qs from this key block's first query on
  const int qs0 = kblk * kBQ / kBQS, nqs = S / kBQS, per = nqs - qs0, nst = G * per;
  u16x8 qr[CH], dr[CH];
  float lr = 0.f, dsr = 0.f;
  auto gload = [&](int st) {
    const int g = st / per, qs = qs0 + st % per, h = kvh * G + g;
    const uint16_t* qp = q + (static_cast<int64_t>(b * H + h) * S + qs * kBQS) * kD;
    const uint16_t* dp = dout + (static_cast<int64_t>(b) * S + qs * kBQS) * H * kD + h * kD;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int id = threadIdx.x + i * 256, r = id >> 4, ch = id & 15;
      qr[i] = *reinterpret_cast<const u16x8*>(qp + static_cast<int64_t>(r) * kD + ch * 8);
      dr[i] = *reinterpret_cast<const u16x8*>(dp + static_cast<int64_t>(r) * H * kD + ch * 8);
    }
    if (threadIdx.x < kBQS) {
      const int64_t li = static_cast<int64_t>(b * H + h) * S + qs * kBQS + threadIdx.x;
      lr = lse[li] * kLog2e;
      dsr = dsum[li];
    }
  };
  auto swrite = [&]() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int id = threadIdx.x + i * 256, r = id >> 4, ch = id & 15;
      *reinterpret_cast<u16x8*>(Qs + off<128>(r, ch * 8)) = qr[i];
      *reinterpret_cast<u16x8*>(dOs + off<128>(r, ch * 8)) = dr[i];
    }
    if (threadIdx.x < kBQS) {
      Ls[threadIdx.x] = lr;
      Ds[threadIdx.x] = dsr;
    }
  };
  gload(0);
  for (int st = 0; st < nst; ++st) {
    const int qbase = (qs0 + st % per) * kBQS;
    __syncthreads();  // the previous stage is read out
    swrite();
    __syncthreads();
    if (st + 1 < nst) gload(st + 1);  // in flight behind this stage's math
#pragma unroll
    for (int sl = 0; sl < kBQS / 32; ++sl) {
      const int qr0 = qbase + sl * 32;
      if (qr0 + 31 < k0) continue;  // wave-uniform: every query precedes every key of this wave
      f32x16 sa, dp;
      zero(sa);
      zero(dp);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        sa = mma(frag<128>(Qs, sl * 32 + c, 2 * s + hl), kf[s], sa);
        dp = mma(frag<128>(dOs, sl * 32 + c, 2 * s + hl), vf[s], dp);
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int qr = sl * 32 + (e & 3) + 8 * (e >> 2) + 4 * hl;
        const float p = key > qbase + qr ? 0.f : exp2f(sa[e] * k2 - Ls[qr]);
        sa[e] = p;
        dp[e] = p * (dp[e] - Ds[qr]);  // dS
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8_t pb = acc_to_b(sa, s2, hl), sb = acc_to_b(dp, s2, hl);
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          dv[db] = mma(tfrag<128>(dOs, sl * 2 + s2, db * 32, lane), pb, dv[db]);
          dk[db] = mma(tfrag<128>(Qs, sl * 2 + s2, db * 32, lane), sb, dk[db]);
        }
      }
    }
  }
  // bf16 rows of this KV head: lane column = key, rows d -> 8-B pieces
  uint16_t* kr = dko + (static_cast<int64_t>(b * KV + kvh) * S + key) * kD;
  uint16_t* vr = dvo + (static_cast<int64_t>(b * KV + kvh) * S + key) * kD;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = db * 32 + 8 * g + 4 * hl;
      *reinterpret_cast<u16x4*>(kr + d) = u16x4{f32_to_bf16(dk[db][4 * g] * scale), f32_to_bf16(dk[db][4 * g + 1] * scale),
                                                f32_to_bf16(dk[db][4 * g + 2] * scale),
                                                f32_to_bf16(dk[db][4 * g + 3] * scale)};
      *reinterpret_cast<u16x4*>(vr + d) = u16x4{f32_to_bf16(dv[db][4 * g]), f32_to_bf16(dv[db][4 * g + 1]),
                                                f32_to_bf16(dv[db][4 * g + 2]), f32_to_bf16(dv[db][4 * g + 3])};
    }
}

}  // namespace

void launch_fa_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* out, float* lse, int B, int S,
                   int H, int KV, float scale, hipStream_t s) {
  if (S % 256 == 0)
    hipLaunchKernelGGL(fa_fwd_kernel<8>, dim3(S / 256, H, B), dim3(512), 0, s, q, k, v, out, lse, S, H, KV, scale);
  else
    hipLaunchKernelGGL(fa_fwd_kernel<4>, dim3(S / kBQ, H, B), dim3(256), 0, s, q, k, v, out, lse, S, H, KV, scale);
}

void launch_fa_bwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, const uint16_t* out, const uint16_t* dout,
                   const float* lse, float* dsum, uint16_t* dq, uint16_t* dk, uint16_t* dv, int B, int S, int H,
                   int KV, float scale, hipStream_t s) {
  hipLaunchKernelGGL(fa_bwd_dq_kernel, dim3(S / kBQ, H, B), dim3(256), 0, s, q, k, v, out, dout, lse, dsum, dq, S, H,
                     KV, scale);
  hipLaunchKernelGGL(fa_bwd_dkdv_kernel, dim3(S / kBQ, KV, B), dim3(256), 0, s, q, k, v, dout, lse, dsum, dk, dv, S,
                     H, KV, scale);
}

}  // namespace psamd
