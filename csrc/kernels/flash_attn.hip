// Causal grouped-query flash attention (Llama-3: head dim 128, S a multiple of 128), forward and
// backward on v_mfma_f32_32x32x16_bf16 -- the default attention of the Llama family; on the
// Llama-3-8B bench shape it runs ahead of SDPA's library kernels forward and backward
// (profiles/r3_flash_v3_probe.jsonl).
//
// Forward / dQ (grid: query blocks of 256 (8 waves x 32 queries) x heads x batch): the block's
// keys stream through a double-buffered LDS image 64 at a time, prefetched into registers two
// tiles ahead (one barrier per tile); S^T = K Q^T is held in registers with ONE query per lane
// column, so the online softmax (deferred reference max, running sum) is in-register plus one
// cross-half permlane32_swap, P^T goes straight from the accumulators into the O^T = V^T P^T
// MFMAs (acc_to_b), and O leaves as 8-B row pieces in the [B, S, H, D] layout the output
// projection reads.  The dQ kernel recomputes P^T from the forward's log-sum-exp, forms
// dS^T = P^T (dO V^T - D), and accumulates dQ^T = K^T dS^T; it also stores D = rowsum(dO * O).
// dK / dV (grid: key blocks of 128 x KV heads x batch, 4 waves of 32 keys): every query head
// of the GQA group streams through LDS 64 queries at a time (LDS-DMA, double buffer); S =
// Q K^T and dP = dO V^T with ONE key per lane column, so P and dS feed dV^T += dO^T P and
// dK^T += Q^T dS straight from the accumulators, which sum the whole group in registers -- the
// backward is deterministic (no atomics, no partials).
// Forward and dQ grids run their heaviest (latest) query blocks first, dK / dV its heaviest
// (earliest) key blocks first.
// The softmax is VALU work the MFMAs cannot hide in the one-wave-per-SIMD dK / dV kernel (PMC:
// 15 VALU instructions per MFMA), so it is kept lean: bare v_exp_f32 (fast_exp2), one packed
// bf16 convert per pair (pk_bf16), and the causal mask only on diagonal tiles / slices
// (profiles/r5_flash_valu_trim.txt: bwd -18 %, fwd -17 %).
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
// XCD-aware 1-D block order.  The hardware deals consecutive block ids round-robin over the 8
// XCDs, each with its own L2; a "unit" is every block that reads one (batch, KV head)'s K / V
// (forward, dQ) or Q / dO (dK / dV), so each XCD is given whole units -- block L runs on XCD
// L mod 8 and takes the (L / 8) mod per -th item of unit (L mod 8) + 8 ((L / 8) / per).  Needs
// units % 8 == 0 (else plain order).  Items run heaviest first within a unit.
__device__ __forceinline__ void xcd_unit(int L, int per, int units, int& unit, int& r) {
  if ((units & 7) == 0) {
    const int x = L & 7, j = L >> 3;
    unit = x + 8 * (j / per);
    r = j % per;
  } else {
    unit = L / per;
    r = L % per;
  }
}

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

// NW waves x 32 queries per block share each 64-key K / V tile.  The tiles are double-buffered in
// LDS and prefetched into registers two tiles ahead: tile kb + 1 is written (from registers)
// into the idle buffer right after tile kb's math, and tile kb + 2's global loads are issued
// behind it, so ONE barrier per tile publishes the next buffer and the loads overlap a whole
// QK^T / softmax / PV.  Cross-half reductions and the P^T -> B-operand relayout use
// permlane32_swap (VALU) rather than LDS shuffles, which would wait behind the in-flight
// fragment reads.  The online softmax keeps a deferred reference max (rescale only when the
// running max grows by more than 2^8 in exp2 units): O and l are exact against that reference,
// P stays <= 256.  Query blocks run latest-first: under the causal mask the last blocks carry
// the most keys, and starting them first keeps the tail short.
constexpr float kRescale = 8.f;

template <int NW>
__global__ __launch_bounds__(NW * 64) void fa_fwd_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                                                         const uint16_t* __restrict__ v, uint16_t* __restrict__ out,
                                                         float* __restrict__ lse, int S, int H, int KV, float scale) {
  constexpr int BQ = NW * 32, NT = NW * 64;
  constexpr int CH = kBK * 16 / NT;  // 16-B chunks per thread per tensor per tile
  static_assert(CH >= 1 && kBK * 16 % NT == 0, "tile / block shape");
  __shared__ __attribute__((aligned(16))) uint16_t Ks[2][kBK * kD];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[2][kBK * kD];
  const int G = H / KV, nqb = S / BQ;
  int unit, rr;
  xcd_unit(blockIdx.x, G * nqb, static_cast<int>(gridDim.x) / (G * nqb), unit, rr);
  const int b = unit / KV, kvh = unit % KV, qb = nqb - 1 - rr / G, h = kvh * G + rr % G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, c = lane & 31;
  const uint16_t* qp = q + static_cast<int64_t>(b * H + h) * S * kD;
  const uint16_t* kp = k + static_cast<int64_t>(b * KV + kvh) * S * kD;
  const uint16_t* vp = v + static_cast<int64_t>(b * KV + kvh) * S * kD;
  const int q0 = qb * BQ + w * 32, qi = q0 + c;
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
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int id = threadIdx.x + i * NT, r = id >> 4, ch = id & 15;
      *reinterpret_cast<u16x8*>(Ks[buf] + off<128>(r, ch * 8)) = kr[i];
      *reinterpret_cast<u16x8*>(Vs[buf] + off<128>(r, ch * 8)) = vr[i];
    }
  };
  gload(0);
  bf16x8_t qf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8_t*>(qp + static_cast<int64_t>(qi) * kD + 16 * s + 8 * hl);
  swrite(0);
  if (nkb > 1) gload(1);
  float m2 = -INFINITY, l = 0.f;  // reference max in exp2 units (scores * scale * log2 e)
  f32x16 o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) zero(o[db]);
  for (int kb = 0; kb < nkb; ++kb) {
    __syncthreads();  // tile kb is in LDS; every wave is done with tile kb - 1's buffer
    const uint16_t* K = Ks[kb & 1];
    const uint16_t* V = Vs[kb & 1];
    if (kb * kBK <= q0 + 31) {  // wave-uniform: skip tiles wholly in this wave's future
      f32x16 st[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        zero(st[ks]);
#pragma unroll
        for (int s = 0; s < 8; ++s) st[ks] = mma(frag<128>(K, ks * 32 + c, 2 * s + hl), qf[s], st[ks]);
      }
      if (kb * kBK + kBK - 1 > q0) {  // the diagonal tile: mask the future keys
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int key = kb * kBK + ks * 32 + (e & 3) + 8 * (e >> 2) + 4 * hl;
            if (key > qi) st[ks][e] = -INFINITY;
          }
      }
      float mb = st[0][0];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int e = 0; e < 16; ++e) mb = fmaxf(mb, st[ks][e]);
      mb = xhalf_max(mb) * k2;  // every processed tile holds >= 1 visible key per query
      if (!__all(mb - m2 <= kRescale)) {
        const float mn = fmaxf(m2, mb);
        const float alpha = fast_exp2(m2 - mn);
        l *= alpha;
#pragma unroll
        for (int db = 0; db < 4; ++db)
#pragma unroll
          for (int e = 0; e < 16; ++e) o[db][e] *= alpha;
        m2 = mn;
      }
      float ls = 0.f;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float p = fast_exp2(st[ks][e] * k2 - m2);
          st[ks][e] = p;
          ls += p;
        }
      l += xhalf_sum(ls);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8_t pb = acc_to_b(st[s >> 1], s, hl);
#pragma unroll
        for (int db = 0; db < 4; ++db) o[db] = mma(tfrag<128>(V, s, db * 32, lane), pb, o[db]);
      }
    }
    if (kb + 1 < nkb) {
      swrite((kb + 1) & 1);             // write-late: the loads had a whole tile to land
      if (kb + 2 < nkb) gload(kb + 2);  // in flight behind the next tile's math
    }
  }
  store_t(o, out + (static_cast<int64_t>(b) * S + qi) * H * kD + h * kD, 1.f / l, hl);
  if (hl == 0) lse[static_cast<int64_t>(b * H + h) * S + qi] = m2 * 0.6931471805599453f + __logf(l);
}

// ------------------------------------------------------------------------------ backward: dQ (+ D)
// The forward's structure (NW waves x 32 queries sharing double-buffered K / V tiles prefetched
// two tiles ahead, one barrier per tile), with each 64-key tile taken as two 32-key halves so S^T,
// dP^T and dS^T of only one half are live: at 8 waves the kernel fits two waves per SIMD.
template <int NW>
__global__ __launch_bounds__(NW * 64) void fa_bwd_dq_kernel(const uint16_t* __restrict__ q,
                                                            const uint16_t* __restrict__ k,
                                                            const uint16_t* __restrict__ v,
                                                            const uint16_t* __restrict__ o,
                                                            const uint16_t* __restrict__ dout,
                                                            const float* __restrict__ lse, float* __restrict__ dsum,
                                                            uint16_t* __restrict__ dq, int S, int H, int KV,
                                                            float scale) {
  constexpr int BQ = NW * 32, NT = NW * 64;
  constexpr int CH = kBK * 16 / NT;
  static_assert(CH >= 1 && kBK * 16 % NT == 0, "tile / block shape");
  __shared__ __attribute__((aligned(16))) uint16_t Ks[2][kBK * kD];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[2][kBK * kD];
  const int G = H / KV, nqb = S / BQ;
  int unit, rr;
  xcd_unit(blockIdx.x, G * nqb, static_cast<int>(gridDim.x) / (G * nqb), unit, rr);
  const int b = unit / KV, kvh = unit % KV, qb = nqb - 1 - rr / G, h = kvh * G + rr % G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, c = lane & 31;
  const uint16_t* qp = q + static_cast<int64_t>(b * H + h) * S * kD;
  const uint16_t* kp = k + static_cast<int64_t>(b * KV + kvh) * S * kD;
  const uint16_t* vp = v + static_cast<int64_t>(b * KV + kvh) * S * kD;
  const int q0 = qb * BQ + w * 32, qi = q0 + c;
  const int nkb = (qb * BQ + BQ - 1) / kBK + 1;
  u16x8 kr[CH], vr[CH];
  auto gload = [&](int kb) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int id = threadIdx.x + i * NT, r = id >> 4, ch = id & 15;
      const int64_t off_ = static_cast<int64_t>(kb * kBK + r) * kD + ch * 8;
      kr[i] = *reinterpret_cast<const u16x8*>(kp + off_);
      vr[i] = *reinterpret_cast<const u16x8*>(vp + off_);
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int id = threadIdx.x + i * NT, r = id >> 4, ch = id & 15;
      *reinterpret_cast<u16x8*>(Ks[buf] + off<128>(r, ch * 8)) = kr[i];
      *reinterpret_cast<u16x8*>(Vs[buf] + off<128>(r, ch * 8)) = vr[i];
    }
  };
  gload(0);
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
  dd = xhalf_sum(dd);
  const int64_t li = static_cast<int64_t>(b * H + h) * S + qi;
  if (hl == 0) dsum[li] = dd;
  const float l2 = lse[li] * kLog2e, k2 = scale * kLog2e;
  swrite(0);
  if (nkb > 1) gload(1);
  f32x16 acc[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) zero(acc[db]);
  for (int kb = 0; kb < nkb; ++kb) {
    __syncthreads();
    const uint16_t* K = Ks[kb & 1];
    const uint16_t* V = Vs[kb & 1];
    if (kb * kBK <= q0 + 31) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int kk0 = kb * kBK + ks * 32;
        if (kk0 > q0 + 31) continue;  // wave-uniform: this half is wholly in the future
        f32x16 st, dp;
        zero(st);
        zero(dp);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          st = mma(frag<128>(K, ks * 32 + c, 2 * s + hl), qf[s], st);
          dp = mma(frag<128>(V, ks * 32 + c, 2 * s + hl), df[s], dp);  // dP^T = V dO^T
        }
        if (kk0 + 31 > q0) {  // wave-uniform: only the diagonal half-tile needs the causal mask
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            float p = fast_exp2(st[e] * k2 - l2);
            if (kk0 + (e & 3) + 8 * (e >> 2) + 4 * hl > qi) p = 0.f;
            st[e] = p * (dp[e] - dd);  // dS^T
          }
        } else {
#pragma unroll
          for (int e = 0; e < 16; ++e) st[e] = fast_exp2(st[e] * k2 - l2) * (dp[e] - dd);
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8_t sb = acc_to_b(st, s2, hl);
#pragma unroll
          for (int db = 0; db < 4; ++db) acc[db] = mma(tfrag<128>(K, ks * 2 + s2, db * 32, lane), sb, acc[db]);
        }
      }
    }
    if (kb + 1 < nkb) {
      swrite((kb + 1) & 1);
      if (kb + 2 < nkb) gload(kb + 2);
    }
  }
  store_t(acc, dq + static_cast<int64_t>(b * H + h) * S * kD + static_cast<int64_t>(qi) * kD, scale, hl);
}

// ------------------------------------------------------------------------------ backward: dK / dV
// One block per (128-key block, KV head): the block sweeps EVERY query head of its GQA group, so
// dK / dV of its keys accumulate over the group in registers and leave once, in bf16 (no per-q-
// head fp32 partials, no group-sum pass).  Key blocks with the most queries (the first ones) run
// first.  dK / dV take 128 accumulator registers, so the kernel runs one wave per SIMD and hides
// latency inside the wave: query stages of 64 rows arrive by LDS-DMA into a double buffer (one
// barrier per stage), and per 32-query slice every LDS read is issued a phase ahead of the MFMAs
// that consume it -- L / D and the Q fragments, then the dO fragments behind the S chain, then
// all transposed dO / Q fragments behind the dP chain and under the softmax VALU work.
constexpr int kBQS = 64;  // queries per dK / dV stage

template <int N>
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ f32x4 lds_f4(const float* p) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(reinterpret_cast<const uint16_t*>(p))) : "memory");
  return v;
}
__device__ __forceinline__ void tie4(f32x4& v) { asm volatile("" : "+v"(v)); }

__global__ __launch_bounds__(256) void fa_bwd_dkdv_kernel(const uint16_t* __restrict__ q,
                                                          const uint16_t* __restrict__ k,
                                                          const uint16_t* __restrict__ v,
                                                          const uint16_t* __restrict__ dout,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ dsum, uint16_t* __restrict__ dko,
                                                          uint16_t* __restrict__ dvo, int S, int H, int KV, float scale) {
  __shared__ __attribute__((aligned(16))) uint16_t Qs[2][kBQS * kD];
  __shared__ __attribute__((aligned(16))) uint16_t dOs[2][kBQS * kD];
  __shared__ __attribute__((aligned(16))) float Ls[2][kBQS];
  __shared__ __attribute__((aligned(16))) float Ds[2][kBQS];
  const int G = H / KV, nkb = S / kBQ;
  int unit, kblk;
  xcd_unit(blockIdx.x, nkb, static_cast<int>(gridDim.x) / nkb, unit, kblk);
  const int b = unit / KV, kvh = unit % KV;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, c = lane & 31;
  const uint16_t* kp = k + static_cast<int64_t>(b * KV + kvh) * S * kD;
  const uint16_t* vp = v + static_cast<int64_t>(b * KV + kvh) * S * kD;
  const int k0 = kblk * kBQ + w * 32, key = k0 + c;
  // stages: (q head g, query stage qs) for qs from this key block's first query on
  const int qs0 = kblk * kBQ / kBQS, nqs = S / kBQS, per = nqs - qs0, nst = G * per;
  auto issue = [&](int st) {
    const int g = st / per, qs = qs0 + st % per, h = kvh * G + g, buf = st & 1;
    const int64_t li = static_cast<int64_t>(b * H + h) * S + qs * kBQS;
    dma_tile128(Qs[buf], q + li * kD, kD, kBQS, w, 4, lane);
    dma_tile128(dOs[buf], dout + (static_cast<int64_t>(b) * S + qs * kBQS) * H * kD + h * kD, static_cast<int64_t>(H) * kD,
                kBQS, w, 4, lane);
    if (w == 0) __builtin_amdgcn_global_load_lds((gptr_t*)(lse + li + lane), (lptr_t*)Ls[buf], 4, 0, 0);
    if (w == 1) __builtin_amdgcn_global_load_lds((gptr_t*)(dsum + li + lane), (lptr_t*)Ds[buf], 4, 0, 0);
  };
  issue(0);
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
  for (int st = 0; st < nst; ++st) {
    const int qbase = (qs0 + st % per) * kBQS, buf = st & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // stage st landed everywhere; stage st - 1's buffer is read out
    if (st + 1 < nst) issue(st + 1);
    const uint16_t* Q = Qs[buf];
    const uint16_t* dO = dOs[buf];
#pragma unroll
    for (int sl = 0; sl < kBQS / 32; ++sl) {
      const int qr0 = qbase + sl * 32;
      if (qr0 + 31 < k0) continue;  // wave-uniform: every query precedes every key of this wave
      f32x4 lv[4], dv4[4];
      bf16x8_t qa[8], da[8];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        lv[g] = lds_f4(Ls[buf] + sl * 32 + 8 * g + 4 * hl);
        dv4[g] = lds_f4(Ds[buf] + sl * 32 + 8 * g + 4 * hl);
      }
#pragma unroll
      for (int s = 0; s < 8; ++s) qa[s] = frag_a<128>(Q, sl * 32 + c, 2 * s + hl);
#pragma unroll
      for (int s = 0; s < 8; ++s) da[s] = frag_a<128>(dO, sl * 32 + c, 2 * s + hl);
      lgkm_wait<8>();
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        tie4(lv[g]);
        tie4(dv4[g]);
      }
#pragma unroll
      for (int s = 0; s < 8; ++s) tie(qa[s]);
      f32x16 sa, dp;
      zero(sa);
      zero(dp);
#pragma unroll
      for (int s = 0; s < 8; ++s) sa = mma(qa[s], kf[s], sa);
      lgkm_wait<0>();
#pragma unroll
      for (int s = 0; s < 8; ++s) tie(da[s]);
#pragma unroll
      for (int s = 0; s < 8; ++s) dp = mma(da[s], vf[s], dp);
      bf16x8_t ta[2][4], tq[2][4];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          ta[s2][db] = tfrag_a<128>(dO, sl * 2 + s2, db * 32, lane);
          tq[s2][db] = tfrag_a<128>(Q, sl * 2 + s2, db * 32, lane);
        }
      if (k0 + 31 > qr0) {  // wave-uniform: only slices on the diagonal need the causal mask
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float p = fast_exp2(sa[e] * k2 - lv[e >> 2][e & 3] * kLog2e);
          if (key > qr0 + (e & 3) + 8 * (e >> 2) + 4 * hl) p = 0.f;
          sa[e] = p;
          dp[e] = p * (dp[e] - dv4[e >> 2][e & 3]);  // dS
        }
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float p = fast_exp2(sa[e] * k2 - lv[e >> 2][e & 3] * kLog2e);
          sa[e] = p;
          dp[e] = p * (dp[e] - dv4[e >> 2][e & 3]);
        }
      }
      lgkm_wait<0>();
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          tie(ta[s2][db]);
          tie(tq[s2][db]);
        }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8_t pb = acc_to_b(sa, s2, hl), sb = acc_to_b(dp, s2, hl);
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          dv[db] = mma(ta[s2][db], pb, dv[db]);
          dk[db] = mma(tq[s2][db], sb, dk[db]);
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
    hipLaunchKernelGGL(fa_fwd_kernel<8>, dim3(S / 256 * H * B), dim3(512), 0, s, q, k, v, out, lse, S, H, KV, scale);
  else
    hipLaunchKernelGGL(fa_fwd_kernel<4>, dim3(S / kBQ * H * B), dim3(256), 0, s, q, k, v, out, lse, S, H, KV, scale);
}

void launch_fa_bwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, const uint16_t* out, const uint16_t* dout,
                   const float* lse, float* dsum, uint16_t* dq, uint16_t* dk, uint16_t* dv, int B, int S, int H,
                   int KV, float scale, hipStream_t s) {
  if (S % 256 == 0)
    hipLaunchKernelGGL(fa_bwd_dq_kernel<8>, dim3(S / 256 * H * B), dim3(512), 0, s, q, k, v, out, dout, lse, dsum, dq, S,
                       H, KV, scale);
  else
    hipLaunchKernelGGL(fa_bwd_dq_kernel<4>, dim3(S / kBQ * H * B), dim3(256), 0, s, q, k, v, out, dout, lse, dsum, dq, S,
                       H, KV, scale);
  hipLaunchKernelGGL(fa_bwd_dkdv_kernel, dim3(S / kBQ * KV * B), dim3(256), 0, s, q, k, v, dout, lse, dsum, dk, dv, S,
                     H, KV, scale);
}

}  // namespace psamd
