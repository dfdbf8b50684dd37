// Fused multi-head self-attention for short sequences (BERT: S <= 128, head dim 64), forward and
// backward, on v_mfma_f32_32x32x16_bf16 -- replaces SDPA's library kernels for the BERT config,
// whose backward ran at ~60 TF/s (6x its forward) with the attention-probability dropout on.
//
// One workgroup per (batch, head), 4 waves; wave w owns queries [32w, 32w + 32) (and, in the
// backward, keys [32w, 32w + 32)).  The whole sequence of one head fits on chip, so there is no
// online softmax: S^T = K Q^T is held in registers (32 keys x 32 queries per MFMA block, a
// lane owns ONE query column -> the softmax over keys is in-register plus one cross-half
// shuffle), P^T feeds the O^T = V^T P^T GEMM straight from registers (an xor-32 exchange turns
// the accumulator layout into the B-operand layout), and every output leaves as 8-B row pieces.
// I/O is in the Linear layouts: q / k / v are read from the fused qkv projection output
// [B, S, 3, H, 64] and O is written as [B, S, H * 64] (no head split / merge copies); the
// backward writes dq / dk / dv into one [B, S, 3, H, 64] gradient (no concatenation).
//
// Dropout on the attention probabilities: element e = (bh * S + i) * S + j is kept if its 16-bit
// half of hash(seed, e >> 1) is >= p * 2^16 (one hash per key pair), regenerated in the backward
// (nothing stored); kept values scaled by 1 / (1 - p).
// The backward stores the per-row log-sum-exp of the forward and recomputes P:
//   dV = P_drop^T dO,   dP = (dO V^T) * mask / (1 - p),   dS = P * (dP - rowsum(dO * O)),
//   dQ = scale dS K,    dK = scale dS^T Q.
// LDS tiles are row-major with a 16-B chunk XOR swizzle that keeps both access kinds conflict
// free: direct ds_read_b128 fragments (16 rows, one chunk) and transposed ds_read_b64_tr_b16
// fragments (4 consecutive rows x 64 B).
#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kD = 64;    // head dim
constexpr int kS = 128;   // max sequence length
constexpr float kLog2e = 1.4426950408889634f;

// 128-B rows (RL 64): chunk ^ f(row pair), f(p) = ((p & 1) << 2) | (p >> 1) on p = (r >> 1) & 7
// 256-B rows (RL 128): chunk ^ (((r & 3) << 2) | ((r >> 2) & 3))
template <int RL>
__device__ __forceinline__ int sw(int r) {
  if constexpr (RL == 64) {
    const int p = (r >> 1) & 7;
    return ((p & 1) << 2) | (p >> 1);
  } else {
    return ((r & 3) << 2) | ((r >> 2) & 3);
  }
}
template <int RL>
__device__ __forceinline__ int off(int r, int col) {
  return r * RL + (((col >> 3) ^ sw<RL>(r)) << 3) + (col & 7);
}

// direct fragment: row r, logical 16-B chunk ch
template <int RL>
__device__ __forceinline__ bf16x8_t frag(const uint16_t* T, int r, int ch) {
  return *reinterpret_cast<const bf16x8_t*>(T + r * RL + ((ch ^ sw<RL>(r)) << 3));
}

// transposed fragment: lane l receives T[16 s + 8 (l >> 5) + j][c0 + (l & 31)], j = 0..7
// (the B-operand layout of a [k][n] tile, or the A operand of its transpose)
template <int RL>
__device__ __forceinline__ bf16x8_t tfrag(const uint16_t* T, int s, int c0, int lane) {
  const int gi = lane >> 4, i16 = lane & 15;
  const int r = 16 * s + 8 * (gi >> 1) + (i16 >> 2);
  const int col = c0 + 16 * (gi & 1) + 4 * (i16 & 3);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(T + off<RL>(r, col)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(T + off<RL>(r + 4, col)));
  return __builtin_bit_cast(bf16x8_t, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// one 32-bit hash per PAIR of elements (2j, 2j + 1): a 16-bit draw each, kept if >= p * 2^16.
// The 64-bit seed folds into one 32-bit key (uniform: scalar ALU), so a pair costs ONE avalanche
// finalizer (bijective in the pair index): the dropout hash had been the largest VALU item of the
// fused attention kernels (two finalizers per pair, ~85 VALU per MFMA in the forward).
__device__ __forceinline__ uint32_t pair_hash(uint64_t seed, uint32_t pair) {
  const uint32_t k = static_cast<uint32_t>(seed) ^ (static_cast<uint32_t>(seed >> 32) * 0x9E3779B9u);
  return mix32(pair ^ k);
}
__device__ __forceinline__ bool keep_lo(uint32_t h, uint32_t thr) { return (h & 0xffffu) >= thr; }
__device__ __forceinline__ bool keep_hi(uint32_t h, uint32_t thr) { return (h >> 16) >= thr; }

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return pk_bf16(a, b);
}

// B operand (keys 16 s + 8 hl + e, query = lane column) of P^T held in the accumulator layout
// of its 32-key block: lane half hl holds keys (q & 3) + 8 (q >> 2) + 4 hl.  Half 0 needs keys
// 0..7 of the 16-key step = its own 4 + the partner's 4; half 1 needs 8..15 = partner's 4 + own 4.
__device__ __forceinline__ bf16x8_t p_operand(const f32x16& blk, int s, int hl) {
  const int qb = 8 * (s & 1);
  // pack own values as bf16 pairs: lo = keys qb..qb+3, hi = qb+4..qb+7 (in register order)
  const uint32_t lo0 = pack2(blk[qb + 0], blk[qb + 1]), lo1 = pack2(blk[qb + 2], blk[qb + 3]);
  const uint32_t hi0 = pack2(blk[qb + 4], blk[qb + 5]), hi1 = pack2(blk[qb + 6], blk[qb + 7]);
  // one permlane32_swap per pair (VALU, no LDS queue): {own lo, partner lo} on half 0,
  // {partner hi, own hi} on half 1 -- see mfma::acc_to_b (psamd_mfma.h)
  (void)hl;
  const auto a = __builtin_amdgcn_permlane32_swap(lo0, hi0, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(lo1, hi1, false, false);
  return __builtin_bit_cast(bf16x8_t, u32x4{a[0], b[0], a[1], b[1]});
}

// stage rows [0, S) of N heads' 64-wide slices (row strides rs[i] elements) into [128][64] tiles,
// rows S..127 zeroed; 256 threads: every chunk's global load is issued before any LDS store (a
// load-store loop paid one HBM round trip per 4 KiB: the kernels ran at ~2.4 TB/s)
template <int N>
__device__ __forceinline__ void stage64n(uint16_t* const (&T)[N], const uint16_t* const (&src)[N],
                                         const int64_t (&rs)[N], int S) {
  constexpr int PER = kS * 8 / 256;  // 16-B chunks per thread per tile
  u16x8 v[N][PER];
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = threadIdx.x + i * 256, r = id >> 3, ch = id & 7;
      v[n][i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (r < S) v[n][i] = *reinterpret_cast<const u16x8*>(src[n] + r * rs[n] + ch * 8);
    }
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = threadIdx.x + i * 256, r = id >> 3, ch = id & 7;
      *reinterpret_cast<u16x8*>(T[n] + off<64>(r, ch * 8)) = v[n][i];
    }
}


// ------------------------------------------------------------------------------ forward
template <bool DROP>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ out,
                                                       float* __restrict__ lse, int S, int H, float scale,
                                                       uint64_t seed, uint32_t thr, float rkeep) {
  __shared__ __attribute__((aligned(16))) uint16_t Ks[kS * kD];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[kS * kD];
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, c = lane & 31;
  const int64_t rs = 3LL * H * kD;
  const uint16_t* base = qkv + static_cast<int64_t>(b) * S * rs + h * kD;
  const int q0 = w * 32;
  // Q^T as the B operand: lane holds Q[q0 + c][16 s + 8 hl + e] -- loaded before the K / V staging
  // so its latency overlaps theirs
  bf16x8_t qf[4];
  const int qr = min(q0 + c, S - 1);
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const bf16x8_t*>(base + qr * rs + 16 * s + 8 * hl);
  {
    uint16_t* const tt[2] = {Ks, Vs};
    const uint16_t* const ss[2] = {base + H * kD, base + 2 * H * kD};
    const int64_t rr[2] = {rs, rs};
    stage64n<2>(tt, ss, rr, S);
  }
  __syncthreads();
  if (q0 >= S) return;  // no barrier below
  const int nkb = S >> 5;
  f32x16 st[4];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
    for (int e = 0; e < 16; ++e) st[kb][e] = 0.f;
    if (kb < nkb) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag<64>(Ks, kb * 32 + c, 2 * s + hl), qf[s], st[kb], 0, 0, 0);
      }
    }
  }
  // softmax over keys of query column c (scale folded into the exponent)
  float m = -3.0e38f;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
    if (kb < nkb)
#pragma unroll
      for (int e = 0; e < 16; ++e) m = fmaxf(m, st[kb][e]);
  {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
    m = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
  const float k2 = scale * kLog2e;
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float p = kb < nkb ? fast_exp2((st[kb][e] - m) * k2) : 0.f;
      st[kb][e] = p;
      sum += p;
    }
  {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(sum), __float_as_uint(sum), false, false);
    sum = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const float inv = 1.f / sum;
  const int q = q0 + c;
  if (hl == 0) lse[static_cast<int64_t>(bh) * S + q] = m * scale + __logf(sum);
  const uint32_t rowbase = (static_cast<uint32_t>(bh) * S + q) * S;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      float p0 = st[kb][e] * inv, p1 = st[kb][e + 1] * inv;
      if constexpr (DROP) {  // keys key, key + 1 (key even): one hash
        const int key = kb * 32 + (e & 3) + 8 * (e >> 2) + 4 * hl;
        const uint32_t hh = pair_hash(seed, (rowbase + key) >> 1);
        p0 = keep_lo(hh, thr) ? p0 * rkeep : 0.f;
        p1 = keep_hi(hh, thr) ? p1 * rkeep : 0.f;
      }
      st[kb][e] = p0;
      st[kb][e + 1] = p1;
    }
  // O^T[d][q] = sum_key V^T[d][key] P^T[key][q]
  f32x16 o[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[db][e] = 0.f;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    if (s < 2 * nkb) {
      const bf16x8_t pb = p_operand(st[s >> 1], s, hl);
#pragma unroll
      for (int db = 0; db < 2; ++db)
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tfrag<64>(Vs, s, db * 32, lane), pb, o[db], 0, 0, 0);
    }
  }
  // lane column q, rows d = db*32 + (e & 3) + 8 (e >> 2) + 4 hl: 4 consecutive d per 8-B store
  uint16_t* orow = out + (static_cast<int64_t>(b) * S + q) * H * kD + h * kD;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const u16x4 v = {f32_to_bf16(o[db][4 * g]), f32_to_bf16(o[db][4 * g + 1]), f32_to_bf16(o[db][4 * g + 2]),
                       f32_to_bf16(o[db][4 * g + 3])};
      *reinterpret_cast<u16x4*>(orow + db * 32 + 8 * g + 4 * hl) = v;
    }
}

// ------------------------------------------------------------------------------ backward
template <bool DROP>
__global__ __launch_bounds__(256) void attn_bwd_kernel(const uint16_t* __restrict__ qkv, const uint16_t* __restrict__ o,
                                                       const uint16_t* __restrict__ dout, const float* __restrict__ lse,
                                                       uint16_t* __restrict__ dqkv, int S, int H, float scale,
                                                       uint64_t seed, uint32_t thr, float rkeep) {
  __shared__ __attribute__((aligned(16))) uint16_t Qs[kS * kD];
  __shared__ __attribute__((aligned(16))) uint16_t Ks[kS * kD];
  __shared__ __attribute__((aligned(16))) uint16_t dOs[kS * kD];
  __shared__ __attribute__((aligned(16))) uint16_t T[kS * kS];  // [query][key]: P_drop, then dS
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, c = lane & 31;
  const int64_t rs = 3LL * H * kD, ors = static_cast<int64_t>(H) * kD;
  const uint16_t* base = qkv + static_cast<int64_t>(b) * S * rs + h * kD;
  const uint16_t* obase = o + static_cast<int64_t>(b) * S * ors + h * kD;
  const uint16_t* dobase = dout + static_cast<int64_t>(b) * S * ors + h * kD;
  uint16_t* gbase = dqkv + static_cast<int64_t>(b) * S * rs + h * kD;
  const int q0 = w * 32, q = q0 + c;
  const bool act = q0 < S;  // wave-uniform
  // this lane's O / dO row halves and the row's log-sum-exp, loaded before the staging so their
  // latency overlaps it (Dq = rowsum(dO * O) is formed after the barrier)
  const int qq = min(q, S - 1);
  u16x8 orow[4], drow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    orow[j] = *reinterpret_cast<const u16x8*>(obase + static_cast<int64_t>(qq) * ors + 32 * hl + 8 * j);
    drow[j] = *reinterpret_cast<const u16x8*>(dobase + static_cast<int64_t>(qq) * ors + 32 * hl + 8 * j);
  }
  const float lse_q = lse[static_cast<int64_t>(bh) * S + qq];
  {
    uint16_t* const tt[3] = {Qs, Ks, dOs};
    const uint16_t* const ss[3] = {base, base + H * kD, dobase};
    const int64_t rr[3] = {rs, rs, ors};
    stage64n<3>(tt, ss, rr, S);
  }
  __syncthreads();
  const int nkb = S >> 5;
  float dd = 0.f;  // formed right away: the row registers die before the MFMA accumulators live
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) dd += bf16_to_f32(orow[j][e]) * bf16_to_f32(drow[j][e]);
  dd += __shfl_xor(dd, 32, 64);
  f32x16 pt[4], ds[4];
  if (act) {
    // S^T = K Q^T and dP^T = V dO^T for this wave's 32 queries
    bf16x8_t qf[4], of[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = frag<64>(Qs, q, 2 * s + hl);
      of[s] = frag<64>(dOs, q, 2 * s + hl);
    }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
      for (int e = 0; e < 16; ++e) pt[kb][e] = ds[kb][e] = 0.f;
      if (kb < nkb) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          pt[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag<64>(Ks, kb * 32 + c, 2 * s + hl), qf[s], pt[kb], 0, 0, 0);
          const bf16x8_t vf =
              *reinterpret_cast<const bf16x8_t*>(base + 2 * H * kD + (kb * 32 + c) * rs + 16 * s + 8 * hl);
          ds[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, of[s], ds[kb], 0, 0, 0);
        }
      }
    }
    // Dq = rowsum(dO * O) for query q: this lane's half of the 64 d, then the other half
    const float l2 = lse_q * kLog2e, k2 = scale * kLog2e;
    const uint32_t rowbase = (static_cast<uint32_t>(bh) * S + q) * S;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        uint32_t hh = 0;
        if constexpr (DROP) {  // keys key, key + 1 (key even): one hash
          const int key = kb * 32 + (e & 3) + 8 * (e >> 2) + 4 * hl;
          hh = pair_hash(seed, (rowbase + key) >> 1);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const float p = kb < nkb ? fast_exp2(pt[kb][e + u] * k2 - l2) : 0.f;
          float dp = ds[kb][e + u];
          float pd = p;
          if constexpr (DROP) {
            const bool kp = u ? keep_hi(hh, thr) : keep_lo(hh, thr);
            pd = kp ? p * rkeep : 0.f;
            dp = kp ? dp * rkeep : 0.f;
          }
          ds[kb][e + u] = p * (dp - dd);
          pt[kb][e + u] = pd;
        }
      }
  }
  // P_drop -> T[q][key]: a lane's 4 consecutive keys of its query row per 8-B store (rows of idle
  // waves' queries are zero)
  auto put = [&](const f32x16 (&v)[4]) {
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const u16x4 x = act ? u16x4{f32_to_bf16(v[kb][4 * g]), f32_to_bf16(v[kb][4 * g + 1]),
                                    f32_to_bf16(v[kb][4 * g + 2]), f32_to_bf16(v[kb][4 * g + 3])}
                            : u16x4{0, 0, 0, 0};
        *reinterpret_cast<u16x4*>(T + off<128>(q, kb * 32 + 8 * g + 4 * hl)) = x;
      }
  };
  put(pt);
  __syncthreads();
  const int k0 = w * 32;
  const bool kact = k0 < S;
  const int nqs = S >> 4;  // 16-query steps
  uint16_t* krow = gbase + static_cast<int64_t>(k0 + c) * rs;
  auto store_t = [&](const f32x16 (&acc)[2], uint16_t* row, float mul) {
    // acc^T layout: lane column = key (or query) row of the output, rows d: 8-B pieces
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const u16x4 v = {f32_to_bf16(acc[db][4 * g] * mul), f32_to_bf16(acc[db][4 * g + 1] * mul),
                         f32_to_bf16(acc[db][4 * g + 2] * mul), f32_to_bf16(acc[db][4 * g + 3] * mul)};
        *reinterpret_cast<u16x4*>(row + db * 32 + 8 * g + 4 * hl) = v;
      }
  };
  f32x16 acc[2];
  if (kact) {
    // dV^T[d][key] = sum_q dO^T[d][q] P_drop[q][key]
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[db][e] = 0.f;
    for (int s = 0; s < nqs; ++s) {
      const bf16x8_t pb = tfrag<128>(T, s, k0, lane);  // P_drop[16 s + 8 hl + j][k0 + c]
#pragma unroll
      for (int db = 0; db < 2; ++db)
        acc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tfrag<64>(dOs, s, db * 32, lane), pb, acc[db], 0, 0, 0);
    }
    store_t(acc, krow + 2 * H * kD, 1.f);
  }
  __syncthreads();  // P_drop read out
  put(ds);
  __syncthreads();
  if (kact) {
    // dK^T[d][key] = scale sum_q Q^T[d][q] dS[q][key]
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[db][e] = 0.f;
    for (int s = 0; s < nqs; ++s) {
      const bf16x8_t sb = tfrag<128>(T, s, k0, lane);  // dS[16 s + 8 hl + j][k0 + c]
#pragma unroll
      for (int db = 0; db < 2; ++db)
        acc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tfrag<64>(Qs, s, db * 32, lane), sb, acc[db], 0, 0, 0);
    }
    store_t(acc, krow + H * kD, scale);
  }
  if (act) {
    // dQ^T[d][q] = scale sum_key K^T[d][key] dS^T[key][q]
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[db][e] = 0.f;
    for (int s = 0; s < 2 * nkb; ++s) {
      const bf16x8_t sb = frag<128>(T, q0 + c, 2 * s + hl);  // dS[q0 + c][16 s + 8 hl + j]
#pragma unroll
      for (int db = 0; db < 2; ++db)
        acc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tfrag<64>(Ks, s, db * 32, lane), sb, acc[db], 0, 0, 0);
    }
    store_t(acc, gbase + static_cast<int64_t>(q) * rs, scale);
  }
}

// keep mask of the attention dropout (tests / debugging): mask[bh][i][j] = 1 if kept
__global__ void attn_dropout_mask_kernel(uint8_t* __restrict__ mask, int64_t n, uint64_t seed, uint32_t thr) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint32_t e = static_cast<uint32_t>(i), hh = pair_hash(seed, e >> 1);
    mask[i] = ((e & 1) ? keep_hi(hh, thr) : keep_lo(hh, thr)) ? 1 : 0;
  }
}

}  // namespace

void launch_attn_fwd(const uint16_t* qkv, uint16_t* out, float* lse, int B, int S, int H, float scale, float p,
                     uint64_t seed, hipStream_t s) {
  const uint32_t thr = static_cast<uint32_t>(static_cast<double>(p) * 65536.0 + 0.5);
  const float rkeep = thr > 0 ? static_cast<float>(65536.0 / (65536.0 - thr)) : 1.f;  // 1 / (1 - p_eff)
  const dim3 grid(B * H);
  if (p > 0.f) hipLaunchKernelGGL(attn_fwd_kernel<true>, grid, dim3(256), 0, s, qkv, out, lse, S, H, scale, seed, thr, rkeep);
  else hipLaunchKernelGGL(attn_fwd_kernel<false>, grid, dim3(256), 0, s, qkv, out, lse, S, H, scale, seed, thr, rkeep);
}

void launch_attn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse, uint16_t* dqkv,
                     int B, int S, int H, float scale, float p, uint64_t seed, hipStream_t s) {
  const uint32_t thr = static_cast<uint32_t>(static_cast<double>(p) * 65536.0 + 0.5);
  const float rkeep = thr > 0 ? static_cast<float>(65536.0 / (65536.0 - thr)) : 1.f;  // 1 / (1 - p_eff)
  const dim3 grid(B * H);
  if (p > 0.f)
    hipLaunchKernelGGL(attn_bwd_kernel<true>, grid, dim3(256), 0, s, qkv, out, dout, lse, dqkv, S, H, scale, seed, thr,
                       rkeep);
  else
    hipLaunchKernelGGL(attn_bwd_kernel<false>, grid, dim3(256), 0, s, qkv, out, dout, lse, dqkv, S, H, scale, seed,
                       thr, rkeep);
}

void launch_attn_dropout_mask(uint8_t* mask, int64_t n, float p, uint64_t seed, hipStream_t s) {
  const uint32_t thr = static_cast<uint32_t>(static_cast<double>(p) * 65536.0 + 0.5);
  hipLaunchKernelGGL(attn_dropout_mask_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, mask, n,
                     seed, thr);
}

}  // namespace psamd
