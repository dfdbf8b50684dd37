// Device-side helpers shared by every ps_amd HIP kernel (gfx950 / CDNA4 only).
//
// Conventions
//  * wave64: every cross-lane idiom here assumes 64 lanes (hard-coded, see
//    cdna_hip_programming.md §1) and a block size that is a multiple of 64.
//  * bf16 is carried as raw uint16_t in memory; conversion to bf16 uses the clang
//    `__bf16` cast which lowers to v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN-safe).
//  * memory-bound kernels move 16 bytes per lane per access (8 x bf16 or 4 x f32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psamd {

constexpr int kWave = 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, b);
}

// two floats -> one dword of two bf16 (RNE): ONE v_cvt_pk_bf16_f32, not two conversions + shift / or
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef float f2v __attribute__((ext_vector_type(2)));
  typedef __bf16 b2v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2v){a, b}, b2v));
}
// Per-element bit masks over 8 x bf16 (bit e of `bits` -> element e), branch-free: an
// `if ((bits >> e) & 1) v[e] = ...` compiles to one exec-mask branch per element (saveexec /
// restore + the arm), which made the data-gradient epilogues issue-bound.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
// 16-bit lane mask of dword w (elements 2w, 2w + 1): one signed 1-bit extract per half + a bitfield insert
__device__ __forceinline__ uint32_t bf16_pair_mask(unsigned bits, int w) {
  const uint32_t lo = static_cast<uint32_t>(static_cast<int32_t>(bits << (31 - 2 * w)) >> 31);
  const uint32_t hi = static_cast<uint32_t>(static_cast<int32_t>(bits << (30 - 2 * w)) >> 31);
  return (lo & 0xffffu) | (hi & 0xffff0000u);
}
// v[e] + r[e] (one bf16 rounding of the fp32 sum) where bit e is set, v[e] elsewhere
__device__ __forceinline__ u16x8 bf16_add_where(u16x8 v, u16x8 r, unsigned bits) {
  const u32x4_t vw = __builtin_bit_cast(u32x4_t, v), rw = __builtin_bit_cast(u32x4_t, r);
  u32x4_t o;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const float a0 = __uint_as_float(vw[w] << 16), a1 = __uint_as_float(vw[w] & 0xffff0000u);
    const float b0 = __uint_as_float(rw[w] << 16), b1 = __uint_as_float(rw[w] & 0xffff0000u);
    const uint32_t m = bf16_pair_mask(bits, w);
    o[w] = (pk_bf16(a0 + b0, a1 + b1) & m) | (vw[w] & ~m);
  }
  return __builtin_bit_cast(u16x8, o);
}
// v[e] where bit e is set, 0 elsewhere
__device__ __forceinline__ u16x8 bf16_keep_where(u16x8 v, unsigned bits) {
  u32x4_t o = __builtin_bit_cast(u32x4_t, v);
#pragma unroll
  for (int w = 0; w < 4; ++w) o[w] &= bf16_pair_mask(bits, w);
  return __builtin_bit_cast(u16x8, o);
}

// 2^x as the bare v_exp_f32: for softmax arguments (<= 0) a denormal result is as good as 0, so
// exp2f's denormal-range fix-up (compare, select, scale, ldexp per element) is waste there
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Grad / weight element loaders: T is float or uint16_t (bf16 storage).
template <typename T> struct Elem;
template <> struct Elem<float> {
  __device__ __forceinline__ static float load(const float* p, int64_t i) { return p[i]; }
  __device__ __forceinline__ static void store(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct Elem<uint16_t> {
  __device__ __forceinline__ static float load(const uint16_t* p, int64_t i) { return bf16_to_f32(p[i]); }
  __device__ __forceinline__ static void store(uint16_t* p, int64_t i, float v) { p[i] = f32_to_bf16(v); }
};

// Load 8 consecutive elements (16 B of bf16 or 2 x 16 B of f32) into registers.
__device__ __forceinline__ void load8(const float* __restrict__ p, int64_t i, float (&o)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p + i);
  const f32x4 b = *reinterpret_cast<const f32x4*>(p + i + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
__device__ __forceinline__ void load8(const uint16_t* __restrict__ p, int64_t i, float (&o)[8]) {
  const u16x8 v = *reinterpret_cast<const u16x8*>(p + i);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = bf16_to_f32(v[j]);
}
__device__ __forceinline__ void store8(float* __restrict__ p, int64_t i, const float (&o)[8]) {
  *reinterpret_cast<f32x4*>(p + i) = f32x4{o[0], o[1], o[2], o[3]};
  *reinterpret_cast<f32x4*>(p + i + 4) = f32x4{o[4], o[5], o[6], o[7]};
}
__device__ __forceinline__ void store8(uint16_t* __restrict__ p, int64_t i, const float (&o)[8]) {
  u16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f32_to_bf16(o[j]);
  *reinterpret_cast<u16x8*>(p + i) = v;
}

// 4 consecutive elements as f32x4 (16 B of fp32 / 8 B of bf16); p + i must be aligned.
__device__ __forceinline__ f32x4 load4(const float* __restrict__ p, int64_t i) {
  return *reinterpret_cast<const f32x4*>(p + i);
}
__device__ __forceinline__ f32x4 load4(const uint16_t* __restrict__ p, int64_t i) {
  const u16x4 v = *reinterpret_cast<const u16x4*>(p + i);
  return f32x4{bf16_to_f32(v[0]), bf16_to_f32(v[1]), bf16_to_f32(v[2]), bf16_to_f32(v[3])};
}
__device__ __forceinline__ void store4(float* __restrict__ p, int64_t i, f32x4 v) {
  *reinterpret_cast<f32x4*>(p + i) = v;
}
__device__ __forceinline__ void store4(uint16_t* __restrict__ p, int64_t i, f32x4 v) {
  *reinterpret_cast<u16x4*>(p + i) = u16x4{f32_to_bf16(v.x), f32_to_bf16(v.y), f32_to_bf16(v.z), f32_to_bf16(v.w)};
}

// Sum over aligned groups of 2^lg lanes (every lane of the wave must execute this).
__device__ __forceinline__ float group_sum(float v, int lg) {
  for (int off = 1; off < (1 << lg); off <<= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Wave64 sum via DPP-friendly xor shuffles.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

// Block-wide sum; `scratch` must hold blockDim.x/64 floats. Result valid in all threads.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nw = blockDim.x / kWave;
  v = wave_sum(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = (lane < nw) ? scratch[lane] : 0.f;
  r = wave_sum(r);
  __syncthreads();
  return r;
}

// Grid size for grid-stride memory-bound kernels: cap at 256 CUs x 8 blocks.
__host__ inline int stream_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return static_cast<int>(g);
}

// Philox-4x32-10 counter-based RNG (stateless; (seed, counter) -> 4 uniform u32).
struct Philox {
  __device__ __forceinline__ static void round(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    // one 32x32->64 multiply (v_mad_u64_u32) per product instead of separate hi / lo multiplies
    const uint64_t p0 = static_cast<uint64_t>(M0) * c[0], p1 = static_cast<uint64_t>(M1) * c[2];
    const uint32_t hi0 = static_cast<uint32_t>(p0 >> 32), lo0 = static_cast<uint32_t>(p0);
    const uint32_t hi1 = static_cast<uint32_t>(p1 >> 32), lo1 = static_cast<uint32_t>(p1);
    uint32_t n0 = hi1 ^ c[1] ^ k0, n1 = lo1, n2 = hi0 ^ c[3] ^ k1, n3 = lo0;
    c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
  }
  // 128-bit counter: ctr = low 64 bits, ctr_hi = high 64 bits
  __device__ __forceinline__ static void gen(uint64_t seed, uint64_t ctr, uint32_t (&out)[4], uint64_t ctr_hi = 0) {
    uint32_t c[4] = {static_cast<uint32_t>(ctr), static_cast<uint32_t>(ctr >> 32), static_cast<uint32_t>(ctr_hi),
                     static_cast<uint32_t>(ctr_hi >> 32)};
    uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      round(c, k0, k1);
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = c[3];
  }
  // uniform in [0, 1)
  __device__ __forceinline__ static float u01(uint32_t x) { return (x >> 8) * (1.0f / 16777216.0f); }
};

}  // namespace psamd
