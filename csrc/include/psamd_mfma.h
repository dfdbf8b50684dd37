// Shared helpers of the attention kernels (attention.hip, flash_attn.hip): swizzled row-major
// LDS tiles readable both as direct ds_read_b128 MFMA fragments and as transposed
// ds_read_b64_tr_b16 fragments, and the accumulator -> B-operand register relayout.
//
// v_mfma_f32_32x32x16_bf16(a, b, c): lane l provides A[l & 31][8 (l >> 5) + e] and
// B[8 (l >> 5) + e][l & 31] (e = 0..7) and holds C[(q & 3) + 8 (q >> 2) + 4 (l >> 5)][l & 31].
#pragma once
#include "psamd_device.h"

namespace psamd {
namespace mfma {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-B chunk XOR per row.  128-B rows (RL 64): chunk ^ f(row pair), f(p) = ((p & 1) << 2) | (p >> 1)
// on p = (r >> 1) & 7; 256-B rows (RL 128): chunk ^ (((r & 3) << 2) | ((r >> 2) & 3)).  Both keep
// the 16 rows of a direct fragment read and the 4 consecutive rows x 64 B of a transposed read
// on distinct banks.
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
template <int RL>
__device__ __forceinline__ bf16x8_t tfrag(const uint16_t* T, int s, int c0, int lane) {
  const int gi = lane >> 4, i16 = lane & 15;
  const int r = 16 * s + 8 * (gi >> 1) + (i16 >> 2);
  const int col = c0 + 16 * (gi & 1) + 4 * (i16 & 3);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(T + off<RL>(r, col)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(T + off<RL>(r + 4, col)));
  return __builtin_bit_cast(bf16x8_t, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
}

// The same reads as inline asm, for kernels that keep LDS-DMA (global_load_lds) in flight to
// another buffer: the compiler cannot tell such a DMA from these reads and would put
// s_waitcnt vmcnt(0) before every builtin LDS read, serialising the prefetch.  The caller waits
// lgkmcnt itself and ties the results (lds_wait) before using them.
__device__ __forceinline__ unsigned lds_addr(const uint16_t* p) {
  return static_cast<unsigned>(reinterpret_cast<uintptr_t>((const lds_s16x4*)p));
}
template <int RL>
__device__ __forceinline__ bf16x8_t frag_a(const uint16_t* T, int r, int ch) {
  bf16x8_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(T + r * RL + ((ch ^ sw<RL>(r)) << 3))) : "memory");
  return v;
}
template <int RL>
__device__ __forceinline__ bf16x8_t tfrag_a(const uint16_t* T, int s, int c0, int lane) {
  const int gi = lane >> 4, i16 = lane & 15;
  const int r = 16 * s + 8 * (gi >> 1) + (i16 >> 2);
  const int col = c0 + 16 * (gi & 1) + 4 * (i16 & 3);
  s16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(lds_addr(T + off<RL>(r, col))) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(lds_addr(T + off<RL>(r + 4, col))) : "memory");
  return __builtin_bit_cast(bf16x8_t, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
}
__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void tie(bf16x8_t& v) { asm volatile("" : "+v"(v)); }

typedef __attribute__((address_space(1))) const void gptr_t;
typedef __attribute__((address_space(3))) void lptr_t;

// LDS-DMA of a [rows][128] bf16 tile (rows % 4 == 0) from rows of stride rs elements: one wave
// instruction moves 4 rows (64 lanes x 16 B) lane-linearly, so the chunk swizzle is applied to
// the SOURCE chunk (the XOR is an involution).  nw waves split the instructions.
__device__ __forceinline__ void dma_tile128(uint16_t* T, const uint16_t* src, int64_t rs, int rows, int wave, int nw,
                                            int lane) {
  for (int i = wave; i < rows / 4; i += nw) {
    const int lc = i * 64 + lane, r = lc >> 4, pc = lc & 15;
    const uint16_t* g = src + r * rs + ((pc ^ sw<128>(r)) << 3);
    __builtin_amdgcn_global_load_lds((gptr_t*)g, (lptr_t*)(T + i * 512), 16, 0, 0);
  }
}

__device__ __forceinline__ uint32_t pack2(float a, float b) { return pk_bf16(a, b); }

// v_permlane32_swap(x, y): x's upper 32 lanes <-> y's lower 32 lanes (a VALU op: no LDS queue,
// no lgkmcnt wait behind in-flight fragment reads, unlike a ds_bpermute shuffle).
__device__ __forceinline__ float xhalf_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);  // same two addends on both halves
}

// B operand (k = rows 16 (s & 1) + 8 hl + e of a 32-row accumulator block, n = lane column)
// from that block held in the accumulator layout: half hl holds rows (q & 3) + 8 (q >> 2) + 4 hl;
// half 0 needs rows 0..7 of the 16-row step = its own 4 + the partner half's 4, half 1 rows
// 8..15 = the partner's 4 + its own 4.  With x = own rows 0..3 and y = own rows 4..7 packed,
// swap(x, y) leaves {x', y'} = {own x, partner x} on half 0 and {partner y, own y} on half 1:
// exactly the four pairs each half needs, in order, with no per-half select.
__device__ __forceinline__ bf16x8_t acc_to_b(const f32x16& blk, int s, int hl) {
  (void)hl;
  const int qb = 8 * (s & 1);
  const uint32_t lo0 = pack2(blk[qb + 0], blk[qb + 1]), lo1 = pack2(blk[qb + 2], blk[qb + 3]);
  const uint32_t hi0 = pack2(blk[qb + 4], blk[qb + 5]), hi1 = pack2(blk[qb + 6], blk[qb + 7]);
  const auto a = __builtin_amdgcn_permlane32_swap(lo0, hi0, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(lo1, hi1, false, false);
  return __builtin_bit_cast(bf16x8_t, u32x4{a[0], b[0], a[1], b[1]});
}

__device__ __forceinline__ f32x16 mma(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void zero(f32x16& a) {
#pragma unroll
  for (int e = 0; e < 16; ++e) a[e] = 0.f;
}

}  // namespace mfma
}  // namespace psamd
