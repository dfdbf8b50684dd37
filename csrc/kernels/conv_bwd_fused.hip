// Fused backward of the ResNet bottleneck's last 1x1 convolution (conv3: CI -> CO channels,
// stride 1) with bn3's backward in its prologue -- ONE pass over the layer's widest tensors.
//
// Reference hot op: layer/Conv2DLayer.java:146-240 (a conv layer's backward = data gradient +
// weight gradient of the same output gradient).  The unfused chain (ops/convgemm.py) ran
//   dz3 = bf16(ca * g + cb * z3 + cc)          (bn3 backward: a two-source prologue that STORES dz3)
//   gy2 = mask(dz3 W3) + bn2 backward sums     (conv3 data gradient, epilogue 3)
//   dW3 = dz3^T relu(bn2(z2))                  (a second kernel: re-reads dz3 and z2)
// i.e. dz3 went to HBM and back ([M, CO] bf16 written + read) and z2 was read twice.  Here a
// persistent block per CU builds dz3 in LDS one 64-channel stage at a time and feeds BOTH GEMMs
// from that stage tile:
//   data gradient   acc_dg[c][px] += W3t[c][n] dz3[px][n]      (A = the resident weight, B = dz3)
//   weight gradient accW[n][c]    += dz3[px][n] a2[px][c]       (A = dz3 read transposed, B = a2)
// where a2 = relu(bf16(z2 sc2 + sh2)) is recomputed once per tile from the z2 tile in LDS (the
// same tile gives the epilogue its ReLU mask and x-hat), the per-block dW accumulates in
// registers over every tile of the block and leaves as ONE fp32 slab (fixed-order reduce), and
// bn2's partial sums leave as [2][blocks][CI] like conv_gemm's epilogue 3.
//
// Streams per 128-pixel tile: g and z3 (2 x 128 x CO bf16) through a 3-slot LDS-DMA ring of
// stage tiles (g lands by DMA, z3 by register loads one stage ahead, the BN-backward pass writes
// dz3 over g in place), the z2 tile (double-buffered, issued one tile ahead), the gy rows out.
// The layer is HBM-bound (MFMA ~15 % busy at CI = 64): the design goal is bytes, not FLOPs --
// per layer-1 block 4.0 GB instead of 5.6 GB (dgrad) + 2.0 GB (wgrad).
//
// LDS layout of a [128 px][64 ch] bf16 tile: 128-B rows, 16-B chunk c of row r at physical chunk
// c ^ f((r >> 1) & 7) with f(y) = y ^ ((y & 1) << 2): the row reads of the B operand
// (ds_read_b128, 16 rows x one chunk per lane group) and the transposed reads of the A operand
// (ds_read_b64_tr_b16: 4 rows x 4 chunks per half-wave) are both conflict-free.  The resident
// transposed weight [CI][CO] keeps 2*CO-byte rows with chunk c at c ^ (row & 15).
#include <algorithm>
#include <cstdlib>

#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8i __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(1))) const void gptr_t;
typedef __attribute__((address_space(3))) void lptr_t;
typedef __attribute__((address_space(3))) const char lds_char;

__device__ __attribute__((aligned(16))) uint16_t kZeroRow[8] = {0, 0, 0, 0, 0, 0, 0, 0};

constexpr int kTM = 128;             // pixels per tile
constexpr int kKS = 64;              // bn3 channels per stage
constexpr int kNW = 8;               // waves per block
constexpr int kSlot = kTM * kKS * 2;  // bytes of a [128][64] bf16 tile

__device__ __forceinline__ int swf(int r) {
  const int y = (r >> 1) & 7;
  return y ^ ((y & 1) << 2);
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_char*)p));
}

// LDS reads as inline asm: the compiler would otherwise order every LDS read behind the LDS-DMA
// loads in flight to the other ring slots (s_waitcnt vmcnt(0)), collapsing the prefetch.  Callers
// wait lgkmcnt themselves and tie the results (tie()) so no use is scheduled above the wait.
__device__ __forceinline__ bf16x8_t ld_b128(uint32_t a) {
  bf16x8_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ f32x4 ld_f4(uint32_t a) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ s16x4 ld_b64(uint32_t a) {
  s16x4 v;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ s16x4 ld_tr(uint32_t a) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ void st_b128(uint32_t a, bf16x8_t v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <typename T>
__device__ __forceinline__ void tie(T& v) {
  asm volatile("" : "+v"(v));
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// LDS hand-off barrier: this wave's LDS traffic only (the DMA ring stays in flight)
__device__ __forceinline__ void lds_bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ bf16x8_t cat8(s16x4 lo, s16x4 hi) {
  return __builtin_bit_cast(bf16x8_t, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
}

// PLAIN: the same pass for the block's DOWNSAMPLE branch (1x1, stride 1, CI -> CO): g / z3 are the
// block-output gradient and the downsample BN's input, z2 is the block input itself (the weight
// gradient's operand as is: no BN / ReLU), and the data gradient leaves unmasked with no sums --
// it is the residual-branch term the consumer's conv1 data-gradient epilogue adds.
//
// Persistent grid of one 8-wave block per CU (LDS: resident weight + 3 stage slots + 2 z2 slots).
// Waves: data gradient 4 pixel blocks x 2 channel blocks of 32 x 32 (pb = wave & 3, cb = wave >> 2);
// weight gradient 2 n blocks x 2 c blocks x 2 pixel halves (nb = wave & 1, cw = (wave >> 1) & 1,
// kh = wave >> 2) -- the two halves of a dW block are summed in fixed order at the end.
template <int CI, int CO, bool PLAIN>
__global__ __launch_bounds__(512, 1) void conv11_bwd_fused_kernel(const Conv11BwdArgs p) {
  static_assert(CI == 64 && CO == 256, "the layer-1 conv3 shape (64 -> 256): 4 stages per tile");
  constexpr int NS = CO / kKS;        // stages per tile
  constexpr int NR = 5, PD = NR - 1;  // ring slots; stage q + PD is issued during stage q
  constexpr int WROW = CO * 2;        // bytes per weight row
  constexpr int W_BYTES = CI * WROW;  // resident W3t
  constexpr int RING = W_BYTES;
  constexpr int Z2 = RING + NR * kSlot;
  constexpr int PAR = Z2 + 2 * kSlot;
  constexpr int NPAR = 3 * CO + 4 * CI;  // ca | cb | cc | sc2 | sh2 | mean2 | invstd2
  constexpr int LDS_BYTES = PAR + NPAR * 4;
  static_assert(LDS_BYTES <= 163840, "LDS budget");
  static_assert(4 * NS * 16 * 64 * 4 <= (NR + 2) * kSlot, "dW half-sum scratch fits the ring + z2 slots");
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  float* const par = reinterpret_cast<float*>(lds + PAR);
  const uint32_t L0 = lds_addr(lds);

  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int fr = lane & 31, fh = lane >> 5;
  const int GM = gridDim.x, mg = blockIdx.x;
  const int ntiles = (p.M + kTM - 1) / kTM;
  const int my_tiles = mg < ntiles ? (ntiles - mg + GM - 1) / GM : 0;  // block-uniform
  const int nq = my_tiles * NS;
  auto stage_m0 = [&](int q) { return q < nq ? (mg + (q / NS) * GM) * kTM : p.M; };

  // ---- prologue: parameters, resident weight, z2 of tile 0, stages 0 and 1, z3 of stage 0
  for (int i = t; i < NPAR; i += kNW * 64) {
    float v;
    if (i < 3 * CO) v = p.cbwd[i];
    else if (PLAIN) v = 0.f;
    else if (i < 3 * CO + 2 * CI) v = p.cf2[i - 3 * CO];
    else if (i < 3 * CO + 3 * CI) v = p.mean2[i - 3 * CO - 2 * CI];
    else v = p.invstd2[i - 3 * CO - 3 * CI];
    par[i] = v;
  }
  {
    constexpr int CPR = CO / 8, RPP = 64 / CPR, PPW = W_BYTES / 1024 / kNW;
    const int lr = lane / CPR, lp = lane % CPR;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int k = wave * PPW + i, r = k * RPP + lr;
      __builtin_amdgcn_global_load_lds((gptr_t*)(p.wt + static_cast<int64_t>(r) * CO + (lp ^ (r & 15)) * 8),
                                       (lptr_t*)(lds + k * 1024), 16, 0, 0);
    }
  }
  // a [128][64] tile of rows m0.. (columns col0.. of a row-major [*, stride] matrix) into LDS at
  // byte offset dst: 16 pieces of 8 rows, 2 per wave; rows past M load the zero row.  ALWAYS two
  // DMA instructions per wave (the ring's counted waits rely on it)
  auto issue_tile = [&](const uint16_t* base, int stride, int col0, int m0, int dst) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = wave * 2 + i, r = 8 * k + (lane >> 3), m = m0 + r;
      const int lc = (lane & 7) ^ swf(r);
      const uint16_t* src = m < p.M ? base + static_cast<int64_t>(m) * stride + col0 + lc * 8 : kZeroRow;
      __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(lds + dst + k * 1024), 16, 0, 0);
    }
  };
  // z3 of a stage into registers: thread t owns logical chunk t & 7 of rows (t >> 3) + 64 i
  const int zr = t >> 3, zc = t & 7;
  // two register sets by stage parity: z3 of stage q + 2 is loaded while stage q + 1's waits
  u16x8 z3r[2][2];
  auto load_z3 = [&](int q, u16x8 (&dst)[2]) {
    const int m0 = stage_m0(q), col = (q % NS) * kKS + zc * 8;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = m0 + zr + 64 * i;
      dst[i] = m < p.M ? *reinterpret_cast<const u16x8*>(p.z3 + static_cast<int64_t>(m) * CO + col)
                       : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  issue_tile(p.z2, CI, 0, stage_m0(0), Z2);
#pragma unroll
  for (int i = 0; i < PD; ++i) issue_tile(p.g, CO, (i % NS) * kKS, stage_m0(i), RING + i * kSlot);
  load_z3(0, z3r[0]);
  load_z3(1, z3r[1]);
  wait_vm<0>();
  lds_bar();

  // ---- per-lane constants
  const int pb = wave & 3, cbd = wave >> 2;                  // data gradient block
  const int nb = wave & 1, cw = (wave >> 1) & 1, khw = wave >> 2;  // weight gradient block
  const int dpx = 32 * pb + fr, dsw = swf(dpx);
  const uint32_t wrow = L0 + static_cast<uint32_t>((32 * cbd + fr) * WROW);
  // transposed reads (ds_read_b64_tr_b16): lane reads row 16 s + trow (+ 4), columns c0 + tcol..+3
  const int gi = lane >> 4, i16 = lane & 15;
  const int trow = 8 * (gi >> 1) + (i16 >> 2), tcol = 16 * (gi & 1) + 4 * (i16 & 3);
  auto tr_off = [&](int c0, int h) {
    const int r = trow + 4 * h;  // (r >> 1) & 7 is the same for every 16-row group s
    return static_cast<uint32_t>(r * 128 + ((((c0 + tcol) >> 3) ^ swf(r)) << 4) + (tcol & 7) * 2);
  };
  const uint32_t tD0 = tr_off(32 * nb, 0), tD1 = tr_off(32 * nb, 1);
  const uint32_t tZ0 = tr_off(32 * cw, 0), tZ1 = tr_off(32 * cw, 1);
  const float asc = par[3 * CO + 32 * cw + fr], ash = par[3 * CO + CI + 32 * cw + fr];

  f32x16 acc_dg, accW[NS];
  auto zero16 = [](f32x16& a) {
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = 0.f;
  };
  zero16(acc_dg);
#pragma unroll
  for (int s = 0; s < NS; ++s) zero16(accW[s]);
  // data-gradient lane: ONE channel (c = 32 cb + fr) over 16 pixels per tile -> two running sums
  // and its four epilogue coefficients in registers
  const int ec = 32 * cbd + fr;
  const float emc = par[3 * CO + ec], esh = par[3 * CO + CI + ec], emu = par[3 * CO + 2 * CI + ec],
              eis = par[3 * CO + 3 * CI + ec];
  float s1 = 0.f, s2 = 0.f;

  // a2 = relu(bf16(z2 sc + sh)) fragments of this tile (B operand of the weight gradient): lane's
  // channel is fixed (32 cw + fr), its 8 values are 8 consecutive pixels
  bf16x8_t a2f[4];
  auto make_a2 = [&](int ti) {
    const uint32_t zs = L0 + Z2 + (ti & 1) * kSlot + khw * (4 * 2048);
    s16x4 lo[4], hi[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      lo[ks] = ld_tr(zs + ks * 2048 + tZ0);
      hi[ks] = ld_tr(zs + ks * 2048 + tZ1);
    }
    lgkm0();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      tie(lo[ks]);
      tie(hi[ks]);
      if constexpr (PLAIN) {
        a2f[ks] = cat8(lo[ks], hi[ks]);
        continue;
      }
      u16x8 v = __builtin_bit_cast(u16x8, cat8(lo[ks], hi[ks]));
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = f32_to_bf16(bf16_to_f32(v[j]) * asc + ash);
      const s16x8i z = {0, 0, 0, 0, 0, 0, 0, 0};
      a2f[ks] = __builtin_bit_cast(bf16x8_t, __builtin_elementwise_max(__builtin_bit_cast(s16x8i, v), z));
    }
  };
  // bn3 backward over stage slot `sl` in place: dz3 = bf16(ca g + cb z3 + cc); rows past M -> 0
  auto transform = [&](int sl, int s, int m0, const u16x8 (&z3v)[2]) {
    const uint32_t ds = L0 + RING + sl * kSlot;
    const uint32_t pa = L0 + PAR + (s * kKS + zc * 8) * 4;
    const f32x4 ca0 = ld_f4(pa), ca1 = ld_f4(pa + 16);
    const f32x4 cb0 = ld_f4(pa + CO * 4), cb1 = ld_f4(pa + CO * 4 + 16);
    const f32x4 cc0 = ld_f4(pa + 2 * CO * 4), cc1 = ld_f4(pa + 2 * CO * 4 + 16);
    bf16x8_t gv[2];
    uint32_t ga[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = zr + 64 * i;
      ga[i] = ds + r * 128 + ((zc ^ swf(r)) << 4);
      gv[i] = ld_b128(ga[i]);
    }
    lgkm0();
    f32x4 c0a = ca0, c0b = ca1, c1a = cb0, c1b = cb1, c2a = cc0, c2b = cc1;
    tie(c0a); tie(c0b); tie(c1a); tie(c1b); tie(c2a); tie(c2b);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      tie(gv[i]);
      const u16x8 g8 = __builtin_bit_cast(u16x8, gv[i]);
      const u16x8 z8 = z3v[i];
      u16x8 d;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = j < 4 ? c0a[j] : c0b[j - 4], b = j < 4 ? c1a[j] : c1b[j - 4], c = j < 4 ? c2a[j] : c2b[j - 4];
        d[j] = f32_to_bf16(a * bf16_to_f32(g8[j]) + b * bf16_to_f32(z8[j]) + c);
      }
      if (m0 + zr + 64 * i >= p.M) d = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      st_b128(ga[i], __builtin_bit_cast(bf16x8_t, d));
    }
  };
  // both GEMMs of one stage from slot `sl`, in two halves of two k-steps (register budget)
  auto compute = [&](int sl, f32x16& aw, int s) {
    const uint32_t ds = L0 + RING + sl * kSlot;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8_t wa[2], xb[2];
      s16x4 dlo[2], dhi[2];
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        const int ks = 2 * h + k2;
        wa[k2] = ld_b128(wrow + ((((8 * s + 2 * ks + fh) ^ (fr & 15))) << 4));
        xb[k2] = ld_b128(ds + dpx * 128 + (((2 * ks + fh) ^ dsw) << 4));
        dlo[k2] = ld_tr(ds + (4 * khw + ks) * 2048 + tD0);
        dhi[k2] = ld_tr(ds + (4 * khw + ks) * 2048 + tD1);
      }
      lgkm0();
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        tie(wa[k2]);
        tie(xb[k2]);
        tie(dlo[k2]);
        tie(dhi[k2]);
      }
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
        acc_dg = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xb[k2], wa[k2], acc_dg, 0, 0, 0);
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
        aw = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cat8(dlo[k2], dhi[k2]), a2f[2 * h + k2], aw, 0, 0, 0);
    }
  };
  // data-gradient epilogue of tile ti (the conv_gemm epi-3 arithmetic): bn2's ReLU mask from z2,
  // the backward sums sum(g), sum(g (z2 - mean) invstd), masked gy out.  Register q of the lane is
  // pixel 32 pb + 8 (q >> 2) + 4 fh + (q & 3) of channel ec; its four z2 values per q >> 2 come from
  // ONE transposed read (each 16-lane group reads the 4 x 16 block of its rows / channels)
  auto epilogue = [&](int ti) {
    const int m0 = (mg + ti * GM) * kTM;
    if constexpr (PLAIN) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + 32 * pb + 8 * (q >> 2) + 4 * fh + (q & 3);
        if (m < p.M) p.gy[static_cast<int64_t>(m) * CI + ec] = f32_to_bf16(acc_dg[q]);
      }
      zero16(acc_dg);
      return;
    }
    const uint32_t zs = L0 + Z2 + (ti & 1) * kSlot;
    s16x4 zv[4];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const int r = 32 * pb + 8 * q4 + 4 * (gi >> 1) + (i16 >> 2);
      const int col = 32 * cbd + 16 * (gi & 1) + 4 * (i16 & 3);
      zv[q4] = ld_tr(zs + r * 128 + (((col >> 3) ^ swf(r)) << 4) + (col & 7) * 2);
    }
    lgkm0();
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      tie(zv[q4]);
      const u16x4 z4 = __builtin_bit_cast(u16x4, zv[q4]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint16_t val = f32_to_bf16(acc_dg[4 * q4 + e]);
        const float z = bf16_to_f32(z4[e]);
        const bool on = z * emc + esh > 0.f;
        const float gv = on ? bf16_to_f32(val) : 0.f;
        s1 += gv;
        s2 += gv * ((z - emu) * eis);
        const int m = m0 + 32 * pb + 8 * q4 + 4 * fh + e;
        if (m < p.M) p.gy[static_cast<int64_t>(m) * CI + ec] = on ? val : static_cast<uint16_t>(0);
      }
    }
    zero16(acc_dg);
  };

  // ---- main loop: stage q of tile ti in ring slot q % NR; G(q + PD) and z3(q + 2) are issued
  // during stage q (and z2 of tile ti + 1 during its stage 0), every issue unconditional (zero
  // rows past the block's work) so the counted waits hold
  int sl = 0, q = 0;
  for (int ti = 0; ti < my_tiles; ++ti) {
    const int m0 = (mg + ti * GM) * kTM;
#pragma unroll
    for (int s = 0; s < NS; ++s, ++q) {
      if (s == 0) make_a2(ti);
      transform(sl, s, m0, z3r[s & 1]);
      lds_bar();  // dz3 of stage q complete in slot sl; stage q - 1's slot is free
      const int slp = sl == 0 ? NR - 1 : sl - 1;  // (q + PD) % NR = (q - 1) % NR
      issue_tile(p.g, CO, ((q + PD) % NS) * kKS, stage_m0(q + PD), RING + slp * kSlot);
      load_z3(q + 2, z3r[s & 1]);
      if (s == 0) issue_tile(p.z2, CI, 0, ti + 1 < my_tiles ? m0 + GM * kTM : p.M, Z2 + ((ti + 1) & 1) * kSlot);
      compute(sl, accW[s], s);
      if (s == NS - 1) epilogue(ti);
      // G(q + 1) (issued during stage q - 3) landed: younger than it are the G DMAs of stages
      // q - 2 .. q (6) and the z2 tile issued in stage q - 3 .. q (2): vmcnt(8).  At a tile's last
      // stage the z2 tile of the next one (issued at its stage 0) must have landed too: vmcnt(6)
      if (s == NS - 1) wait_vm<6>();
      else wait_vm<8>();
      lds_bar();
      sl = sl == NR - 1 ? 0 : sl + 1;
    }
  }
  wait_vm<0>();  // no DMA may land in LDS after the block (or into the scratch below)
  lds_bar();

  // ---- bn2 partial sums: lanes l and l + 32 (pixel halves), then the 4 pixel-block waves in
  // fixed order
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 32, 64);
  float* red = reinterpret_cast<float*>(lds + RING);  // [2][4 pb][CI]
  if (!PLAIN && fh == 0) {
    red[pb * CI + ec] = s1;
    red[(4 + pb) * CI + ec] = s2;
  }
  __syncthreads();
  if (!PLAIN && t < CI) {
    p.part[static_cast<int64_t>(mg) * CI + t] = (red[t] + red[CI + t]) + (red[2 * CI + t] + red[3 * CI + t]);
    p.part[static_cast<int64_t>(GM + mg) * CI + t] =
        (red[4 * CI + t] + red[5 * CI + t]) + (red[6 * CI + t] + red[7 * CI + t]);
  }
  __syncthreads();
  // ---- dW slab: pixel half 1 (waves 4..7) hands its accumulators to its half-0 partner
  float* wsc = reinterpret_cast<float*>(lds + RING);
  if (khw == 1) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int i = 0; i < 16; ++i) wsc[(((wave - 4) * NS + s) * 16 + i) * 64 + lane] = accW[s][i];
  }
  __syncthreads();
  if (khw == 0) {
    float* slab = p.ws + static_cast<int64_t>(mg) * CO * CI;
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int n = s * kKS + 32 * nb + 8 * (i >> 2) + 4 * fh + (i & 3);
        slab[n * CI + 32 * cw + fr] = accW[s][i] + wsc[((wave * NS + s) * 16 + i) * 64 + lane];
      }
  }
}

// out[y][e] = sum_{b in [y*per, y*per + per)} in[b][e], fixed order (bf16 or fp32 out)
template <bool BF16>
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ in, int nslab, int per, int64_t E,
                                                       void* __restrict__ out) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= E) return;
  const int b0 = blockIdx.y * per, b1 = min(nslab, b0 + per);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int b = b0;
  for (; b + 3 < b1; b += 4) {
    a0 += in[b * E + e];
    a1 += in[(b + 1) * E + e];
    a2 += in[(b + 2) * E + e];
    a3 += in[(b + 3) * E + e];
  }
  for (; b < b1; ++b) a0 += in[b * E + e];
  const float v = (a0 + a1) + (a2 + a3);
  if constexpr (BF16) static_cast<uint16_t*>(out)[blockIdx.y * E + e] = f32_to_bf16(v);
  else static_cast<float*>(out)[blockIdx.y * E + e] = v;
}

int slab_levels(int nslab) { return nslab > 16 ? (nslab + 15) / 16 : 0; }

}  // namespace

// Layer 1 only (64 -> 256).  A layer-2 variant (128 -> 512, 64-pixel tiles, the weight streamed
// per stage) ran 0.78 ms against the two-kernel chain's 0.76 ms at batch 1024
// (profiles/r5_conv3_bwd_fused_probe_w128.jsonl) and was removed in round 6.
bool conv11_bwd_fused_ok(int CI, int CO) { return CI == 64 && CO == 256; }

bool conv11_bwd_plain_ok(int CI, int CO) { return CI == 64 && CO == 256; }

bool conv11_bwd_built(int CI, int CO) { return CI == 64 && CO == 256; }

int conv11_bwd_blocks(int M, int CI, int CO) {
  (void)CI, (void)CO;
  const int ntiles = (M + kTM - 1) / kTM;
  return std::max(1, std::min(ntiles, 256));  // one block per CU (LDS-bound)
}

int64_t conv11_bwd_ws(int M, int CI, int CO) {
  const int gm = conv11_bwd_blocks(M, CI, CO);
  return static_cast<int64_t>(gm + slab_levels(gm)) * CI * CO;
}

void launch_conv11_bwd_fused(const Conv11BwdArgs& a, int CI, int CO, hipStream_t s) {
  if (a.M <= 0) return;
  const int gm = conv11_bwd_blocks(a.M, CI, CO);
  if (CI == 64 && CO == 256 && a.cf2 == nullptr)
    hipLaunchKernelGGL((conv11_bwd_fused_kernel<64, 256, true>), dim3(gm), dim3(512), 0, s, a);
  else if (CI == 64 && CO == 256) hipLaunchKernelGGL((conv11_bwd_fused_kernel<64, 256, false>), dim3(gm), dim3(512), 0, s, a);
  else if (a.cf2 == nullptr) return;  // PLAIN: the 64 -> 256 kernel only
  else return;
  const int64_t E = static_cast<int64_t>(CI) * CO;
  const unsigned eb = static_cast<unsigned>((E + 255) / 256);
  const int groups = slab_levels(gm);
  if (groups) {
    float* mid = a.ws + static_cast<int64_t>(gm) * E;
    hipLaunchKernelGGL(slab_sum_kernel<false>, dim3(eb, groups), dim3(256), 0, s, a.ws, gm, 16, E,
                       static_cast<void*>(mid));
    hipLaunchKernelGGL(slab_sum_kernel<true>, dim3(eb), dim3(256), 0, s, mid, groups, groups, E,
                       static_cast<void*>(a.dw));
  } else {
    hipLaunchKernelGGL(slab_sum_kernel<true>, dim3(eb), dim3(256), 0, s, a.ws, gm, gm, E, static_cast<void*>(a.dw));
  }
}

}  // namespace psamd
