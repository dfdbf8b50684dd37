// 256 x 256 output tiles for the deep-K 1x1 convolution GEMMs (ResNet-50 layers 3-4: K = 256-2048
// input channels, N = 256-2048 output channels; stride 1 or a stride-2 downsample).
//
// Reference hot op: layer/Conv2DLayer.java:146-240 (the conv forward GEMM) and its data-gradient
// twin.  The general conv_fwd_kernel (convgemm.hip) runs 128 x 128 tiles, two blocks per CU and a
// barrier pair per 64-deep stage: 450-800 TF/s on these shapes, which are MFMA-bound at N >= 512 and
// HBM-bound at N = 256.  Here one 512-thread block per CU owns a 256 x 256 tile:
//   * 8 waves as 2 (pixels) x 4 (channels), each 128 pixels x 64 channels = 4 x 2 blocks of
//     v_mfma_f32_32x32x16_bf16 (6 fragment reads per 8 MFMAs, half the LDS traffic per FLOP of a
//     64 x 64 wave tile);
//   * both operands global -> LDS by LDS-DMA into an NST-deep ring of BK-deep stages (128 KiB in
//     total: BK = 64 x 2 stages or BK = 32 x 4), the DMA of stage kt + NST - 1 issued right after
//     the ONE barrier of stage kt and waited for by a counted vmcnt, so NST - 1 stages stay in
//     flight across the barrier (raw s_barrier: __syncthreads() would drain them);
//   * fragment reads as inline asm, the next k-step's issued before this one's MFMAs;
//   * the epilogue (plain store, BN statistics, the data-gradient ReLU mask + BN-backward sums,
//     or the conv1 data gradients' residual / fold epilogues -- every conv_gemm epilogue 0-9) from
//     a bf16 output tile in LDS, one 16-B column group per thread, rows coalesced.
// Blocks are XCD-remapped so the channel tiles of one pixel tile share its A rows in one L2.
// What bounds it (profiles/r5_conv_big_kloop.txt): the K loop runs at the memory system's stage
// rate (~64 KiB per 1.8 us per CU).  Variants measured and removed (round 6): 256 x 128 tiles two
// per CU, 4 waves of 128 x 128, a 4 x 32-deep ring, stream-K with fixed-order partials, a per-tile
// K-order rotation -- none faster on the ResNet-50 shapes (profiles/r5_conv_big_kloop.txt,
// r5_conv_big_stream_k.txt).
#include <algorithm>

#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(1))) const void gptr_t;
typedef __attribute__((address_space(3))) void lptr_t;
typedef __attribute__((address_space(3))) const char lds_char;

__device__ __attribute__((aligned(16))) uint16_t kBigZero[8] = {0, 0, 0, 0, 0, 0, 0, 0};

constexpr int kTM = 256;

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_char*)p));
}
__device__ __forceinline__ bf16x8_t ld_b128(uint32_t a) {
  bf16x8_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
template <int OFF>
__device__ __forceinline__ bf16x8_t ld_b128o(uint32_t a) {
  bf16x8_t v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF) : "memory");
  return v;
}
template <typename T>
__device__ __forceinline__ void tie(T& v) {
  asm volatile("" : "+v"(v));
}
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
// a global 16-B load the compiler does not track: mixed with LDS-DMA in flight, a plain load's use
// makes hipcc wait vmcnt(0) (draining the DMA); callers count vmcnt themselves and tie() the result
__device__ __forceinline__ f32x4 gld_f4(const float* ptr) {
  f32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(ptr) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lds_bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ int xcd_remap_big(int b, int nblk) {
  const int q = nblk >> 3, r = nblk & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}
__device__ __forceinline__ uint32_t fdiv_big(uint32_t n, const FastDiv& f) { return (__umulhi(n, f.mul) + n) >> f.shift; }

// Stage tile rows of 64 bf16 (128 B): chunk c of row r at c ^ ((r >> 1) & 7), so the 16 rows of a
// ds_read_b128 lane group land on 16 distinct 16-B bank slots, and the swizzle of a 32-row
// fragment block depends on fr = r & 31 only.
__device__ __forceinline__ int bswz(int r, int c) { return c ^ ((r >> 1) & 7); }

// PRO (conv_gemm's A prologues, applied by ONE in-place pass over each landed A stage):
//   0 none; 1 relu(bf16(a sc + sh)) (the previous BN + ReLU); 2 the BN backward
//   bf16(ca a + cb a2 + cc) from two row sources, the result also stored to aout (the weight
//   gradient's operand) by the channel-tile-0 blocks; 3 the previous block's output
//   relu(a sc + sh + r), r = a2 or a2 sc2 + sh2, stored to aout with its ReLU bits (abits).
// The second row source a2 lands by LDS-DMA into one extra 32 KiB tile, refilled for stage kt + 1
// once the pass over stage kt has read it.  With a 256-wide channel tile the A rows are staged
// (and transformed) once per channel tile -- once in all for N = 256, and for wider N the other
// channel tiles of the pixel tile run on the same XCD (L2 re-reads, not HBM).
template <int EPI, int PRO>
__global__ __launch_bounds__(512, 1) void conv_big_kernel(const ConvGemmArgs p) {
  static_assert(EPI >= 0 && EPI <= 9, "conv_gemm's epilogues");
  static_assert(PRO != 2 || (EPI != 0 && EPI != 1), "the BN-backward prologue feeds a data-gradient GEMM");

  constexpr int BK = 64, TN = 256, NW = 8, NT = 64 * NW;
  constexpr int WCH = 64;                         // channels per wave (2 waves along the pixels)
  constexpr int WN = TN / WCH, TI = WCH / 32;     // waves along the channels; 32-ch blocks per wave
  constexpr int kRing = 131072;
  constexpr int kTN = TN, kCS = TN + 4;          // output tile row stride (elements)
  constexpr bool TWO = PRO == 2 || PRO == 3;
  constexpr int RB = 2 * BK;                    // bytes per stage row
  constexpr int A_BYTES = kTM * RB, STAGE = (kTM + kTN) * RB;
  constexpr int NST = kRing / STAGE;            // 2
  static_assert(NST >= 2, "ring depth");
  constexpr int CPR = RB / 16;                  // 16-B chunks per row
  constexpr int RPI = 64 / CPR;                 // rows per DMA wave-instruction
  constexpr int PA = kTM / RPI / NW;            // A DMA instructions per wave per stage
  constexpr int PB = kTN / RPI / NW;
  constexpr int GPS = PA + PB;                  // DMA instructions per wave per stage
  constexpr int KSTEPS = BK / 16;
  constexpr int OUT_BYTES = kTM * kCS * 2;
  constexpr int RED_OFF = OUT_BYTES > kRing ? OUT_BYTES : kRing;
  constexpr int Z_OFF = kRing;                                    // TWO: the a2 stage tile
  constexpr int LDS_A = RED_OFF + 3 * NW * kTN * 4, LDS_Z = TWO ? Z_OFF + A_BYTES : 0;
  constexpr int LDS_BYTES = LDS_A > LDS_Z ? LDS_A : LDS_Z;
  static_assert(LDS_BYTES <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  const uint32_t L0 = lds_addr(lds);

  const int nN = p.N / kTN, mtiles = (p.M + kTM - 1) / kTM;
  const ConvGeo& g = p.g;
  const int nk = p.K / BK;
  // diagnostics (p.tbuf set by probes only): wall-clock stamps of this block's phases
  auto stamp = [&](int i) {
    if (p.tbuf != nullptr && threadIdx.x == 0) p.tbuf[static_cast<int64_t>(blockIdx.x) * 8 + i] = wall_clock64();
  };
  stamp(0);
  // ---- one 256 x 256 tile per block, over all of K
  const int L = xcd_remap_big(blockIdx.x, gridDim.x);
  constexpr int kb = 0;
  const int ke = nk;
  const int mt = L / nN, n0 = (L - mt * nN) * kTN;
  const int m0 = mt * kTM;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int fr = lane & 31, fh = lane >> 5;

  // ---- DMA sources: lane-linear LDS rows, swizzled source chunk; A rows past M read zeros
  const int lrow = lane / CPR, lch = lane % CPR;
  int64_t abase[PA];
  unsigned aok = 0;
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int r = (wave * PA + i) * RPI + lrow, m = m0 + r;
    int64_t off = 0;
    if (m < p.M) {
      if (g.stride == 1) {
        off = static_cast<int64_t>(m) * g.C;
      } else {  // stride-2 downsample: output pixel (img, oh, ow) reads input (img, 2 oh, 2 ow)
        const int img = static_cast<int>(fdiv_big(static_cast<uint32_t>(m), p.fd_ohw));
        const int rr = m - img * (g.OH * g.OW);
        const int oh = static_cast<int>(fdiv_big(static_cast<uint32_t>(rr), p.fd_ow)), ow = rr - oh * g.OW;
        off = ((static_cast<int64_t>(img) * g.H + oh * g.stride) * g.W + ow * g.stride) * g.C;
      }
      aok |= 1u << i;
    }
    abase[i] = off + bswz(r, lch) * 8;
  }
  const uint16_t* bsrc[PB];
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int r = (wave * PB + i) * RPI + lrow;
    bsrc[i] = p.b + static_cast<int64_t>(n0 + r) * p.K + bswz(r, lch) * 8;
  }
  auto issue_z = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const uint16_t* src = ((aok >> i) & 1u) ? p.a2 + abase[i] + k0 : kBigZero;
      __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(lds + Z_OFF + (wave * PA + i) * 1024), 16, 0, 0);
    }
  };
  // the prologue pass over stage kt's A tile (in place): thread t owns logical chunk t & 7 (fixed
  // channels: one coefficient load per stage) of rows (t >> 3) + (NT / 8) i
  // coefficients of the pass over stage kt (thread t: logical chunk t & 7): NCO untracked 16-B loads
  // issued before the stage's DMA, waited for by vmcnt(GPS) behind it
  constexpr int NCO = PRO == 1 ? 4 : PRO == 2 ? 6 : 8;
  f32x4 co[NCO];
  auto load_coef = [&](int kt) {
    const int cc = kt * BK + (t & 7) * 8;
    const float* src[4] = {p.pro, p.pro, p.pro, p.pro};
    if constexpr (PRO == 2) {
      src[0] = p.bwd;
      src[1] = p.bwd + g.C;
      src[2] = p.bwd + 2 * g.C;
    } else {
      src[0] = p.pro;
      src[1] = p.pro + g.C;
      if constexpr (PRO == 3) {
        const bool dual = p.pro2 != nullptr;  // block-uniform; without it two dummy loads keep the count
        src[2] = dual ? p.pro2 : p.pro;
        src[3] = dual ? p.pro2 + g.C : p.pro;
      }
    }
#pragma unroll
    for (int i = 0; i < NCO / 2; ++i) {
      co[2 * i] = gld_f4(src[i] + cc);
      co[2 * i + 1] = gld_f4(src[i] + cc + 4);
    }
  };
  // the prologue pass over stage kt's A tile (in place): thread t owns logical chunk t & 7 (fixed
  // channels) of rows (t >> 3) + TRP i
  auto transform = [&](int kt, int buf) {
    uint8_t* As = lds + buf * STAGE;
    const uint8_t* Zs = lds + Z_OFF;
    const int lc = t & 7, tr0 = t >> 3, cc = kt * BK + lc * 8;
#pragma unroll
    for (int i = 0; i < NCO; ++i) tie(co[i]);
    float c0[8], c1[8], c2[8], c3[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c0[j] = co[0][j];
      c0[j + 4] = co[1][j];
      c1[j] = co[2][j];
      c1[j + 4] = co[3][j];
      if constexpr (NCO >= 6) {
        c2[j] = co[4][j];
        c2[j + 4] = co[5][j];
      }
      if constexpr (NCO >= 8) {
        c3[j] = co[6][j];
        c3[j + 4] = co[7][j];
      }
    }
    const bool dual = PRO == 3 && p.pro2 != nullptr;
    const bool store_a = (PRO == 2 || PRO == 3) && p.aout != nullptr && n0 == 0;
    constexpr int TRP = NT / 8, NR = kTM / TRP, HB = TWO ? 2 : NR;  // rows read together (register budget)
#pragma unroll
    for (int h = 0; h < NR; h += HB) {
    u16x8 va[HB], za[HB];
#pragma unroll
    for (int i = 0; i < HB; ++i) {  // the rows' reads before any use (one LDS latency per group)
      const int r = tr0 + TRP * (h + i), off = r * RB + bswz(r, lc) * 16;
      va[i] = *reinterpret_cast<const u16x8*>(As + off);
      if constexpr (TWO) za[i] = *reinterpret_cast<const u16x8*>(Zs + off);
    }
#pragma unroll
    for (int i = 0; i < HB; ++i) {
      const int r = tr0 + TRP * (h + i), m = m0 + r;
      const int off = r * RB + bswz(r, lc) * 16;
      u16x8 v = va[i];
      unsigned ob = 0;
      if constexpr (PRO == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float o = bf16_to_f32(v[j]) * c0[j] + c1[j];
          v[j] = f32_to_bf16(o > 0.f ? o : 0.f);
        }
      } else if constexpr (PRO == 2) {
        const u16x8 z8 = za[i];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = f32_to_bf16(c0[j] * bf16_to_f32(v[j]) + c1[j] * bf16_to_f32(z8[j]) + c2[j]);
      } else if constexpr (PRO == 3) {  // the arithmetic of bn_apply_kernel / bn_apply_dual_kernel
        const u16x8 z8 = za[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float o = bf16_to_f32(v[j]) * c0[j] + c1[j];
          if (dual) o = o + (bf16_to_f32(z8[j]) * c2[j] + c3[j]);
          else o += bf16_to_f32(z8[j]);
          o = o > 0.f ? o : 0.f;
          ob |= (o > 0.f ? 1u : 0u) << j;
          v[j] = f32_to_bf16(o);
        }
      }
      const bool ok = m < p.M;
      if (!ok) v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      *reinterpret_cast<u16x8*>(As + off) = v;
      if (store_a && ok) {
        const int64_t e = static_cast<int64_t>(m) * g.C + cc;
        *reinterpret_cast<u16x8*>(p.aout + e) = v;
        if constexpr (PRO == 3) p.abits[e >> 3] = static_cast<uint8_t>(ob);
      }
    }
    }
  };
  auto issue = [&](int kt, int buf) {
    uint8_t* As = lds + buf * STAGE;
    uint8_t* Bs = As + A_BYTES;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const uint16_t* src = ((aok >> i) & 1u) ? p.a + abase[i] + k0 : kBigZero;
      __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(As + (wave * PA + i) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < PB; ++i)
      __builtin_amdgcn_global_load_lds((gptr_t*)(bsrc[i] + k0), (lptr_t*)(Bs + (wave * PB + i) * 1024), 16, 0, 0);
  };

  // ---- fragment addresses: wave (wm, wn) = pixels 128 wm.., channels 64 wn..; the chunk swizzle
  // of rows 32 j + fr is the same for every block j, so one address per k-step and operand, and
  // the blocks are immediate offsets (32 rows = 32 RB bytes apart)
  const int wm = wave / WN, wn = wave % WN;
  uint32_t fa[KSTEPS], fb[KSTEPS];
#pragma unroll
  for (int s = 0; s < KSTEPS; ++s) {
    const int ch = bswz(fr, 2 * s + fh) * 16;
    fa[s] = static_cast<uint32_t>((128 * wm + fr) * RB + ch);
    fb[s] = static_cast<uint32_t>(A_BYTES + (WCH * wn + fr) * RB + ch);
  }
  f32x16 acc[TI][4];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  constexpr int OJ = 32 * RB;  // bytes between 32-row fragment blocks
  bf16x8_t xa[2][4], wb[2][TI];
  auto fetch = [&](uint32_t sb, int s, int set) {
    const uint32_t a = sb + fa[s], b = sb + fb[s];
    xa[set][0] = ld_b128o<0>(a);
    xa[set][1] = ld_b128o<OJ>(a);
    xa[set][2] = ld_b128o<2 * OJ>(a);
    xa[set][3] = ld_b128o<3 * OJ>(a);
    wb[set][0] = ld_b128o<0>(b);
    wb[set][1] = ld_b128o<OJ>(b);
  };
  constexpr int FR = 4 + TI;  // fragment reads per k-step
  auto mfma_set = [&](int set) {
#pragma unroll
    for (int j = 0; j < 4; ++j) tie(xa[set][j]);
#pragma unroll
    for (int i = 0; i < TI; ++i) tie(wb[set][i]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wb[set][i], xa[set][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (PRO != 0) {
    // stage kt + 1 (and a2 of kt + 1 once the pass over kt has read the a2 tile) in flight behind
    // stage kt's pass and MFMAs; the pass's aout stores drain with them
    issue(kb, 0);
    if constexpr (TWO) issue_z(kb);
    for (int kt = kb; kt < ke; ++kt) {
      wait_vm<0>();
      lds_bar();  // stage kt (and its a2 tile) landed; every wave is done with stage kt - 1
      load_coef(kt);
      if (kt + 1 < ke) {
        issue(kt + 1, (kt + 1 - kb) & 1);
        wait_vm<GPS>();  // the coefficients (older than the stage's GPS DMAs)
      } else {
        wait_vm<0>();
      }
      transform(kt, (kt - kb) & 1);
      lds_bar();  // the A tile is transformed and the a2 tile is free
      if constexpr (TWO) {
        if (kt + 1 < ke) issue_z(kt + 1);
      }
      const uint32_t sb = L0 + static_cast<uint32_t>(((kt - kb) & 1) * STAGE);
      fetch(sb, 0, 0);
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        if (s + 1 < KSTEPS) {
          fetch(sb, s + 1, (s + 1) & 1);
          wait_lgkm<FR>();
        } else {
          wait_lgkm<0>();
        }
        mfma_set(s & 1);
      }
    }
  }
  // ---- prologue: stages 0 .. NST - 2 in flight
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) {
    if (PRO == 0 && kb + s < ke) issue(kb + s, s);
  }
  for (int kt = kb; kt < (PRO == 0 ? ke : kb); ++kt) {
    // stage kt landed (this wave's DMAs): younger are the min(NST - 2, ke - 1 - kt) stages after it
    const int younger = min(NST - 2, ke - 1 - kt);
    if (younger >= 2) {
      wait_vm<2 * GPS>();
    } else if (younger == 1) {
      wait_vm<GPS>();
    } else {
      wait_vm<0>();
    }
    lds_bar();  // every wave's stage kt landed; every wave is done with stage kt - 1's buffer
    if (kt == kb) stamp(1);
    if (kt + NST - 1 < ke) issue(kt + NST - 1, (kt - kb + NST - 1) % NST);
    const uint32_t sb = L0 + static_cast<uint32_t>(((kt - kb) % NST) * STAGE);
    fetch(sb, 0, 0);
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      if (s + 1 < KSTEPS) {
        fetch(sb, s + 1, (s + 1) & 1);
        wait_lgkm<FR>();
      } else {
        wait_lgkm<0>();
      }
      mfma_set(s & 1);
    }
  }
  stamp(2);
  wait_vm<0>();
  lds_bar();  // the output tile overlays the stage ring

  // ---- accumulators -> bf16 output tile [256 px][kCS]: register q of acc[i][j] is channel
  // 64 wn + 32 i + 8 (q >> 2) + 4 fh + (q & 3) of pixel 128 wm + 32 j + fr
  uint16_t* Cs = reinterpret_cast<uint16_t*>(lds);
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const int nl = WCH * wn + 32 * i + 8 * q4 + 4 * fh, ml = 128 * wm + 32 * j + fr;
        const u16x4 v = {f32_to_bf16(acc[i][j][4 * q4]), f32_to_bf16(acc[i][j][4 * q4 + 1]),
                         f32_to_bf16(acc[i][j][4 * q4 + 2]), f32_to_bf16(acc[i][j][4 * q4 + 3])};
        *reinterpret_cast<u16x4*>(Cs + ml * kCS + nl) = v;
      }
  lds_bar();
  stamp(3);

  // ---- row pass: thread t owns channels [8 cg, 8 cg + 8) of rows r0 + 16 i
  // EPI 5/6/9: + the residual rows masked by the block output's ReLU bits (aux, bits); EPI 2/7:
  // + the residual rows; EPI 4/8: + the stride-2 residual map at even (h, w); 6-9 also mask by the
  // previous block's output bits (bits2) and reduce its bn3 backward sums over aux2 (and, 9, the
  // downsample BN's sum over aux3) -- conv_gemm's epilogues, see convgemm.hip conv_fwd_body
  constexpr bool FOLD = EPI >= 6;
  constexpr bool FOLD_DS = EPI == 9;
  constexpr int BASE = EPI == 6 || EPI == 9 ? 5 : EPI == 7 ? 2 : EPI == 8 ? 4 : EPI;
  constexpr bool SUMS = EPI == 1 || EPI == 3 || FOLD;
  constexpr bool RD_AUX = BASE == 2 || BASE == 4 || BASE == 5 || EPI == 3;
  constexpr int CG = kTN / 8, RPP = NT / CG;  // 16-B column groups per row; rows per pass
  const int cg = t % CG, r0 = t / CG, nc = n0 + cg * 8;
  float e0[8], e1[8], e2[8], e3[8], s1[8], s2[8], s3[FOLD_DS ? 8 : 1], e4[FOLD_DS ? 8 : 1], e5[FOLD_DS ? 8 : 1];
#pragma unroll
  for (int e = 0; e < 8; ++e) e0[e] = e1[e] = e2[e] = e3[e] = s1[e] = s2[e] = 0.f;
  if constexpr (FOLD_DS) {
#pragma unroll
    for (int e = 0; e < 8; ++e) s3[e] = 0.f;
    load8(p.mean2, nc, e4);
    load8(p.invstd2, nc, e5);
  }
  if constexpr (EPI == 1) {
    if (p.kshift) load8(p.kshift, nc, e0);
  } else if constexpr (EPI == 3) {
    load8(p.mc, nc, e0);
    load8(p.mc + p.N, nc, e1);
    load8(p.mean, nc, e2);
    load8(p.invstd, nc, e3);
  } else if constexpr (FOLD) {
    load8(p.mean, nc, e2);
    load8(p.invstd, nc, e3);
  }
  constexpr int NPASS = kTM / RPP;
  // rows in flight per group: all of a group's row reads are issued before any is consumed (8: no
  // spill with every epilogue at the K loop's 204-VGPR high-water mark)
  constexpr int RIF = 4;
#pragma unroll
  for (int h = 0; h < NPASS; h += RIF) {
    u16x8 ra[RD_AUX ? RIF : 1], rz[FOLD ? RIF : 1], rd[FOLD_DS ? RIF : 1];
    uint32_t rb[BASE == 5 ? RIF : 1], rp[FOLD ? RIF : 1];
    unsigned rodd = 0;
#pragma unroll
    for (int i = 0; i < RIF; ++i) {
      const int m = min(m0 + r0 + RPP * (h + i), p.M - 1);
      const int64_t o = static_cast<int64_t>(m) * p.N + nc;
      if constexpr (BASE == 4) {  // residual map (OH+1)/2 x (OW+1)/2, present at even (h, w)
        const int ohw = g.OH * g.OW;
        const int im = static_cast<int>(fdiv_big(static_cast<uint32_t>(m), p.fd_ohw)), r = m - im * ohw,
                  hh = static_cast<int>(fdiv_big(static_cast<uint32_t>(r), p.fd_ow)), ww = r - hh * g.OW;
        const int RH = (g.OH + 1) >> 1, RW = (g.OW + 1) >> 1;
        rodd |= static_cast<unsigned>((hh | ww) & 1) << i;
        const int64_t ro = ((static_cast<int64_t>(im) * RH + (hh >> 1)) * RW + (ww >> 1)) * p.N + nc;
        ra[i] = *reinterpret_cast<const u16x8*>(p.aux + ((hh | ww) & 1 ? int64_t(0) : ro));
      } else if constexpr (RD_AUX) {
        ra[i] = *reinterpret_cast<const u16x8*>(p.aux + o);
      }
      if constexpr (BASE == 5) rb[i] = p.bits[o >> 3];
      if constexpr (FOLD) {
        rz[i] = *reinterpret_cast<const u16x8*>(p.aux2 + o);
        rp[i] = p.bits2[o >> 3];
      }
      if constexpr (FOLD_DS) rd[i] = *reinterpret_cast<const u16x8*>(p.aux3 + o);
    }
#pragma unroll
    for (int i = 0; i < RIF; ++i) {
      const int rr = r0 + RPP * (h + i), m = m0 + rr;
      if (m >= p.M) break;
      const u16x4 lo = *reinterpret_cast<const u16x4*>(Cs + rr * kCS + cg * 8);
      const u16x4 hi = *reinterpret_cast<const u16x4*>(Cs + rr * kCS + cg * 8 + 4);
      u16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if constexpr (BASE == 5) {  // identity-branch gradient = dout * relu'(block output), from bits
        v = bf16_add_where(v, ra[i], rb[i]);
      } else if constexpr (BASE == 2 || BASE == 4) {
        if (BASE == 2 || !((rodd >> i) & 1u)) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = f32_to_bf16(bf16_to_f32(v[e]) + bf16_to_f32(ra[i][e]));
        }
      } else if constexpr (EPI == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = bf16_to_f32(v[e]) - e0[e];
          s1[e] += d;
          s2[e] += d * d;
        }
      } else if constexpr (EPI == 3) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float z = bf16_to_f32(ra[i][e]);
          const bool on = z * e0[e] + e1[e] > 0.f;
          const float gv = on ? bf16_to_f32(v[e]) : 0.f;
          s1[e] += gv;
          s2[e] += gv * ((z - e2[e]) * e3[e]);
          if (!on) v[e] = 0;
        }
      }
      if constexpr (FOLD) {  // previous block's bn3: ReLU mask from its output bits + reduce sums
        v = bf16_keep_where(v, rp[i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gv = bf16_to_f32(v[e]);
          s1[e] += gv;
          s2[e] += gv * ((bf16_to_f32(rz[i][e]) - e2[e]) * e3[e]);
          if constexpr (FOLD_DS) s3[e] += gv * ((bf16_to_f32(rd[i][e]) - e4[e]) * e5[e]);
        }
      }
      *reinterpret_cast<u16x8*>(p.c + static_cast<int64_t>(m) * p.N + nc) = v;
    }
  }
  if constexpr (SUMS) {
    // threads of one column group: lanes l, l + CG, .. of each wave, then the NW waves in fixed order
#pragma unroll
    for (int off = CG; off < 64; off *= 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += __shfl_xor(s1[e], off, 64);
        s2[e] += __shfl_xor(s2[e], off, 64);
        if constexpr (FOLD_DS) s3[e] += __shfl_xor(s3[e], off, 64);
      }
    }
    float* red = reinterpret_cast<float*>(lds + RED_OFF);  // [NSUM][NW waves][TN]
    if (lane < CG) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[wave * kTN + cg * 8 + e] = s1[e];
        red[(NW + wave) * kTN + cg * 8 + e] = s2[e];
        if constexpr (FOLD_DS) red[(2 * NW + wave) * kTN + cg * 8 + e] = s3[e];
      }
    }
    __syncthreads();
    if (t < kTN) {
      float a = 0.f, b = 0.f, c3 = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        a += red[w * kTN + t];
        b += red[(NW + w) * kTN + t];
        if constexpr (FOLD_DS) c3 += red[(2 * NW + w) * kTN + t];
      }
      const int64_t PG = p.pgm > 0 ? p.pgm : mtiles;
      p.part[static_cast<int64_t>(mt) * p.N + n0 + t] = a;
      p.part[(PG + mt) * p.N + n0 + t] = b;
      if constexpr (FOLD_DS) p.part[(2 * PG + mt) * p.N + n0 + t] = c3;
    }
  }
  if (p.tbuf != nullptr) {
    stamp(4);  // stores issued
    wait_vm<0>();
    stamp(5);  // thread 0's stores acknowledged
    if (threadIdx.x == 0) p.tbuf[static_cast<int64_t>(blockIdx.x) * 8 + 6] = __smid();
  }
}

}  // namespace

// the 256-channel-tile launches
static void launch_big256(const ConvGemmArgs& a, hipStream_t s, bool bwd, bool resp) {
  const int nblk = conv_big_gm(a.M) * (a.N / 256);
#define PSAMD_BIG(E, P) hipLaunchKernelGGL((conv_big_kernel<E, P>), dim3(nblk), dim3(512), 0, s, a)
  if (bwd) {
    switch (a.epi) {
      case 2: PSAMD_BIG(2, 2); break;
      case 4: PSAMD_BIG(4, 2); break;
      case 5: PSAMD_BIG(5, 2); break;
      case 6: PSAMD_BIG(6, 2); break;
      case 7: PSAMD_BIG(7, 2); break;
      case 8: PSAMD_BIG(8, 2); break;
      case 9: PSAMD_BIG(9, 2); break;
      default: PSAMD_BIG(3, 2); break;
    }
  } else if (resp) {
    if (a.epi == 1) PSAMD_BIG(1, 3);
    else PSAMD_BIG(0, 3);
  } else if (a.pro != nullptr) {
    if (a.epi == 1) PSAMD_BIG(1, 1);
    else PSAMD_BIG(0, 1);
  } else {
    switch (a.epi) {
      case 1: PSAMD_BIG(1, 0); break;
      case 2: PSAMD_BIG(2, 0); break;
      case 3: PSAMD_BIG(3, 0); break;
      case 4: PSAMD_BIG(4, 0); break;
      case 5: PSAMD_BIG(5, 0); break;
      case 6: PSAMD_BIG(6, 0); break;
      case 7: PSAMD_BIG(7, 0); break;
      case 8: PSAMD_BIG(8, 0); break;
      case 9: PSAMD_BIG(9, 0); break;
      default: PSAMD_BIG(0, 0); break;
    }
  }
#undef PSAMD_BIG
}

// Eligible: a 1x1 GEMM (rows in order) with K = C, N a multiple of 256, K >= 256, and >= 1024
// blocks or K >= 1024 (with >= 256 blocks); epilogues 0 / 1 / 3 with or without a stride-1
// prologue, the residual / fold epilogues 2, 4-9 without one (or with the BN backward one).
int conv_big_tn(int M, int N, int K, bool pro, const ConvGeo& g, int src2, int epi) {
  if (g.RH != 0) return 0;
  if (g.ks != 1 || g.ksw > 1 || g.pad != 0 || g.C != K) return 0;
  if (epi < 0 || epi > 9) return 0;
  if (N % 256 != 0 || K % 64 != 0 || K < 256) return 0;
  const bool plain_epi = epi == 0 || epi == 1 || epi == 3;
  // the residual / fold epilogues (2, 4-9: the conv1 data gradients): no prologue, or the BN
  // backward one (the conv1 data gradient with bn1's backward applied)
  if (!plain_epi && ((pro && src2 != 2) || src2 == 1)) return 0;
  // prologues (PRO 1: pro, src2 0; PRO 3: src2 1; PRO 2: src2 2 + a data-gradient epilogue): stride 1 only
  if (pro || src2 != 0) {
    if (g.stride != 1) return 0;
    if (src2 == 2 && (epi == 0 || epi == 1)) return 0;
    if (src2 == 1 && epi == 3) return 0;
  }
  // one block per CU: below ~4 rounds of blocks the last round's idle CUs and the per-tile
  // prologue / epilogue outweigh the faster K loop unless K is deep (profiles/r5_conv_big_probe.txt:
  // at batch 256 the K = 256 / 512 shapes with 784 blocks ran 2-15 % slower, K >= 1024 faster)
  const int64_t nblk = static_cast<int64_t>(conv_big_gm(M)) * (N / 256);
  return nblk >= 256 && (nblk >= 1024 || K >= 1024) ? 256 : 0;
}

bool conv_big_ok(int M, int N, int K, bool pro, const ConvGeo& g, int src2, int epi) {
  return conv_big_tn(M, N, K, pro, g, src2, epi) != 0;
}

int conv_big_gm(int M) { return (M + kTM - 1) / kTM; }

void launch_conv_big(const ConvGemmArgs& a, hipStream_t s) {
  const bool bwd = a.bwd != nullptr, resp = a.pro != nullptr && a.a2 != nullptr && !bwd;
  launch_big256(a, s, bwd, resp);
}

}  // namespace psamd
