// The 64-channel 3x3 stride-1 convolutions of ResNet-50 layer 1 (56 x 56 maps): forward (epilogue
// 1: the next BN's statistics) and data gradient (the same GEMM over dz with the flipped,
// channel-transposed weight; epilogue 3: the previous BN's ReLU mask + backward sums).
//
// Reference hot op: layer/Conv2DLayer.java:146-240 (im2col + GEMM).  The im2col view re-reads
// every input pixel nine times; here a persistent block per CU keeps the WHOLE weight
// (9 taps x 64 x 64 bf16 = 72 KiB) resident in LDS and walks tiles of two output rows (112 pixels):
// each tile's input PATCH -- 4 rows x 58 columns with zero halo -- lands once by LDS-DMA, two
// patch slots deep (the next tile's patch streams in while this one computes), and the nine taps
// read their B fragments from the same patch at shifted slots.
//
// Both LDS images are PLANAR: 16-B chunk c (channels 8c .. 8c + 7) of every slot / weight row is
// stored contiguously (plane c), so a fragment read of 32 consecutive pixels (or output channels)
// is 512 contiguous bytes -- conflict-free with no swizzle -- and a DMA piece is 64 consecutive
// slots of one plane.  Fragment reads are inline asm (ds_read_b128): the compiler otherwise
// orders every LDS read behind the patch DMA in flight to the other slot (s_waitcnt vmcnt(0) at
// the loop edge -- what kept the round-4 version of this kernel at 0.48 ms), and the reads of
// k-step i + 1 are issued before the MFMAs of step i.  One wave per SIMD (4 waves): each wave
// owns 64 pixels x 32 output channels (two 32 x 32 blocks sharing the weight fragment: 1.5 LDS
// reads per MFMA).  The epilogue leaves straight from the accumulators (4 channels = 8 B per
// store); its statistics accumulate per lane over the block's tiles and fold once at the end.
#include <algorithm>
#include <cstdlib>

#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8_c64 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(1))) const void gptr_t;
typedef __attribute__((address_space(3))) void lptr_t;
typedef __attribute__((address_space(3))) const char lds_char;

__device__ __attribute__((aligned(16))) uint16_t kZeroPatch[8] = {0, 0, 0, 0, 0, 0, 0, 0};
// store sink of the epilogue's invalid pixels: every tile issues the same number of stores, so
// the counted wait on the next patch never depends on how many pixels a tile has
__device__ __attribute__((aligned(16))) uint16_t kStoreSink[64 * 4];

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_char*)p));
}
__device__ __forceinline__ bf16x8_t ld_b128(uint32_t a) {
  bf16x8_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ f32x4 ld_f4c(uint32_t a) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ void st_b128(uint32_t a, bf16x8_t v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}
template <typename T>
__device__ __forceinline__ void tie(T& v) {
  asm volatile("" : "+v"(v));
}
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
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

template <int W, int EPI, int LA>
__global__ __launch_bounds__(256, 1) void conv3x3_c64s_kernel(const ConvGemmArgs p) {
  static_assert(EPI == 1 || EPI == 3, "forward statistics or data-gradient mask + sums");
  constexpr int C = 64, N = 64, RT = 2, TP = RT * W;       // rows / pixels per tile
  constexpr int PW = W + 2, PR = RT + 2, NSL = PR * PW;     // patch slots (rows x cols)
  constexpr int PLS = (NSL + 63) / 64 * 64;                 // slots per plane (whole 1-KiB pieces)
  constexpr int PLB = PLS * 16;                             // bytes per patch plane
  constexpr int SLOT = 8 * PLB;                             // bytes per patch
  constexpr int PPW = (8 * PLS / 64) / 4;                   // patch pieces per wave
  constexpr int WPL = 9 * N * 16;                           // bytes per weight plane (9 taps x 64 rows)
  constexpr int WPW = (8 * 9 * N / 64) / 4;                 // weight pieces per wave
  constexpr int P_OFF = 8 * WPL, RED_OFF = P_OFF + 2 * SLOT;
  constexpr int LDS_BYTES = RED_OFF + 2 * 2 * N * 4;
  static_assert((8 * PLS / 64) % 4 == 0 && (8 * 9 * N / 64) % 4 == 0, "pieces over 4 waves");
  static_assert(LDS_BYTES <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  const uint32_t L0 = lds_addr(lds);

  const ConvGeo& g = p.g;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int fr = lane & 31, fh = lane >> 5;
  const int GM = gridDim.x, mg = blockIdx.x;
  const int tpi = g.OH / RT, ntiles = (p.M / (g.OH * W)) * tpi;
  const int my_tiles = mg < ntiles ? (ntiles - mg + GM - 1) / GM : 0;  // block-uniform

  // ---- resident weight, planar: plane c holds chunk c of row (tap * 64 + n); piece k = 64 rows
  {
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      const int pc = wave * WPW + i, pl = pc / 9, r = (pc - pl * 9) * 64 + lane;  // row = tap * 64 + n
      const int tap = r >> 6, n = r & 63;
      __builtin_amdgcn_global_load_lds((gptr_t*)(p.b + static_cast<int64_t>(n) * p.K + tap * C + pl * 8),
                                       (lptr_t*)(lds + pl * WPL + (pc - pl * 9) * 1024), 16, 0, 0);
    }
  }
  // ---- patch of tile mt into slot sl: plane pl, piece k (64 lane-linear slots); ALWAYS PPW DMA
  // instructions per wave (zero rows past the block's tiles)
  auto issue_patch = [&](int mt, bool real, int sl) {
    const int img = mt / tpi, oh0 = (mt - img * tpi) * RT;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i, pl = pc / (PLS / 64), sq = (pc - pl * (PLS / 64)) * 64 + lane;
      const int pr = sq / PW, pcol = sq - pr * PW, ih = oh0 - 1 + pr, iw = pcol - 1;
      const bool ok = real && sq < NSL && static_cast<unsigned>(ih) < static_cast<unsigned>(g.H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(W);
      const uint16_t* src =
          ok ? p.a + ((static_cast<int64_t>(img) * g.H + ih) * W + iw) * C + pl * 8 : kZeroPatch;
      __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(lds + P_OFF + sl * SLOT + pc * 1024), 16, 0, 0);
    }
  };

  // ---- lane constants: wave = 64 pixels (blocks j = 0, 1) x 32 output channels
  const int ob = wave & 1, pp = wave >> 1;
  const int oc0 = 32 * ob + fr;                                      // A-fragment row (output channel)
  const uint32_t abase = L0 + static_cast<uint32_t>(fh * WPL + oc0 * 16);  // + plane 2ks, tap * 1024
  uint32_t bbase[2];
  bool pvalid[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int px = 64 * pp + 32 * j + fr;
    pvalid[j] = px < TP;
    const int sl0 = pvalid[j] ? (px / W) * PW + (px % W) : 0;
    bbase[j] = static_cast<uint32_t>(P_OFF + fh * PLB + sl0 * 16);
  }
  // epilogue: register q of block j = output channel 32 ob + 8 (q >> 2) + 4 fh + (q & 3) of pixel
  // 64 pp + 32 j + fr -> four consecutive channels per q >> 2 (one 8-B store)
  float e0[16], e1[16], e2[16], e3[16];  // EPI 1: kshift; EPI 3: scale, shift, mean, invstd
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = 32 * ob + 8 * (i >> 2) + 4 * fh + (i & 3);
    if constexpr (EPI == 1) {
      e0[i] = p.kshift ? p.kshift[c] : 0.f;
      e1[i] = e2[i] = e3[i] = 0.f;
    } else {
      e0[i] = p.mc[c];
      e1[i] = p.mc[N + c];
      e2[i] = p.mean[c];
      e3[i] = p.invstd[c];
    }
  }
  float s1[16], s2[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) s1[i] = s2[i] = 0.f;

  // ---- prologue: weight, patch 0 (and 1); wait for the weight and patch 0
  if (my_tiles > 0) issue_patch(mg, true, 0);
  issue_patch(my_tiles > 1 ? mg + GM : mg, my_tiles > 1, 1);
  wait_vm<PPW>();
  lds_bar();

  f32x16 acc[2];
  for (int ti = 0, mt = mg; ti < my_tiles; ++ti, mt += GM) {
    const int sl = ti & 1;
    // EPI 3: this tile's BN-input rows, issued before the MFMAs (rows past M read the last row)
    u16x4 zr[2][4];
    const int m0 = mt * TP;
    if constexpr (EPI == 3) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const int px = 64 * pp + 32 * j + fr, m = min(m0 + (pvalid[j] ? px : 0), p.M - 1);
          zr[j][q4] = *reinterpret_cast<const u16x4*>(p.aux + static_cast<int64_t>(m) * N + 32 * ob + 8 * q4 + 4 * fh);
        }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[j][q] = 0.f;
    // ---- 36 k-steps (9 taps x 4 of 16 channels): the reads of step i + 1 before the MFMAs of i
    const uint32_t pb0 = L0 + static_cast<uint32_t>(sl * SLOT) + bbase[0], pb1 = L0 + static_cast<uint32_t>(sl * SLOT) + bbase[1];
    // LA + 1 register sets: the reads of step st + LA are in flight while step st's MFMAs issue
    // (LDS latency exceeds the 64 cycles of one step's two MFMAs at one wave per SIMD)
    constexpr int NB = LA + 1;
    bf16x8_t wa[NB], xa[NB][2];
    auto fetch = [&](int st, int buf) {
      const int tap = st >> 2, ks = st & 3, kh = tap / 3, kw = tap - kh * 3;
      const uint32_t ao = static_cast<uint32_t>(2 * ks * WPL + tap * 1024);
      const uint32_t bo = static_cast<uint32_t>(2 * ks * PLB + (kh * PW + kw) * 16);
      wa[buf] = ld_b128(abase + ao);
      xa[buf][0] = ld_b128(pb0 + bo);
      xa[buf][1] = ld_b128(pb1 + bo);
    };
#pragma unroll
    for (int st = 0; st < LA; ++st) fetch(st, st);
#pragma unroll
    for (int st = 0; st < 36; ++st) {
      const int cur = st % NB;
      if (st + LA < 36) {
        fetch(st + LA, (st + LA) % NB);
        wait_lgkm<3 * LA>();  // step st's three reads landed; the next LA steps' stay in flight
      } else if (st + 2 == 36 && LA >= 2) {
        wait_lgkm<3>();
      } else {
        wait_lgkm<0>();
      }
      tie(wa[cur]);
      tie(xa[cur][0]);
      tie(xa[cur][1]);
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[cur], xa[cur][0], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[cur], xa[cur][1], acc[1], 0, 0, 0);
    }
    // ---- every wave is done with patch slot sl: the patch of tile ti + 2 may stream into it
    lds_bar();
    const bool more2 = ti + 2 < my_tiles;
    issue_patch(more2 ? mt + 2 * GM : mg, more2, sl);
    // ---- epilogue straight from the accumulators: 8 stores per lane, always issued
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int px = 64 * pp + 32 * j + fr, m = m0 + px;
      const bool ok = pvalid[j] && m < p.M;
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        u16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f32_to_bf16(acc[j][4 * q4 + e]);
        if constexpr (EPI == 1) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = ok ? bf16_to_f32(v[e]) - e0[4 * q4 + e] : 0.f;
            s1[4 * q4 + e] += d;
            s2[4 * q4 + e] += d * d;
          }
        } else {
          const u16x4 z4 = zr[j][q4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int i = 4 * q4 + e;
            const float z = bf16_to_f32(z4[e]);
            const bool on = ok && z * e0[i] + e1[i] > 0.f;
            const float gv = on ? bf16_to_f32(v[e]) : 0.f;
            s1[i] += gv;
            s2[i] += gv * ((z - e2[i]) * e3[i]);
            if (!on) v[e] = 0;
          }
        }
        uint16_t* dst = ok ? p.c + static_cast<int64_t>(m) * N + 32 * ob + 8 * q4 + 4 * fh : kStoreSink + (lane & 63) * 4;
        *reinterpret_cast<u16x4*>(dst) = v;
      }
    }
    // ---- patch ti + 1 landed (this wave's pieces): younger than it are the patch ti + 2 just
    // issued (PPW) and the 8 epilogue stores; then every wave's pieces
    wait_vm<PPW + 8>();
    lds_bar();
  }
  wait_vm<0>();
  lds_bar();
  // ---- statistics: over the 32 pixel lanes of each half, then the two pixel-pair waves
#pragma unroll
  for (int off = 1; off < 32; off <<= 1)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      s1[i] += __shfl_xor(s1[i], off, 64);
      s2[i] += __shfl_xor(s2[i], off, 64);
    }
  float* red = reinterpret_cast<float*>(lds + RED_OFF);  // [2 stats][2 pp][N]
  if (fr == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 32 * ob + 8 * (i >> 2) + 4 * fh + (i & 3);
      red[pp * N + c] = s1[i];
      red[(2 + pp) * N + c] = s2[i];
    }
  }
  __syncthreads();
  if (t < N) {
    p.part[static_cast<int64_t>(mg) * N + t] = red[t] + red[N + t];
    p.part[(static_cast<int64_t>(GM) + mg) * N + t] = red[2 * N + t] + red[3 * N + t];
  }
}


// Mode 3: the weight in REGISTERS.  Every wave holds the whole 64 x 576 weight as MFMA A fragments
// (36 k-steps x 2 output-channel blocks x 16 B = 288 VGPRs, one wave per SIMD) and owns 32 pixels x
// all 64 channels of the tile, so a k-step is ONE ds_read_b128 of the patch for two MFMAs (0.5
// LDS reads per MFMA, against 1.5 with the weight in LDS: there the LDS array was ~75 % busy
// beside the MFMAs).  The LDS holds only the two patch slots and the epilogue parameters.
template <int W, int EPI, int LA, int DBG = 0>
__global__ __launch_bounds__(256, 1) void conv3x3_c64r_kernel(const ConvGemmArgs p) {
  // DBG (timing probes only): 1 = no MFMAs (data movement + epilogue), 2 = no patch DMA (compute
  // on whatever the slots hold), 3 = no epilogue stores
  static_assert(EPI == 1 || EPI == 3, "forward statistics or data-gradient mask + sums");
  constexpr int C = 64, N = 64, RT = 2, TP = RT * W;
  constexpr int PW = W + 2, PR = RT + 2, NSL = PR * PW;
  constexpr int PLS = (NSL + 63) / 64 * 64;
  constexpr int PLB = PLS * 16;
  constexpr int SLOT = 8 * PLB;
  constexpr int PPW = (8 * PLS / 64) / 4;
  constexpr int PAR_OFF = 2 * SLOT;                    // [64 ch][4] floats: e0..e3 per channel
  constexpr int RED_OFF = PAR_OFF + N * 4 * 4;
  constexpr int LDS_BYTES = RED_OFF + 2 * 4 * N * 4;
  static_assert((8 * PLS / 64) % 4 == 0, "pieces over 4 waves");
  static_assert(LDS_BYTES <= 163840, "LDS budget");
  static_assert(TP <= 128, "four 32-pixel waves per tile");
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  const uint32_t L0 = lds_addr(lds);

  const ConvGeo& g = p.g;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int fr = lane & 31, fh = lane >> 5;
  const int GM = gridDim.x, mg = blockIdx.x;
  const int tpi = g.OH / RT, ntiles = (p.M / (g.OH * W)) * tpi;
  const int my_tiles = mg < ntiles ? (ntiles - mg + GM - 1) / GM : 0;

  auto issue_patch = [&](int mt, bool real, int sl) {
    const int img = mt / tpi, oh0 = (mt - img * tpi) * RT;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i, pl = pc / (PLS / 64), sq = (pc - pl * (PLS / 64)) * 64 + lane;
      const int pr = sq / PW, pcol = sq - pr * PW, ih = oh0 - 1 + pr, iw = pcol - 1;
      const bool ok = real && sq < NSL && static_cast<unsigned>(ih) < static_cast<unsigned>(g.H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(W);
      const uint16_t* src =
          ok ? p.a + ((static_cast<int64_t>(img) * g.H + ih) * W + iw) * C + pl * 8 : kZeroPatch;
      if constexpr (DBG == 2) src = kZeroPatch;
      __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(lds + sl * SLOT + pc * 1024), 16, 0, 0);
    }
  };

  // ---- epilogue parameters -> LDS [c][4]
  for (int c = t; c < N; c += 256) {
    float* pr = reinterpret_cast<float*>(lds + PAR_OFF) + c * 4;
    if constexpr (EPI == 1) {
      pr[0] = p.kshift ? p.kshift[c] : 0.f;
      pr[1] = pr[2] = pr[3] = 0.f;
    } else {
      pr[0] = p.mc[c];
      pr[1] = p.mc[N + c];
      pr[2] = p.mean[c];
      pr[3] = p.invstd[c];
    }
  }
  // ---- the weight as A fragments: k-step st = tap (st >> 2), channels 16 (st & 3) + 8 fh + j
  bf16x8_t wr[36][2];
#pragma unroll
  for (int st = 0; st < 36; ++st)
#pragma unroll
    for (int i = 0; i < 2; ++i)
      wr[st][i] = *reinterpret_cast<const bf16x8_t*>(p.b + static_cast<int64_t>(32 * i + fr) * p.K + (st >> 2) * C +
                                                      16 * (st & 3) + 8 * fh);
  // ---- this lane's pixel: 32 wave + fr of the tile
  const int px = 32 * wave + fr;
  const bool pvalid = px < TP;
  const uint32_t bbase = static_cast<uint32_t>(fh * PLB + (pvalid ? (px / W) * PW + (px % W) : 0) * 16);
  float s1[32], s2[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) s1[i] = s2[i] = 0.f;

  if (my_tiles > 0) issue_patch(mg, true, 0);
  issue_patch(my_tiles > 1 ? mg + GM : mg, my_tiles > 1, 1);
  wait_vm<PPW>();
  __syncthreads();  // (the weight loads are plain loads: drained here with everything else once)

  f32x16 acc[2];
  for (int ti = 0, mt = mg; ti < my_tiles; ++ti, mt += GM) {
    const int sl = ti & 1;
    const int m0 = mt * TP;
    u16x4 zr[2][4];  // EPI 3: the BN input at this lane's pixel, 4 channels per (block, q4)
    if constexpr (EPI == 3) {
      const int m = min(m0 + (pvalid ? px : 0), p.M - 1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4)
          zr[i][q4] = *reinterpret_cast<const u16x4*>(p.aux + static_cast<int64_t>(m) * N + 32 * i + 8 * q4 + 4 * fh);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;
    const uint32_t pb = L0 + static_cast<uint32_t>(sl * SLOT) + bbase;
    constexpr int NB = LA + 1;
    bf16x8_t xb[NB];
    auto fetch = [&](int st, int buf) {
      const int tap = st >> 2, ks = st & 3, kh = tap / 3, kw = tap - kh * 3;
      xb[buf] = ld_b128(pb + static_cast<uint32_t>(2 * ks * PLB + (kh * PW + kw) * 16));
    };
#pragma unroll
    for (int st = 0; st < LA; ++st) fetch(st, st);
#pragma unroll
    for (int st = 0; st < 36; ++st) {
      const int cur = st % NB;
      if (st + LA < 36) {
        fetch(st + LA, (st + LA) % NB);
        wait_lgkm<LA>();
      } else if (st + 2 == 36 && LA >= 2) {
        wait_lgkm<1>();
      } else {
        wait_lgkm<0>();
      }
      tie(xb[cur]);
      if constexpr (DBG != 1) {
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wr[st][0], xb[cur], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wr[st][1], xb[cur], acc[1], 0, 0, 0);
      } else {
        acc[0][0] += static_cast<float>(__builtin_bit_cast(s16x8_c64, xb[cur])[0]);
      }
    }
    lds_bar();  // every wave is done with patch slot sl
    const bool more2 = ti + 2 < my_tiles;
    issue_patch(more2 ? mt + 2 * GM : mg, more2, sl);
    // ---- epilogue from the accumulators: register q of block i = channel 32 i + 8 (q >> 2) + 4 fh +
    // (q & 3) of this lane's pixel; 8 stores of 4 channels, always issued (sink past the tile)
    const int m = m0 + px;
    const bool ok = pvalid && m < p.M;
    const float* par = reinterpret_cast<const float*>(lds + PAR_OFF);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const int c0 = 32 * i + 8 * q4 + 4 * fh;
        u16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f32_to_bf16(acc[i][4 * q4 + e]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const f32x4 pe = *reinterpret_cast<const f32x4*>(par + (c0 + e) * 4);
          const int si = 16 * i + 4 * q4 + e;
          if constexpr (EPI == 1) {
            const float d = ok ? bf16_to_f32(v[e]) - pe[0] : 0.f;
            s1[si] += d;
            s2[si] += d * d;
          } else {
            const float z = bf16_to_f32(zr[i][q4][e]);
            const bool on = ok && z * pe[0] + pe[1] > 0.f;
            const float gv = on ? bf16_to_f32(v[e]) : 0.f;
            s1[si] += gv;
            s2[si] += gv * ((z - pe[2]) * pe[3]);
            if (!on) v[e] = 0;
          }
        }
        uint16_t* dst = ok && DBG != 3 ? p.c + static_cast<int64_t>(m) * N + c0 : kStoreSink + (lane & 63) * 4;
        *reinterpret_cast<u16x4*>(dst) = v;
      }
    wait_vm<PPW + 8>();  // patch ti + 1 landed; younger: patch ti + 2 (PPW) + the 8 stores
    lds_bar();
  }
  wait_vm<0>();
  lds_bar();
  // ---- statistics: over the 32 pixel lanes of each half, then the 4 pixel waves (fixed order)
#pragma unroll
  for (int off = 1; off < 32; off <<= 1)
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      s1[i] += __shfl_xor(s1[i], off, 64);
      s2[i] += __shfl_xor(s2[i], off, 64);
    }
  float* red = reinterpret_cast<float*>(lds + RED_OFF);  // [2 stats][4 waves][N]
  if (fr == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 32 * i + 8 * q4 + 4 * fh + e, si = 16 * i + 4 * q4 + e;
          red[wave * N + c] = s1[si];
          red[(4 + wave) * N + c] = s2[si];
        }
  }
  __syncthreads();
  if (t < N) {
    p.part[static_cast<int64_t>(mg) * N + t] = (red[t] + red[N + t]) + (red[2 * N + t] + red[3 * N + t]);
    p.part[(static_cast<int64_t>(GM) + mg) * N + t] =
        (red[4 * N + t] + red[5 * N + t]) + (red[6 * N + t] + red[7 * N + t]);
  }
}


// Mode 4: the weight in registers (as mode 3) and a ROLLING row window: a block owns a contiguous
// run of 2-row tiles (whole images top to bottom at ResNet batch sizes), so tile t + 1 shares
// two of its four input rows with tile t and only two new rows are loaded -- the input is read
// once instead of twice (the 2-row tiles of modes 0-3 re-read two halo rows per two output rows),
// and the DMA per tile halves.  LDS: 8 ring row slots + 1 scratch slot per 16-B channel plane,
// each a 64-slot (1 KiB) row: [plane][slot][64 columns] x 16 B.  A new image loads four rows (the
// zero row above it included); a continuing one loads two and sends two dummy loads to the
// scratch slot, so every wave issues the same number of DMAs per tile (counted vmcnt).
template <int W, int EPI, int LA>
__global__ __launch_bounds__(256, 1) void conv3x3_c64v_kernel(const ConvGemmArgs p) {
  static_assert(EPI == 1 || EPI == 3, "forward statistics or data-gradient mask + sums");
  constexpr int C = 64, N = 64, RT = 2, TP = RT * W;
  static_assert(W + 2 <= 64 && TP <= 128, "one 64-column slot row; four 32-pixel waves per tile");
  constexpr int NSLOT = 9, SCRATCH = 8;                // 8 ring slots + scratch
  constexpr int PLANE = NSLOT * 1024;                  // bytes per channel plane
  constexpr int PATCH = 8 * PLANE;
  constexpr int PPW = 8;                               // DMA instructions per wave per tile
  constexpr int PAR_OFF = PATCH;                       // [4][64] floats
  constexpr int PAR4_OFF = PAR_OFF + N * 4 * 4;        // [64][4] floats (EPI 3)
  constexpr int RED_OFF = PAR4_OFF + N * 4 * 4;
  constexpr int LDS_BYTES = RED_OFF + 2 * 4 * N * 4;
  static_assert(LDS_BYTES <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  const uint32_t L0 = lds_addr(lds);

  const ConvGeo& g = p.g;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int fr = lane & 31, fh = lane >> 5;
  const int GM = gridDim.x, mg = blockIdx.x;
  const int tpi = g.OH / RT, ntiles = (p.M / (g.OH * W)) * tpi;
  const int per = (ntiles + GM - 1) / GM;
  const int t0 = mg * per, t1 = min(ntiles, t0 + per);
  const int my_tiles = t1 > t0 ? t1 - t0 : 0;  // block-uniform

  // rows of the tile loaded for tile index q (block-relative): returns the 4 slots of its rows
  // through the running virtual row counter vrow (slot = vrow % 8)
  int vrow = 0;
  // load rows [ih0, ih0 + nrow) of image img into the next ring slots; pieces: plane x row, one
  // 64-lane DMA each (columns -1 .. 62 of the row; zero outside the map); always PPW per wave
  auto issue_rows = [&](int img, int ih0, int nrow, int vbase) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i;          // 0 .. 31: (row j, plane pl)
      const int j = pc >> 3, pl = pc & 7;
      const bool real = j < nrow;
      const int ih = ih0 + j, iw = lane - 1;
      const bool ok = real && static_cast<unsigned>(ih) < static_cast<unsigned>(g.H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(W);
      const uint16_t* src = ok ? p.a + ((static_cast<int64_t>(img) * g.H + ih) * W + iw) * C + pl * 8 : kZeroPatch;
      const int slot = real ? ((vbase + j) & 7) : SCRATCH;
      __builtin_amdgcn_global_load_lds((gptr_t*)src, (lptr_t*)(lds + pl * PLANE + slot * 1024), 16, 0, 0);
    }
  };
  // tile q's (image, first output row)
  auto tile_pos = [&](int q, int& img, int& oh0) {
    const int mt = t0 + q;
    img = mt / tpi;
    oh0 = (mt - img * tpi) * RT;
  };

  // epilogue parameters as [4][64] floats (4 consecutive channels of one parameter = one b128 read)
  for (int c = t; c < N; c += 256) {
    float* pr = reinterpret_cast<float*>(lds + PAR_OFF);
    if constexpr (EPI == 1) {
      pr[c] = p.kshift ? p.kshift[c] : 0.f;
      pr[N + c] = pr[2 * N + c] = pr[3 * N + c] = 0.f;
    } else {
      pr[c] = p.mc[c];
      pr[N + c] = p.mc[N + c];
      pr[2 * N + c] = p.mean[c];
      pr[3 * N + c] = p.invstd[c];
      float* p4 = reinterpret_cast<float*>(lds + PAR4_OFF) + c * 4;
      p4[0] = p.mc[c];
      p4[1] = p.mc[N + c];
      p4[2] = p.mean[c];
      p4[3] = p.invstd[c];
    }
  }
  bf16x8_t wr[36][2];
#pragma unroll
  for (int st = 0; st < 36; ++st)
#pragma unroll
    for (int i = 0; i < 2; ++i)
      wr[st][i] = *reinterpret_cast<const bf16x8_t*>(p.b + static_cast<int64_t>(32 * i + fr) * p.K + (st >> 2) * C +
                                                      16 * (st & 3) + 8 * fh);
  const int px = 32 * wave + fr;
  const bool pvalid = px < TP;
  const int prow = pvalid ? px / W : 0, pcol = pvalid ? px % W : 0;
  float s1[32], s2[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) s1[i] = s2[i] = 0.f;

  // ---- the rows of tile 0 (a new image: four rows), then those of tile 1 in flight
  int slots[4] = {0, 1, 2, 3};   // this tile's four input rows -> ring slots (block-uniform)
  int nslots[4] = {0, 0, 0, 0};  // the next tile's
  int img = 0, oh0 = 0;
  if (my_tiles > 0) {
    tile_pos(0, img, oh0);
    issue_rows(img, oh0 - 1, 4, vrow);
    vrow += 4;
  } else {
    issue_rows(0, 0, 0, 0);
  }
  auto plan_next = [&](int q) {  // issue tile q's new rows (q < my_tiles) and fill nslots
    if (q < my_tiles) {
      int nimg, noh0;
      tile_pos(q, nimg, noh0);
      if (nimg == img && noh0 == oh0 + RT) {  // continuing: rows noh0 + 1, noh0 + 2 are new
        issue_rows(nimg, noh0 + 1, 2, vrow);
        nslots[0] = slots[2];
        nslots[1] = slots[3];
        nslots[2] = vrow & 7;
        nslots[3] = (vrow + 1) & 7;
        vrow += 2;
      } else {  // a new image (or a jump): four rows
        issue_rows(nimg, noh0 - 1, 4, vrow);
#pragma unroll
        for (int j = 0; j < 4; ++j) nslots[j] = (vrow + j) & 7;
        vrow += 4;
      }
    } else {
      issue_rows(0, 0, 0, 0);  // the count stays uniform
    }
  };
  plan_next(1);
  wait_vm<PPW>();
  __syncthreads();

  f32x16 acc[2];
  for (int ti = 0; ti < my_tiles; ++ti) {
    const int m0 = (t0 + ti) * TP;
    u16x4 zr[2][4];
    if constexpr (EPI == 3) {
      const int m = min(m0 + (pvalid ? px : 0), p.M - 1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4)
          zr[i][q4] = *reinterpret_cast<const u16x4*>(p.aux + static_cast<int64_t>(m) * N + 32 * i + 8 * q4 + 4 * fh);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;
    // per-lane bases of the three kernel rows: slot of input row prow + kh, column pcol (tap kw
    // and the plane are immediate offsets)
    uint32_t kb[3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int sl = prow ? slots[kh + 1] : slots[kh];
      kb[kh] = L0 + static_cast<uint32_t>(fh * PLANE + sl * 1024 + pcol * 16);
    }
    constexpr int NB = LA + 1;
    bf16x8_t xb[NB];
    auto fetch = [&](int st, int buf) {
      const int tap = st >> 2, ks = st & 3, kh = tap / 3, kw = tap - kh * 3;
      xb[buf] = ld_b128(kb[kh] + static_cast<uint32_t>(2 * ks * PLANE + kw * 16));
    };
#pragma unroll
    for (int st = 0; st < LA; ++st) fetch(st, st);
#pragma unroll
    for (int st = 0; st < 36; ++st) {
      const int cur = st % NB;
      if (st + LA < 36) {
        fetch(st + LA, (st + LA) % NB);
        wait_lgkm<LA>();
      } else if (st + 2 == 36 && LA >= 2) {
        wait_lgkm<1>();
      } else {
        wait_lgkm<0>();
      }
      tie(xb[cur]);
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wr[st][0], xb[cur], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wr[st][1], xb[cur], acc[1], 0, 0, 0);
    }
    lds_bar();  // every wave is done with this tile's rows
    // the tile after next: its new rows go to slots no tile in flight uses
    {
      int cimg, coh0;
      tile_pos(ti + 1, cimg, coh0);
#pragma unroll
      for (int j = 0; j < 4; ++j) slots[j] = nslots[j];
      img = cimg;
      oh0 = coh0;
      plan_next(ti + 2);
    }
    const int m = m0 + px;
    const bool ok = pvalid && m < p.M;
    const uint32_t parl = L0 + PAR_OFF + static_cast<uint32_t>(4 * fh * 4);  // + (32 i + 8 q4) * 4
    const float* par4 = reinterpret_cast<const float*>(lds + PAR4_OFF);        // EPI 3: [c][4]
    // EPI 1: the 8 groups' shifts in one batch of LDS reads (one wait, not one per value)
    f32x4 sh1[2][4];
    if constexpr (EPI == 1) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) sh1[i][q4] = ld_f4c(parl + static_cast<uint32_t>((32 * i + 8 * q4) * 4));
      wait_lgkm<0>();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const int c0 = 32 * i + 8 * q4 + 4 * fh;
        u16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f32_to_bf16(acc[i][4 * q4 + e]);
        if constexpr (EPI == 1) {
          const f32x4 pa = sh1[i][q4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int si = 16 * i + 4 * q4 + e;
            const float d = ok ? bf16_to_f32(v[e]) - pa[e] : 0.f;
            s1[si] += d;
            s2[si] += d * d;
          }
        } else {  // per channel: [c][4] = mc scale, mc shift, mean, invstd (register budget: one
                  // channel's four at a time)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const f32x4 pe = *reinterpret_cast<const f32x4*>(par4 + (c0 + e) * 4);
            const int si = 16 * i + 4 * q4 + e;
            const float z = bf16_to_f32(zr[i][q4][e]);
            const bool on = ok && z * pe[0] + pe[1] > 0.f;
            const float gv = on ? bf16_to_f32(v[e]) : 0.f;
            s1[si] += gv;
            s2[si] += gv * ((z - pe[2]) * pe[3]);
            if (!on) v[e] = 0;
          }
        }
        uint16_t* dst = ok ? p.c + static_cast<int64_t>(m) * N + c0 : kStoreSink + (lane & 63) * 4;
        *reinterpret_cast<u16x4*>(dst) = v;
      }
    wait_vm<PPW + 8>();  // tile ti + 1's rows landed; younger: tile ti + 2's (PPW) + the 8 stores
    lds_bar();
  }
  wait_vm<0>();
  lds_bar();
#pragma unroll
  for (int off = 1; off < 32; off <<= 1)
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      s1[i] += __shfl_xor(s1[i], off, 64);
      s2[i] += __shfl_xor(s2[i], off, 64);
    }
  float* red = reinterpret_cast<float*>(lds + RED_OFF);
  if (fr == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 32 * i + 8 * q4 + 4 * fh + e, si = 16 * i + 4 * q4 + e;
          red[wave * N + c] = s1[si];
          red[(4 + wave) * N + c] = s2[si];
        }
  }
  __syncthreads();
  if (t < N) {
    p.part[static_cast<int64_t>(mg) * N + t] = (red[t] + red[N + t]) + (red[2 * N + t] + red[3 * N + t]);
    p.part[(static_cast<int64_t>(GM) + mg) * N + t] =
        (red[4 * N + t] + red[5 * N + t]) + (red[6 * N + t] + red[7 * N + t]);
  }
}

}  // namespace

void launch_conv3x3_c64v(const ConvGemmArgs& a, int gm, hipStream_t s) {
  if (a.epi == 1) hipLaunchKernelGGL((conv3x3_c64v_kernel<56, 1, 3>), dim3(gm), dim3(256), 0, s, a);
  else if (a.epi == 3) hipLaunchKernelGGL((conv3x3_c64v_kernel<56, 3, 3>), dim3(gm), dim3(256), 0, s, a);
}

void launch_conv3x3_c64r(const ConvGemmArgs& a, int gm, hipStream_t s) {
  static const int dbg = [] {
    const char* e = std::getenv("PS_AMD_C64R_DBG");
    return e ? std::atoi(e) : 0;
  }();
  if (a.epi == 1) {
    if (dbg == 1) hipLaunchKernelGGL((conv3x3_c64r_kernel<56, 1, 3, 1>), dim3(gm), dim3(256), 0, s, a);
    else if (dbg == 2) hipLaunchKernelGGL((conv3x3_c64r_kernel<56, 1, 3, 2>), dim3(gm), dim3(256), 0, s, a);
    else if (dbg == 3) hipLaunchKernelGGL((conv3x3_c64r_kernel<56, 1, 3, 3>), dim3(gm), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv3x3_c64r_kernel<56, 1, 3>), dim3(gm), dim3(256), 0, s, a);
  } else if (a.epi == 3) {
    hipLaunchKernelGGL((conv3x3_c64r_kernel<56, 3, 3>), dim3(gm), dim3(256), 0, s, a);
  }
}

void launch_conv3x3_c64s(const ConvGemmArgs& a, int gm, hipStream_t s) {
  static const int la = [] {
    const char* e = std::getenv("PS_AMD_C64_LOOKAHEAD");
    return e != nullptr && e[0] == '1' ? 1 : 2;
  }();
  if (la == 1) {
    if (a.epi == 1) hipLaunchKernelGGL((conv3x3_c64s_kernel<56, 1, 1>), dim3(gm), dim3(256), 0, s, a);
    else if (a.epi == 3) hipLaunchKernelGGL((conv3x3_c64s_kernel<56, 3, 1>), dim3(gm), dim3(256), 0, s, a);
  } else {
    if (a.epi == 1) hipLaunchKernelGGL((conv3x3_c64s_kernel<56, 1, 2>), dim3(gm), dim3(256), 0, s, a);
    else if (a.epi == 3) hipLaunchKernelGGL((conv3x3_c64s_kernel<56, 3, 2>), dim3(gm), dim3(256), 0, s, a);
  }
}

}  // namespace psamd
