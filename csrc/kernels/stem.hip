// ResNet stem convolution (7x7, stride 2, pad 3, 64 output channels) on NHWC bf16 input with
// 3 or 4 channels (staged into LDS as 4-channel 8-B pixels), as MFMA implicit GEMMs.  MIOpen reaches ~140-170 TF/s on this layer (C_in = 3
// gives it no K to tile: scripts/probe_convs.py); the whole layer is HBM-bound (output
// 822 MB at batch 512), so the goal is to stream at the memory rate.
//
// Layout trick: with 4 input channels one input pixel is 8 B, so the 7 (kw) x 4 (c) patch
// segment of an output pixel for one kernel row kh is 56 contiguous bytes at an 8-B aligned
// LDS offset.  Packing K as k' = kh*32 + kw*4 + c (kw = 7 and c = 3 slots carry zero weight)
// makes every MFMA A fragment (8 consecutive k') ONE aligned 16-B ds_read_b128 of the staged
// input rows: no im2col buffer exists anywhere.
//
//   forward      z[p, co]   = sum_k' patch[p, k'] wp[co, k']       (M = pixels, N = 64, K = 224)
//   weight grad  dwp[co, k'] = sum_p dz[p, co] patch[p, k']        (M = 64, N = 224, K = pixels)
//
// The weight-gradient kernel reads both operands transposed out of row-major LDS tiles with
// ds_read_b64_tr_b16 (gfx950 hardware transpose read), accumulates a per-block fp32 partial,
// and a two-level fixed-order reduction produces dW (deterministic, no atomics).
#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

namespace {
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kRS = 1056;   // LDS input-row stride (elements): covers (2*127 + 8) * 4 for OW <= 128
constexpr int kSlots = 16;  // input-row ring: rows 2oh-3 .. 2oh+5 (9) never collide mod 16
constexpr int kDzLd = 68;   // LDS dz-tile row stride (elements), 136 B (8-B aligned rows for tr reads)
constexpr int kKp = 224;    // packed K (7 kh x 32)
constexpr int kUnits = kRS / 4;  // 8-B pixel units per LDS input row

__device__ __forceinline__ bf16x8_t as_bf16x8(s16x8 v) { return __builtin_bit_cast(bf16x8_t, v); }

// Workgroup barrier for LDS hand-offs only: __syncthreads()'s release fence also drains vmcnt,
// i.e. waits for every outstanding global STORE of the wave (CDNA4 counts stores in vmcnt) --
// a per-row stall of the output stream in the forward kernel.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Input pixel PAIRS (iw0 = 2j - 4, iw0 + 1) of row ih as two 8-B units of 4 channels (zero
// outside the image): LDS units u = iw + 3, so pair j covers units 2j - 1 and 2j.
// cin = 4: one 16-B load; cin = 3 (plain NHWC RGB, no padding copy): one 12-B load when the
// pair is 4-B aligned, else 2-B loads.
constexpr int kPairs = kUnits / 2 + 1;

__device__ __forceinline__ uint4 load_pair(const uint16_t* __restrict__ x, int n, int ih, int j, int H, int W,
                                           int cin) {
  const int iw0 = 2 * j - 4;
  if ((W & 1) == 0) {
    // even W: a pair is wholly inside or outside the image, and 3-channel pairs are 4-B aligned.
    // Branch-free (clamped address + select), so unrolled loads stay in flight together instead
    // of draining vmcnt at every divergent join.
    const bool ok = ih >= 0 && ih < H && iw0 >= 0 && iw0 < W;
    const int64_t pix = ok ? (static_cast<int64_t>(n) * H + ih) * W + iw0 : 0;
    if (cin == 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + pix * 4);
      return ok ? v : make_uint4(0u, 0u, 0u, 0u);
    }
    const uint3 d = *reinterpret_cast<const uint3*>(x + pix * 3);  // c0 c1 | c2 c0' | c1' c2'
    return ok ? make_uint4(d.x, d.y & 0xffffu, (d.y >> 16) | (d.z << 16), d.z >> 16) : make_uint4(0u, 0u, 0u, 0u);
  }
  uint4 r = make_uint4(0u, 0u, 0u, 0u);  // odd W: guarded per-pixel path
  if (ih < 0 || ih >= H || iw0 + 1 < 0 || iw0 >= W) return r;
  const int64_t pix = (static_cast<int64_t>(n) * H + ih) * W + iw0;
  if (cin == 4) {
    if (iw0 >= 0) {
      const uint2 a = *reinterpret_cast<const uint2*>(x + pix * 4);
      r.x = a.x, r.y = a.y;
    }
    if (iw0 + 1 < W) {
      const uint2 b = *reinterpret_cast<const uint2*>(x + (pix + 1) * 4);
      r.z = b.x, r.w = b.y;
    }
    return r;
  }
  const uint16_t* q = x + pix * 3;
  if (iw0 >= 0) r.x = q[0] | (uint32_t(q[1]) << 16), r.y = q[2];
  if (iw0 + 1 < W) r.z = q[3] | (uint32_t(q[4]) << 16), r.w = q[5];
  return r;
}

__device__ __forceinline__ void store_pair(uint16_t* lds_in, int ih, int j, uint4 v) {
  uint16_t* row = lds_in + (ih & (kSlots - 1)) * kRS;
  const int u0 = 2 * j - 1;
  if (u0 >= 0) *reinterpret_cast<uint2*>(row + u0 * 4) = make_uint2(v.x, v.y);
  if (u0 + 1 < kUnits) *reinterpret_cast<uint2*>(row + (u0 + 1) * 4) = make_uint2(v.z, v.w);
}

// Register prefetch of the two input rows a block needs next (rows ih0, ih0 + 1): 2 * kPairs
// pairs over NT threads (lane index t), all loads issued before any is consumed.
template <int NT>
struct RowPrefetch {
  static constexpr int kIt = (2 * kPairs + NT - 1) / NT;
  uint4 v[kIt];
  __device__ __forceinline__ void load(const uint16_t* __restrict__ x, int t, int n, int ih0, int H, int W, int cin) {
#pragma unroll
    for (int k = 0; k < kIt; ++k) {
      const int i = t + k * NT;
      v[k] = make_uint4(0u, 0u, 0u, 0u);
      if (i < 2 * kPairs) v[k] = load_pair(x, n, ih0 + (i >= kPairs), i % kPairs, H, W, cin);
    }
  }
  __device__ __forceinline__ void store(uint16_t* lds_in, int t, int ih0) const {
#pragma unroll
    for (int k = 0; k < kIt; ++k) {
      const int i = t + k * NT;
      if (i < 2 * kPairs) store_pair(lds_in, ih0 + (i >= kPairs), i % kPairs, v[k]);
    }
  }
};

// Prologue: input rows 2*oh - 3 .. 2*oh + 3 into their ring slots (loads batched per thread).
__device__ __forceinline__ void stage_window(const uint16_t* __restrict__ x, uint16_t* lds_in, int n, int oh, int H,
                                             int W, int cin) {
  constexpr int kIt = (7 * kPairs + 255) / 256;  // blockDim >= 256
  uint4 v[kIt];
  const int ih0 = 2 * oh - 3;
  const int nt = blockDim.x;
#pragma unroll
  for (int k = 0; k < kIt; ++k) {
    const int i = threadIdx.x + k * nt;
    v[k] = make_uint4(0u, 0u, 0u, 0u);
    if (i < 7 * kPairs) v[k] = load_pair(x, n, ih0 + i / kPairs, i % kPairs, H, W, cin);
  }
#pragma unroll
  for (int k = 0; k < kIt; ++k) {
    const int i = threadIdx.x + k * nt;
    if (i < 7 * kPairs) store_pair(lds_in, ih0 + i / kPairs, i % kPairs, v[k]);
  }
}

// Forward output staging (OW <= 112): pixel p of output row oh goes to the ring slots that row
// oh's MFMAs (input rows 2oh-3 .. 2oh+3) and its prefetch (2oh+4, 2oh+5) leave free -- slots
// 2oh+6 .. 2oh+12, 16 pixels x 128 B each -- so the row leaves as whole 128-B pixel rows.
__device__ __forceinline__ uint16_t* stage_at(uint16_t* lds_in, int oh, int p) {
  return lds_in + ((2 * oh + 6 + (p >> 4)) & (kSlots - 1)) * kRS + (p & 15) * 64;
}
}  // namespace

// grid = N * splits blocks of 256 threads; block b: image b / splits, output rows
// [chunk*rpb, +rpb).  wp: [64][224] packed bf16.  Input rows slide through an LDS ring (2 new
// rows per output row).  Per row: issue the next row's input loads, run all MFMAs into
// registers, publish the prefetched rows to LDS, THEN issue this row's output stores and pass
// an LDS-only barrier -- CDNA4's vmcnt counts stores too, so waiting for the prefetch before
// the stores are issued keeps the output stream from being drained every row.
// Wave w owns output channels [16w, 16w + 16) of every pixel tile of the row: its weight
// fragments are 28 VGPRs (a 2 x 2 wave grid held 56) and the kernel fits 128 VGPRs, i.e. four
// blocks per CU instead of two -- the row loop is latency-bound, so rows in flight per CU set
// the rate (0.79 ms -> see profiles/r4_stem_fwd_occupancy_ab.txt at bs1024).  Each wave's
// accumulators hold 32 B of every pixel (its 16 channels); for OW <= 112 they pass through free
// LDS ring slots (stage_at) so every global store writes whole 128-B pixel rows instead of 32-B
// quarters that four waves complete at different times.
// MT > 0: OW == 16 MT exactly (ResNet's 112: MT = 7), the tile loop and its guards compile away --
// the runtime-mtiles version spends SGPRs on per-tile exec masks (24 spilled to VGPR lanes).
template <int MT>
__global__ __launch_bounds__(256, 4) void stem_conv_fwd_kernel(const uint16_t* __restrict__ x,
                                                               const uint16_t* __restrict__ wp,
                                                               uint16_t* __restrict__ z, int N, int H, int W, int OH,
                                                               int OW, int splits, int rpb, int cin,
                                                               const float* __restrict__ kshift,
                                                               float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) uint16_t lds_in[kSlots * kRS];
  const int n = blockIdx.x / splits, chunk = blockIdx.x - n * splits;
  const int oh0 = chunk * rpb, oh1 = min(OH, oh0 + rpb);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const int c0 = 16 * wave + 4 * g;  // this lane's 4 output channels c0 .. c0 + 3
  // fused BN statistics from the accumulators (combined across the 16 pixel lanes at the end)
  float s1[4], s2[4], ks[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    s1[r] = s2[r] = 0.f;
    ks[r] = part ? kshift[c0 + r] : 0.f;
  }
  bf16x8_t bw[7];
#pragma unroll
  for (int kh = 0; kh < 7; ++kh) bw[kh] = *reinterpret_cast<const bf16x8_t*>(wp + (16 * wave + fr) * kKp + kh * 32 + 8 * g);
  if (oh0 < oh1) stage_window(x, lds_in, n, oh0, H, W, cin);  // block-uniform
  __syncthreads();
  const int mtiles = MT > 0 ? MT : (OW + 15) / 16;  // <= 8
  const bool staged = MT > 0 || OW <= 112;         // block-uniform: 7 free ring slots hold the row
  for (int oh = oh0; oh < oh1; ++oh) {
    RowPrefetch<256> pf;
    const bool more = oh + 1 < oh1;
    if (more) pf.load(x, threadIdx.x, n, 2 * oh + 4, H, W, cin);
    f32x4v acc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      acc[t] = f32x4v{0.f, 0.f, 0.f, 0.f};
      if (t < mtiles) {  // block-uniform
        const int ow = 16 * t + fr;  // pixels >= OW read finite staged data and are never stored
#pragma unroll
        for (int kh = 0; kh < 7; ++kh) {
          const int slot = (2 * oh - 3 + kh) & (kSlots - 1);
          const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(lds_in + slot * kRS + 8 * ow + 8 * g);
          // D[co][pixel] = W . patch^T: the lane ends up with 4 consecutive channels of one pixel
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[kh], a, acc[t], 0, 0, 0);
        }
      }
    }
    if (more) pf.store(lds_in, threadIdx.x, 2 * oh + 4);  // ring slots not read by rows oh-1, oh
    uint16_t* zo = z + (static_cast<int64_t>(n) * OH + oh) * OW * 64;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int ow = 16 * t + fr;
      if (MT > 0 ? t < MT : (t < mtiles && ow < OW)) {
        // C layout: row (channel) = 16 wave + 4 g + r, col (pixel) = fr -> one 8-B store per tile
        uint16_t h[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          h[r] = f32_to_bf16(acc[t][r]);
          if (part) {  // statistics of the bf16 values stored
            const float d = bf16_to_f32(h[r]) - ks[r];
            s1[r] += d;
            s2[r] += d * d;
          }
        }
        const uint2 v = make_uint2(h[0] | (uint32_t(h[1]) << 16), h[2] | (uint32_t(h[3]) << 16));
        if (staged) {  // 8-B unit u = c0 / 4 of pixel ow, XOR-swizzled by the pixel's low 4 bits
          *reinterpret_cast<uint2*>(stage_at(lds_in, oh, ow) + ((c0 >> 2) ^ (ow & 15)) * 4) = v;
        } else {
          *reinterpret_cast<uint2*>(zo + ow * 64 + c0) = v;
        }
      }
    }
    lds_barrier();
    if (staged) {
      // whole 128-B pixel rows: thread -> 16-B chunk k of pixel p, consecutive lanes consecutive chunks
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = threadIdx.x + 256 * i, p = c >> 3, k = c & 7;
        if (p < OW) {
          const int s = p & 15;
          uint4 v = *reinterpret_cast<const uint4*>(stage_at(lds_in, oh, p) + ((2 * k) ^ (s & 14)) * 4);
          if (s & 1) v = make_uint4(v.z, v.w, v.x, v.y);
          *reinterpret_cast<uint4*>(zo + p * 64 + 8 * k) = v;
        }
      }
      lds_barrier();  // the staging slots are the next row's prefetch / staging targets
    }
  }
  if (part) {  // fixed-order combine over the 16 pixel lanes (xor shuffles); waves own disjoint channels
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        s1[r] += __shfl_xor(s1[r], off, 64);
        s2[r] += __shfl_xor(s2[r], off, 64);
      }
    if (fr == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        part[static_cast<int64_t>(blockIdx.x) * 64 + c0 + r] = s1[r];
        part[(static_cast<int64_t>(gridDim.x) + blockIdx.x) * 64 + c0 + r] = s2[r];
      }
    }
  }
}

// dz row -> LDS [128 pixels][kDzLd] (pixels >= OW zero): 4 x 16-B loads per thread.
struct DzPrefetch {
  u16x8 v[4];
  __device__ __forceinline__ void load(const uint16_t* __restrict__ dzr, int OW) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = threadIdx.x + k * 256, pix = c >> 3, ch = c & 7;
      v[k] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (pix < OW) v[k] = *reinterpret_cast<const u16x8*>(dzr + pix * 64 + ch * 8);
    }
  }
  __device__ __forceinline__ void store(uint16_t* lds_dz) const {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = threadIdx.x + k * 256, pix = c >> 3, ch = c & 7;
      uint16_t* d = lds_dz + pix * kDzLd + ch * 8;  // 136-B rows: 8-B aligned stores
      const u16x8 u = v[k];
      *reinterpret_cast<uint2*>(d) = make_uint2(u[0] | (uint32_t(u[1]) << 16), u[2] | (uint32_t(u[3]) << 16));
      *reinterpret_cast<uint2*>(d + 4) = make_uint2(u[4] | (uint32_t(u[5]) << 16), u[6] | (uint32_t(u[7]) << 16));
    }
  }
};

// FUSED: the stem's BN-backward APPLY pass (pool.hip pool_bn_bwd_kernel<true>) computed per dz
// row inside the weight-gradient kernel, so the full-resolution dz is never written nor re-read:
//   dz = ca g' + cb z + cc,   g' = bf16(g) * relu'(z sc + sh),   g = the max-pool scatter of dy
// Thread t owns 16-B channel group ch = t & 7 of the pixel PAIRS pp = (t >> 3) + 32 k (k = 0, 1):
// pixels 2 pp, 2 pp + 1 of z row 2 a + dh take their gradient from the pooled windows (a + i,
// pp + j), i <= dh, j <= dw (argmax code (dh + 1 - 2 i) 3 + (dw + 1 - 2 j)).  Row 2 a + 1 needs
// pooled rows a and a + 1, row 2 a + 2 only a + 1: the windows of one pooled row are loaded per
// TWO z rows and carried in registers.
struct PoolWin {
  u16x8 g[2][2];      // [pair k][j] pooled gradient, 8 channels
  uint64_t c[2][2];   // [pair k][j] argmax codes (8 x 1 B); all-ones = no window
};

__device__ __forceinline__ void load_win(PoolWin& w, const uint16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                         int n, int pa, int OHp, int OWp) {
  const int ch = threadIdx.x & 7;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int pp = (threadIdx.x >> 3) + 32 * k;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool ok = pa < OHp && pp + j < OWp;
      const int64_t o = ok ? ((static_cast<int64_t>(n) * OHp + pa) * OWp + pp + j) * 64 + ch * 8 : 0;
      const u16x8 g = *reinterpret_cast<const u16x8*>(dy + o);
      const uint64_t c = *reinterpret_cast<const uint64_t*>(idx + o);
      w.g[k][j] = ok ? g : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      w.c[k][j] = ok ? c : ~uint64_t(0);
    }
  }
}

struct ZPair {
  u16x8 v[2][2];  // [pair k][pixel d]
  __device__ __forceinline__ void load(const uint16_t* __restrict__ zr, int OW) {
    const int ch = threadIdx.x & 7;
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const int px = 2 * ((threadIdx.x >> 3) + 32 * k) + d;
        v[k][d] = *reinterpret_cast<const u16x8*>(zr + (px < OW ? px : 0) * 64 + ch * 8);
      }
  }
};

// dz of z row r (dh = r & 1) into the LDS dz tile: i = 0 windows from `lo` (pooled row r >> 1),
// i = 1 windows (dh = 1 only) from `hi` (pooled row (r >> 1) + 1)
// cf: LDS [5][64] floats sc | sh | ca | cb | cc (read per row: in registers they cost the kernel
// its second wave per SIMD)
__device__ __forceinline__ void dz_row_to_lds(uint16_t* lds_dz, const ZPair& z, const PoolWin& lo, const PoolWin& hi,
                                              int dh, int OW, const float* cf) {
  const int ch = threadIdx.x & 7;
  float sc[8], sh[8], A[8], B[8], Cc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = cf[ch * 8 + e];
    sh[e] = cf[64 + ch * 8 + e];
    A[e] = cf[128 + ch * 8 + e];
    B[e] = cf[192 + ch * 8 + e];
    Cc[e] = cf[256 + ch * 8 + e];
  }
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const int px = 2 * ((threadIdx.x >> 3) + 32 * k) + d;
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (j > d) continue;  // compile-time
          if (i == 1 && dh == 0) continue;
          const PoolWin& w = i ? hi : lo;
          const uint8_t code = static_cast<uint8_t>((dh + 1 - 2 * i) * 3 + (d + 1 - 2 * j));
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (static_cast<uint8_t>(w.c[k][j] >> (8 * e)) == code) acc[e] += bf16_to_f32(w.g[k][j][e]);
        }
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float zf = bf16_to_f32(z.v[k][d][e]);
        const float g = zf * sc[e] + sh[e] > 0.f ? bf16_to_f32(f32_to_bf16(acc[e])) : 0.f;
        o[e] = f32_to_bf16(A[e] * g + B[e] * zf + Cc[e]);
      }
      // pixels >= OW (finite: z read at pixel 0) are zeroed by one select per word AFTER the math:
      // a per-element `px < OW ? ... : 0` compiled to 8 divergent branches per pixel
      const uint32_t keep = px < OW ? ~0u : 0u;
      uint16_t* dst = lds_dz + px * kDzLd + ch * 8;
      *reinterpret_cast<uint2*>(dst) =
          make_uint2((o[0] | (uint32_t(o[1]) << 16)) & keep, (o[2] | (uint32_t(o[3]) << 16)) & keep);
      *reinterpret_cast<uint2*>(dst + 4) =
          make_uint2((o[4] | (uint32_t(o[5]) << 16)) & keep, (o[6] | (uint32_t(o[7]) << 16)) & keep);
    }
}

struct StemBwdFuse {
  const uint16_t* dy;  // [N, OH/2, OW/2, 64] pooled gradient
  const uint8_t* idx;  // its argmax codes
  const float* mc;     // [2 * 64] bn scale | shift (the ReLU mask)
  const float* coef;   // [3 * 64] ca | cb | cc
};

// grid = N * splits blocks (as the forward); each accumulates its output rows into
// part[b][64][224] (fp32).  dz: the stem BN's input gradient, or (FUSED) z, the BN input.
template <bool FUSED>
__global__ __launch_bounds__(256, 2) void stem_conv_wrw_kernel(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ dz,
                                                            float* __restrict__ part, int N, int H, int W, int OH,
                                                            int OW, int splits, int rpb, int cin, StemBwdFuse fz) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[kSlots * kRS + 2 * 128 * kDzLd + (FUSED ? 5 * 64 * 2 : 0)];
  uint16_t* lds_in = lds;
  float* cf = reinterpret_cast<float*>(lds + kSlots * kRS + 2 * 128 * kDzLd);  // FUSED: [5][64]
  const int n = blockIdx.x / splits, chunk = blockIdx.x - n * splits;
  const int oh0 = chunk * rpb, oh1 = min(OH, oh0 + rpb);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  // this wave's N-tiles (16 packed-k' columns each): w, w+4, w+8, w+12 (< 14)
  const int nnt = wave < 2 ? 4 : 3;
  f32x4v acc[4][4];  // [mt][j]
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[mt][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
  // FUSED: the BN coefficients into LDS, the carried pooled windows
  PoolWin wlo, whi;
  const int OHp = OH / 2, OWp = OW / 2;
  if constexpr (FUSED) {
    for (int i = threadIdx.x; i < 5 * 64; i += 256) cf[i] = i < 128 ? fz.mc[i] : fz.coef[i - 128];
    __syncthreads();
  }
  if (oh0 < oh1) {  // block-uniform
    stage_window(x, lds_in, n, oh0, H, W, cin);
    if constexpr (FUSED) {
      ZPair z0;
      z0.load(dz + (static_cast<int64_t>(n) * OH + oh0) * OW * 64, OW);
      load_win(wlo, fz.dy, fz.idx, n, oh0 >> 1, OHp, OWp);
      if (oh0 & 1) load_win(whi, fz.dy, fz.idx, n, (oh0 >> 1) + 1, OHp, OWp);
      dz_row_to_lds(lds + kSlots * kRS, z0, wlo, whi, oh0 & 1, OW, cf);
      if (oh0 & 1) wlo = whi;
    } else {
      DzPrefetch d0;
      d0.load(dz + (static_cast<int64_t>(n) * OH + oh0) * OW * 64, OW);
      d0.store(lds + kSlots * kRS);
    }
    __syncthreads();
    for (int oh = oh0; oh < oh1; ++oh) {
      const bool more = oh + 1 < oh1;
      RowPrefetch<256> pf;
      DzPrefetch pd;
      ZPair pz;
      const bool odd = (oh + 1) & 1;
      if (more) {
        pf.load(x, threadIdx.x, n, 2 * oh + 4, H, W, cin);
        if constexpr (FUSED) {
          pz.load(dz + (static_cast<int64_t>(n) * OH + oh + 1) * OW * 64, OW);
          if (odd) load_win(whi, fz.dy, fz.idx, n, ((oh + 1) >> 1) + 1, OHp, OWp);
        } else {
          pd.load(dz + (static_cast<int64_t>(n) * OH + oh + 1) * OW * 64, OW);
        }
      }
      const uint16_t* lds_dz = lds + kSlots * kRS + ((oh - oh0) & 1) * 128 * kDzLd;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int pix0 = 32 * s + 8 * g + q;  // tr-read row of this lane (and +4 for the second half)
        bf16x8_t a[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(lds_dz + pix0 * kDzLd + 16 * mt + 4 * p));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(lds_dz + (pix0 + 4) * kDzLd + 16 * mt + 4 * p));
          a[mt] = as_bf16x8(s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j < nnt) {  // wave-uniform
            const int kp = 16 * (wave + 4 * j) + 4 * p;  // packed k' of this lane's 4 columns
            const int kh = kp >> 5, kw = (kp & 31) >> 2;
            const uint16_t* base = lds_in + ((2 * oh - 3 + kh) & (kSlots - 1)) * kRS + kw * 4;
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + 8 * pix0));
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + 8 * (pix0 + 4)));
            const bf16x8_t b = as_bf16x8(s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
              acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b, acc[mt][j], 0, 0, 0);
          }
        }
      }
      if (more) {
        pf.store(lds_in, threadIdx.x, 2 * oh + 4);
        uint16_t* nxt = lds + kSlots * kRS + ((oh + 1 - oh0) & 1) * 128 * kDzLd;
        if constexpr (FUSED) {
          dz_row_to_lds(nxt, pz, wlo, whi, odd ? 1 : 0, OW, cf);
          if (odd) wlo = whi;  // pooled row (oh + 1) / 2 + 1 serves the next (even) row as i = 0
        } else {
          pd.store(nxt);
        }
      }
      __syncthreads();
    }
  }
  // C layout: row (co) = 16*mt + 4*g + r, col (k') = 16*nt + (lane & 15)
  float* pb = part + static_cast<int64_t>(blockIdx.x) * 64 * kKp;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j < nnt) {
      const int col = 16 * (wave + 4 * j) + i16;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) pb[(16 * mt + 4 * g + r) * kKp + col] = acc[mt][j][r];
    }
  }
}

// out[e] = sum_{b in group y} part[b][e]; fixed order.  grid (ceil(E/256), groups)
__global__ __launch_bounds__(256) void stem_wrw_reduce_kernel(const float* __restrict__ part, int nblk, int per,
                                                              float* __restrict__ out) {
  constexpr int E = 64 * kKp;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  const int b0 = blockIdx.y * per, b1 = min(nblk, b0 + per);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int b = b0;
  for (; b + 3 < b1; b += 4) {
    s0 += part[static_cast<int64_t>(b) * E + e];
    s1 += part[static_cast<int64_t>(b + 1) * E + e];
    s2 += part[static_cast<int64_t>(b + 2) * E + e];
    s3 += part[static_cast<int64_t>(b + 3) * E + e];
  }
  for (; b < b1; ++b) s0 += part[static_cast<int64_t>(b) * E + e];
  out[static_cast<int64_t>(blockIdx.y) * E + e] = (s0 + s1) + (s2 + s3);
}

namespace {
constexpr int kFwdSplits = 4;  // blocks per image (forward): N*4 blocks, ~28 rows each at OH = 112
constexpr int kWrwSplits = 2;  // blocks per image (weight grad): fewer fp32 partials to reduce
}  // namespace

int stem_fwd_blocks(int N) { return N * kFwdSplits; }

void launch_stem_conv_fwd(const uint16_t* x, int cin, const uint16_t* wp, uint16_t* z, int N, int H, int W, int OH,
                          int OW, const float* kshift, float* part, hipStream_t s) {
  if (N <= 0 || OH <= 0) return;
  const int rpb = (OH + kFwdSplits - 1) / kFwdSplits;
  if (OW == 112)
    hipLaunchKernelGGL(stem_conv_fwd_kernel<7>, dim3(N * kFwdSplits), dim3(256), 0, s, x, wp, z, N, H, W, OH, OW,
                       kFwdSplits, rpb, cin, kshift, part);
  else
    hipLaunchKernelGGL(stem_conv_fwd_kernel<0>, dim3(N * kFwdSplits), dim3(256), 0, s, x, wp, z, N, H, W, OH, OW,
                     kFwdSplits, rpb, cin, kshift, part);
}

int stem_wrw_blocks(int N, int OH) { return N * kWrwSplits; }

// ws: [nblk * 64 * 224 + 32 * 64 * 224] floats; dwp: [64 * 224] floats
void launch_stem_conv_wrw(const uint16_t* x, int cin, const uint16_t* dz, float* ws, float* dwp, int N, int H, int W,
                          int OH, int OW, hipStream_t s, const uint16_t* pool_dy, const uint8_t* pool_idx,
                          const float* mc, const float* coef) {
  if (N <= 0 || OH <= 0) return;
  const int nblk = stem_wrw_blocks(N, OH);
  const int rpb = (OH + kWrwSplits - 1) / kWrwSplits;
  const StemBwdFuse fz{pool_dy, pool_idx, mc, coef};
  if (pool_dy != nullptr)
    hipLaunchKernelGGL(stem_conv_wrw_kernel<true>, dim3(nblk), dim3(256), 0, s, x, dz, ws, N, H, W, OH, OW, kWrwSplits,
                       rpb, cin, fz);
  else
    hipLaunchKernelGGL(stem_conv_wrw_kernel<false>, dim3(nblk), dim3(256), 0, s, x, dz, ws, N, H, W, OH, OW, kWrwSplits,
                       rpb, cin, fz);
  constexpr int E = 64 * kKp;
  const int groups = 32;
  const int per = (nblk + groups - 1) / groups;
  float* mid = ws + static_cast<int64_t>(nblk) * E;
  hipLaunchKernelGGL(stem_wrw_reduce_kernel, dim3(E / 256, groups), dim3(256), 0, s, ws, nblk, per, mid);
  hipLaunchKernelGGL(stem_wrw_reduce_kernel, dim3(E / 256, 1), dim3(256), 0, s, mid, groups, groups, dwp);
}

}  // namespace psamd
