// NHWC (channels_last) bf16 max pooling with an optional fused BatchNorm-apply + ReLU
// prologue, for the ResNet-50 stem (conv 7x7 -> BN -> ReLU -> maxpool 3x3/2): the BN output
// is never written to HBM -- the pool reads the conv output z, computes relu(z*scale+shift)
// per tap and keeps the max.  The window argmax is stored as one byte per output element
// (tap index kh*k+kw, k <= 15), 1/8 of the int64 indices torch keeps.
//
// Backward is a gather over the (at most ceil(k/s)^2) output windows that cover each input
// pixel: every dx element is written exactly once (no atomics, deterministic), 8 channels
// (16 B) per thread.
//
// Reference counterpart: layer/PoolingLayer.java:62-101 (forward, argmax multimap) and
// :116-134 (backward scatter); the reference CNN path keeps its own NCHW kernel in ref_ops.hip.
#include <algorithm>

#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

// IDX: 32-bit index math when the element count allows it (64-bit div/mod is a long
// instruction sequence on CDNA and dominated these HBM-light, address-heavy kernels)
// LCV >= 0 (C / 8 a power of two, 2^LCV): one output row (n, oh) per block iteration, its
// (ow, channel-group) elements over the threads by shift / mask -- no per-element division (the
// generic mapping's three runtime-divisor div/mods were most of these kernels' instructions).
// K3 (with BN, k = 3): the nine window taps are loaded together (clamped in bounds, flagged) before
// any is used -- the runtime-k loop with its boundary `continue`s issued one tap load per
// dependent step (the ResNet stem pool ran at ~4.2 TB/s)
template <bool BN, typename IDX, bool K3 = false>
__global__ __launch_bounds__(256) void maxpool_nhwc_fwd_kernel(const uint16_t* __restrict__ x,
                                                               const float* __restrict__ coef,
                                                               uint16_t* __restrict__ y, uint8_t* __restrict__ idx,
                                                               int N, int H, int W, int C, int OH, int OW, int k,
                                                               int s, int p, int lcv) {
  const IDX cv = C / 8;
  auto one = [&](IDX v, int n, int oh, int ow, int c8) {
    float sc[8], sh[8];
    if constexpr (BN) {
      load8(coef, c8 * 8, sc);
      load8(coef + C, c8 * 8, sh);
    }
    const int h0 = oh * s - p, w0 = ow * s - p;
    if constexpr (BN && K3) {
      u16x8 a[9];
      unsigned okm = 0;
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        const int h = h0 + q / 3, w = w0 + q % 3;
        const bool ok = h >= 0 && h < H && w >= 0 && w < W;
        okm |= (ok ? 1u : 0u) << q;
        a[q] = *reinterpret_cast<const u16x8*>(
            x + (ok ? ((static_cast<int64_t>(n) * H + h) * W + w) * C + c8 * 8 : 0));
      }
      unsigned key[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // (the same keys as the generic path below)
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        if (!((okm >> q) & 1u)) continue;
        const unsigned tag = 255u - static_cast<unsigned>(q);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = bf16_to_f32(a[q][j]) * sc[j] + sh[j];
          t = t > 0.f ? t : 0.f;
          const unsigned kj = (static_cast<unsigned>(f32_to_bf16(t)) << 8) | tag;
          key[j] = kj > key[j] ? kj : key[j];
        }
      }
      u16x8 yv;
      uint64_t packed = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        yv[j] = static_cast<uint16_t>(key[j] >> 8);
        packed |= static_cast<uint64_t>(255u - (key[j] & 255u)) << (8 * j);
      }
      *reinterpret_cast<u16x8*>(y + static_cast<int64_t>(v) * 8) = yv;
      *reinterpret_cast<uint64_t*>(idx + static_cast<int64_t>(v) * 8) = packed;
      return;
    } else if constexpr (BN) {
      // relu(bn(x)) rounded to bf16 is >= +0, so its bits order like the values: the window max
      // and its first argmax are one unsigned max over key = bits << 8 | (255 - tap) per element
      // (ties keep the lowest tap, as the unfused path's first-max-wins scan does)
      unsigned key[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int kh = 0; kh < k; ++kh) {
        const int h = h0 + kh;
        if (h < 0 || h >= H) continue;
        for (int kw = 0; kw < k; ++kw) {
          const int w = w0 + kw;
          if (w < 0 || w >= W) continue;
          const u16x8 a = *reinterpret_cast<const u16x8*>(x + ((static_cast<int64_t>(n) * H + h) * W + w) * C + c8 * 8);
          const unsigned tag = 255u - static_cast<unsigned>(kh * k + kw);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float t = bf16_to_f32(a[j]) * sc[j] + sh[j];
            t = t > 0.f ? t : 0.f;
            const unsigned kj = (static_cast<unsigned>(f32_to_bf16(t)) << 8) | tag;
            key[j] = kj > key[j] ? kj : key[j];
          }
        }
      }
      u16x8 yv;
      uint64_t packed = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        yv[j] = static_cast<uint16_t>(key[j] >> 8);
        packed |= static_cast<uint64_t>(255u - (key[j] & 255u)) << (8 * j);
      }
      *reinterpret_cast<u16x8*>(y + static_cast<int64_t>(v) * 8) = yv;
      *reinterpret_cast<uint64_t*>(idx + static_cast<int64_t>(v) * 8) = packed;
      return;
    }
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    for (int kh = 0; kh < k; ++kh) {
      const int h = h0 + kh;
      if (h < 0 || h >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int w = w0 + kw;
        if (w < 0 || w >= W) continue;
        float a[8];
        load8(x, ((static_cast<int64_t>(n) * H + h) * W + w) * C + c8 * 8, a);
        const uint8_t code = static_cast<uint8_t>(kh * k + kw);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float t = a[j];
          if (t > best[j] || (t != t && best[j] == best[j])) {  // first max wins; NaN propagates
            best[j] = t;
            bi[j] = code;
          }
        }
      }
    }
    store8(y, static_cast<int64_t>(v) * 8, best);
    uint64_t packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) packed |= static_cast<uint64_t>(bi[j]) << (8 * j);
    *reinterpret_cast<uint64_t*>(idx + static_cast<int64_t>(v) * 8) = packed;
  };
  if (lcv >= 0) {
    const int per_row = OW << lcv;
    for (int row = blockIdx.x; row < N * OH; row += gridDim.x) {
      const int n = row / OH, oh = row - n * OH;
      for (int e = threadIdx.x; e < per_row; e += blockDim.x)
        one(static_cast<IDX>(row) * per_row + e, n, oh, e >> lcv, e & ((1 << lcv) - 1));
    }
    return;
  }
  const IDX total = static_cast<IDX>(N) * OH * OW * cv;
  const IDX stride = static_cast<IDX>(gridDim.x) * blockDim.x;
  for (IDX v = static_cast<IDX>(blockIdx.x) * blockDim.x + threadIdx.x; v < total; v += stride) {
    const int c8 = static_cast<int>(v % cv);
    IDX r = v / cv;
    const int ow = static_cast<int>(r % OW);
    r /= OW;
    const int oh = static_cast<int>(r % OH);
    one(v, static_cast<int>(r / OH), oh, ow, c8);
  }
}

// S2K3: k = 3, s = 2 (the ResNet stem pool) -- the window bounds become shifts instead of four
// integer divisions by a runtime stride
template <typename IDX, bool S2K3>
__global__ __launch_bounds__(256) void maxpool_nhwc_bwd_kernel(const uint16_t* __restrict__ dy,
                                                               const uint8_t* __restrict__ idx,
                                                               uint16_t* __restrict__ dx, int N, int H, int W, int C,
                                                               int OH, int OW, int k, int s, int p, int lcv) {
  if constexpr (S2K3) {
    k = 3;
    s = 2;
  }
  const IDX cv = C / 8;
  auto one = [&](IDX v, int n, int h, int w, int c8) {
    // output windows covering (h, w): oh*s - p <= h <= oh*s - p + k - 1
    const int hp = h + p, wp = w + p;
    int oh_lo, oh_hi, ow_lo, ow_hi;
    if constexpr (S2K3) {
      oh_lo = hp - 2 > 0 ? (hp - 1) >> 1 : 0;
      oh_hi = min(OH - 1, hp >> 1);
      ow_lo = wp - 2 > 0 ? (wp - 1) >> 1 : 0;
      ow_hi = min(OW - 1, wp >> 1);
    } else {
      oh_lo = hp - k + 1 > 0 ? (hp - k + 1 + s - 1) / s : 0;
      oh_hi = min(OH - 1, hp / s);
      ow_lo = wp - k + 1 > 0 ? (wp - k + 1 + s - 1) / s : 0;
      ow_hi = min(OW - 1, wp / s);
    }
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if constexpr (S2K3) {
      // at most 2 x 2 covering windows: issue all four (idx, dy) reads (clamped in bounds) before
      // any is used, then accumulate the valid ones in the generic loop's (oh, ow) order
      uint64_t pk[4];
      u16x8 gv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int oh = min(oh_lo + (q >> 1), OH - 1), ow = min(ow_lo + (q & 1), OW - 1);
        const int64_t o = ((static_cast<int64_t>(n) * OH + oh) * OW + ow) * C + c8 * 8;
        pk[q] = *reinterpret_cast<const uint64_t*>(idx + o);
        gv[q] = *reinterpret_cast<const u16x8*>(dy + o);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int oh = oh_lo + (q >> 1), ow = ow_lo + (q & 1);
        if (oh > oh_hi || ow > ow_hi) continue;
        const uint8_t code = static_cast<uint8_t>((hp - oh * 2) * 3 + (wp - ow * 2));
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (static_cast<uint8_t>(pk[q] >> (8 * j)) == code) acc[j] += bf16_to_f32(gv[q][j]);
      }
      store8(dx, static_cast<int64_t>(v) * 8, acc);
      return;
    }
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const uint8_t code = static_cast<uint8_t>((hp - oh * s) * k + (wp - ow * s));
        const int64_t o = ((static_cast<int64_t>(n) * OH + oh) * OW + ow) * C + c8 * 8;
        const uint64_t packed = *reinterpret_cast<const uint64_t*>(idx + o);
        float g[8];
        load8(dy, o, g);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (static_cast<uint8_t>(packed >> (8 * j)) == code) acc[j] += g[j];
      }
    }
    store8(dx, static_cast<int64_t>(v) * 8, acc);
  };
  if (lcv >= 0) {
    const int per_row = W << lcv;
    for (int row = blockIdx.x; row < N * H; row += gridDim.x) {
      const int n = row / H, h = row - n * H;
      for (int e = threadIdx.x; e < per_row; e += blockDim.x)
        one(static_cast<IDX>(row) * per_row + e, n, h, e >> lcv, e & ((1 << lcv) - 1));
    }
    return;
  }
  const IDX total = static_cast<IDX>(N) * H * W * cv;
  const IDX stride = static_cast<IDX>(gridDim.x) * blockDim.x;
  for (IDX v = static_cast<IDX>(blockIdx.x) * blockDim.x + threadIdx.x; v < total; v += stride) {
    const int c8 = static_cast<int>(v % cv);
    IDX r = v / cv;
    const int w = static_cast<int>(r % W);
    r /= W;
    const int h = static_cast<int>(r % H);
    one(v, static_cast<int>(r / H), h, w, c8);
  }
}

// k = 3, s = 2, p = 1 over even H, W (the ResNet stem pool): the dx pixel quad (2a + dh, 2b + dw)
// is covered by windows (a + i, b + j), i, j in {0, 1} only -- one thread reads those four
// (idx, dy) vectors once and writes the four dx vectors (the per-pixel form read 16 for 4).
// Window (i, j) reaches row dh iff i <= dh (tap row dh + 1 - 2i) and column dw iff j <= dw;
// contributions are summed in the (oh, ow) order of the per-pixel kernel (bitwise equal).
template <typename IDX>
__global__ __launch_bounds__(256) void maxpool_s2k3_bwd_quad_kernel(const uint16_t* __restrict__ dy,
                                                                    const uint8_t* __restrict__ idx,
                                                                    uint16_t* __restrict__ dx, int N, int H, int W,
                                                                    int C, int OH, int OW) {
  const int cv = C / 8, QH = H / 2, QW = W / 2;
  const IDX total = static_cast<IDX>(N) * QH * QW * cv;
  const IDX stride = static_cast<IDX>(gridDim.x) * blockDim.x;
  for (IDX v = static_cast<IDX>(blockIdx.x) * blockDim.x + threadIdx.x; v < total; v += stride) {
    const int c8 = static_cast<int>(v % cv);
    IDX r = v / cv;
    const int b = static_cast<int>(r % QW);
    r /= QW;
    const int a = static_cast<int>(r % QH);
    const int n = static_cast<int>(r / QH);
    uint64_t pk[4];
    u16x8 gv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // windows past the map are clamped in bounds and never used
      const int oh = min(a + (q >> 1), OH - 1), ow = min(b + (q & 1), OW - 1);
      const int64_t o = ((static_cast<int64_t>(n) * OH + oh) * OW + ow) * C + c8 * 8;
      pk[q] = *reinterpret_cast<const uint64_t*>(idx + o);
      gv[q] = *reinterpret_cast<const u16x8*>(dy + o);
    }
    const bool ih = a + 1 < OH, iw = b + 1 < OW;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = q >> 1, j = q & 1;
          if (i > dh || j > dw) continue;  // compile-time after unrolling
          if ((i && !ih) || (j && !iw)) continue;
          const uint8_t code = static_cast<uint8_t>((dh + 1 - 2 * i) * 3 + (dw + 1 - 2 * j));
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (static_cast<uint8_t>(pk[q] >> (8 * e)) == code) acc[e] += bf16_to_f32(gv[q][e]);
        }
        store8(dx, ((static_cast<int64_t>(n) * H + 2 * a + dh) * W + 2 * b + dw) * C + c8 * 8, acc);
      }
  }
}

// ResNet stem backward with the max-pool scatter fused into the BatchNorm backward passes
// (k = 3, s = 2, p = 1, even H / W; the pool input was relu(z * scale + shift), never stored):
// the pool's data gradient g is recomputed per 2x2 dx quad from the four covering windows'
// (argmax, dy) -- pooled-size reads -- instead of being written at full resolution and read twice:
//   REDUCE  per-channel partials sum(g'), sum(g' (z - mean) invstd) with g' = g * relu'(z sc + sh)
//           -> [G][C] (then the shared bn_bwd_finalize_kernel: dgamma, dbeta, ca / cb / cc)
//   APPLY   dz = ca g' + cb z + cc
// (replacing pool-bwd write + reduce read + apply read of the full-resolution gradient: 3 of the
// 7 full-size tensor passes of the stem backward).  g is rounded to bf16 exactly where the
// unfused path stored it.  The grid stride is a multiple of C / 8 (launcher), so every thread
// keeps one channel group and the partials stay in registers.
template <bool APPLY>
__global__ __launch_bounds__(256, 3) void pool_bn_bwd_kernel(const uint16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx,
                                                          const uint16_t* __restrict__ z,
                                                          const float* __restrict__ mc,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ coef, float* __restrict__ pd,
                                                          float* __restrict__ px, uint16_t* __restrict__ dz, int N,
                                                          int H, int W, int C, int OH, int OW) {
  const int cv = C / 8, QH = H / 2, QW = W / 2;
  const uint32_t total = static_cast<uint32_t>(N) * QH * QW * cv;
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t v0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int c8 = static_cast<int>(v0 % cv);
  float sc[8], sh[8], mu[8], is[8], A[8], B[8], Cc[8];
  load8(mc, c8 * 8, sc);
  load8(mc + C, c8 * 8, sh);
  if constexpr (APPLY) {
    load8(coef, c8 * 8, A);
    load8(coef + C, c8 * 8, B);
    load8(coef + 2 * C, c8 * 8, Cc);
  } else {
    load8(mean, c8 * 8, mu);
  }
  float sd[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t v = v0; v < total; v += stride) {
    uint32_t r = v / cv;
    const int b = static_cast<int>(r % QW);
    r /= QW;
    const int a = static_cast<int>(r % QH);
    const int n = static_cast<int>(r / QH);
    uint64_t pk[4];
    u16x8 gv[4], zv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // windows past the map are clamped in bounds and never used
      const int oh = min(a + (q >> 1), OH - 1), ow = min(b + (q & 1), OW - 1);
      const int64_t o = ((static_cast<int64_t>(n) * OH + oh) * OW + ow) * C + c8 * 8;
      pk[q] = *reinterpret_cast<const uint64_t*>(idx + o);
      gv[q] = *reinterpret_cast<const u16x8*>(dy + o);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      zv[q] = *reinterpret_cast<const u16x8*>(
          z + ((static_cast<int64_t>(n) * H + 2 * a + (q >> 1)) * W + 2 * b + (q & 1)) * C + c8 * 8);
    const bool ih = a + 1 < OH, iw = b + 1 < OW;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = q >> 1, j = q & 1;
          if (i > dh || j > dw) continue;
          if ((i && !ih) || (j && !iw)) continue;
          const uint8_t code = static_cast<uint8_t>((dh + 1 - 2 * i) * 3 + (dw + 1 - 2 * j));
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (static_cast<uint8_t>(pk[q] >> (8 * e)) == code) acc[e] += bf16_to_f32(gv[q][e]);
        }
        const u16x8& zz = zv[dh * 2 + dw];
        float out[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float zf = bf16_to_f32(zz[e]);
          const float g = zf * sc[e] + sh[e] > 0.f ? bf16_to_f32(f32_to_bf16(acc[e])) : 0.f;
          if constexpr (APPLY) {
            out[e] = A[e] * g + B[e] * zf + Cc[e];
          } else {
            sd[e] += g;
            sx[e] += g * (zf - mu[e]);  // x invstd once per channel at the end
          }
        }
        if constexpr (APPLY)
          store8(dz, ((static_cast<int64_t>(n) * H + 2 * a + dh) * W + 2 * b + dw) * C + c8 * 8, out);
      }
  }
  if constexpr (!APPLY) {
    __shared__ float lds_d[256 * 8];
    __shared__ float lds_x[256 * 8];
    const int t = threadIdx.x;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      lds_d[t * 8 + e] = sd[e];
      lds_x[t * 8 + e] = sx[e];
    }
    __syncthreads();
    if (t < cv) {  // fixed order over the threads of channel group t
      for (int k = t + cv; k < static_cast<int>(blockDim.x); k += cv)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          sd[e] += lds_d[k * 8 + e];
          sx[e] += lds_x[k * 8 + e];
        }
      load8(invstd, t * 8, is);
#pragma unroll
      for (int e = 0; e < 8; ++e) sx[e] *= is[e];
      float* od = pd + static_cast<int64_t>(blockIdx.x) * C + t * 8;
      float* ox = px + static_cast<int64_t>(blockIdx.x) * C + t * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        od[e] = sd[e];
        ox[e] = sx[e];
      }
    }
  }
}

// blocks of the fused stem backward: a multiple of 8 channel groups' worth of threads so each
// thread keeps its channel group (C / 8 divides 256)
int pool_bn_bwd_blocks(int64_t N, int H, int W, int C) {
  const int64_t quads = N * (H / 2) * (W / 2) * (C / 8);
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(2048, (quads + 255) / 256)));
}

void launch_pool_bn_bwd(const uint16_t* dy, const uint8_t* idx, const uint16_t* z, const float* mc, const float* mean,
                        const float* invstd, const float* gamma, float* ws, int G, float* dgamma, float* dbeta,
                        uint16_t* dz, int N, int H, int W, int C, int OH, int OW, hipStream_t st) {
  float* pd = ws;
  float* px = ws + static_cast<int64_t>(G) * C;
  float* coef = px + static_cast<int64_t>(G) * C;
  hipLaunchKernelGGL((pool_bn_bwd_kernel<false>), dim3(G), dim3(256), 0, st, dy, idx, z, mc, mean, invstd, nullptr, pd,
                     px, nullptr, N, H, W, C, OH, OW);
  launch_bn_bwd_partials(pd, px, G, nullptr, nullptr, gamma, mean, invstd, dgamma, dbeta, coef, nullptr,
                         static_cast<int64_t>(N) * H * W, C, st);
  if (dz == nullptr) return;  // the apply runs inside the stem weight gradient (stem.hip FUSED)
  hipLaunchKernelGGL((pool_bn_bwd_kernel<true>), dim3(G), dim3(256), 0, st, dy, idx, z, mc, nullptr, nullptr, coef,
                     nullptr, nullptr, dz, N, H, W, C, OH, OW);
}

// log2(C / 8) when the row mapping applies (C / 8 a power of two, rows of >= 64 elements so a
// block's threads stay busy, row indices in int range), else -1 (generic flat mapping)
static int row_lcv(int C, int width, int64_t rows) {
  const int cv = C / 8;
  if (cv <= 0 || (cv & (cv - 1)) || static_cast<int64_t>(width) * cv < 64 || rows * width * cv >= (int64_t(1) << 31))
    return -1;
  int l = 0;
  while ((1 << l) < cv) ++l;
  return l;
}

void launch_maxpool_nhwc_fwd(const uint16_t* x, const float* coef, uint16_t* y, uint8_t* idx, int N, int H, int W,
                             int C, int OH, int OW, int k, int s, int p, hipStream_t st) {
  const int64_t total = static_cast<int64_t>(N) * OH * OW * (C / 8);
  if (total <= 0) return;
  const int lcv = row_lcv(C, OW, static_cast<int64_t>(N) * OH);
  const int grid = lcv >= 0 ? static_cast<int>(std::min<int64_t>(static_cast<int64_t>(N) * OH, 1 << 20))
                            : stream_grid(total, 256);
  const bool i32 = total < (int64_t(1) << 31) - 2 * static_cast<int64_t>(stream_grid(total, 256)) * 256;
#define PSAMD_MPF(BN, T) \
  hipLaunchKernelGGL((maxpool_nhwc_fwd_kernel<BN, T>), dim3(grid), dim3(256), 0, st, x, coef, y, idx, N, H, W, C, OH, \
                     OW, k, s, p, lcv)
  if (coef && k == 3) {
    if (i32) {
      hipLaunchKernelGGL((maxpool_nhwc_fwd_kernel<true, uint32_t, true>), dim3(grid), dim3(256), 0, st, x, coef, y, idx,
                         N, H, W, C, OH, OW, k, s, p, lcv);
    } else {
      hipLaunchKernelGGL((maxpool_nhwc_fwd_kernel<true, int64_t, true>), dim3(grid), dim3(256), 0, st, x, coef, y, idx,
                         N, H, W, C, OH, OW, k, s, p, lcv);
    }
  } else if (coef) {
    if (i32) { PSAMD_MPF(true, uint32_t); } else { PSAMD_MPF(true, int64_t); }
  } else {
    if (i32) { PSAMD_MPF(false, uint32_t); } else { PSAMD_MPF(false, int64_t); }
  }
#undef PSAMD_MPF
}

void launch_maxpool_nhwc_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int H, int W, int C, int OH,
                             int OW, int k, int s, int p, hipStream_t st) {
  const int64_t total = static_cast<int64_t>(N) * H * W * (C / 8);
  if (total <= 0) return;
  if (k == 3 && s == 2 && p == 1 && H % 2 == 0 && W % 2 == 0 && OH == H / 2 && OW == W / 2) {
    const int64_t quads = total / 4;
    const int qgrid = stream_grid(quads, 256);
    if (quads < (int64_t(1) << 31) - 2 * static_cast<int64_t>(qgrid) * 256)
      hipLaunchKernelGGL((maxpool_s2k3_bwd_quad_kernel<uint32_t>), dim3(qgrid), dim3(256), 0, st, dy, idx, dx, N, H,
                         W, C, OH, OW);
    else
      hipLaunchKernelGGL((maxpool_s2k3_bwd_quad_kernel<int64_t>), dim3(qgrid), dim3(256), 0, st, dy, idx, dx, N, H,
                         W, C, OH, OW);
    return;
  }
  const int lcv = row_lcv(C, W, static_cast<int64_t>(N) * H);
  const int grid = lcv >= 0 ? static_cast<int>(std::min<int64_t>(static_cast<int64_t>(N) * H, 1 << 20))
                            : stream_grid(total, 256);
  const bool i32 = total < (int64_t(1) << 31) - 2 * static_cast<int64_t>(stream_grid(total, 256)) * 256;
#define PSAMD_MPB(T, SK) \
  hipLaunchKernelGGL((maxpool_nhwc_bwd_kernel<T, SK>), dim3(grid), dim3(256), 0, st, dy, idx, dx, N, H, W, C, OH, OW, \
                     k, s, p, lcv)
  if (k == 3 && s == 2) {
    if (i32) { PSAMD_MPB(uint32_t, true); } else { PSAMD_MPB(int64_t, true); }
  } else {
    if (i32) { PSAMD_MPB(uint32_t, false); } else { PSAMD_MPB(int64_t, false); }
  }
#undef PSAMD_MPB
}

}  // namespace psamd
