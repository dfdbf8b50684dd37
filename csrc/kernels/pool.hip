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
#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

// IDX: 32-bit index math when the element count allows it (64-bit div/mod is a long
// instruction sequence on CDNA and dominated these HBM-light, address-heavy kernels)
template <bool BN, typename IDX>
__global__ __launch_bounds__(256) void maxpool_nhwc_fwd_kernel(const uint16_t* __restrict__ x,
                                                               const float* __restrict__ coef,
                                                               uint16_t* __restrict__ y, uint8_t* __restrict__ idx,
                                                               int N, int H, int W, int C, int OH, int OW, int k,
                                                               int s, int p) {
  const IDX cv = C / 8;
  const IDX total = static_cast<IDX>(N) * OH * OW * cv;
  const IDX stride = static_cast<IDX>(gridDim.x) * blockDim.x;
  for (IDX v = static_cast<IDX>(blockIdx.x) * blockDim.x + threadIdx.x; v < total; v += stride) {
    const int c8 = static_cast<int>(v % cv);
    IDX r = v / cv;
    const int ow = static_cast<int>(r % OW);
    r /= OW;
    const int oh = static_cast<int>(r % OH);
    const int n = static_cast<int>(r / OH);
    float sc[8], sh[8];
    if constexpr (BN) {
      load8(coef, c8 * 8, sc);
      load8(coef + C, c8 * 8, sh);
    }
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    const int h0 = oh * s - p, w0 = ow * s - p;
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
          float t = a[j];
          if constexpr (BN) {
            t = t * sc[j] + sh[j];
            t = t > 0.f ? t : 0.f;
            t = bf16_to_f32(f32_to_bf16(t));  // compare what the unfused path would have stored
          }
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
  }
}

template <typename IDX>
__global__ __launch_bounds__(256) void maxpool_nhwc_bwd_kernel(const uint16_t* __restrict__ dy,
                                                               const uint8_t* __restrict__ idx,
                                                               uint16_t* __restrict__ dx, int N, int H, int W, int C,
                                                               int OH, int OW, int k, int s, int p) {
  const IDX cv = C / 8;
  const IDX total = static_cast<IDX>(N) * H * W * cv;
  const IDX stride = static_cast<IDX>(gridDim.x) * blockDim.x;
  for (IDX v = static_cast<IDX>(blockIdx.x) * blockDim.x + threadIdx.x; v < total; v += stride) {
    const int c8 = static_cast<int>(v % cv);
    IDX r = v / cv;
    const int w = static_cast<int>(r % W);
    r /= W;
    const int h = static_cast<int>(r % H);
    const int n = static_cast<int>(r / H);
    // output windows covering (h, w): oh*s - p <= h <= oh*s - p + k - 1
    const int hp = h + p, wp = w + p;
    const int oh_lo = hp - k + 1 > 0 ? (hp - k + 1 + s - 1) / s : 0;
    const int oh_hi = min(OH - 1, hp / s);
    const int ow_lo = wp - k + 1 > 0 ? (wp - k + 1 + s - 1) / s : 0;
    const int ow_hi = min(OW - 1, wp / s);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
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
  }
}

void launch_maxpool_nhwc_fwd(const uint16_t* x, const float* coef, uint16_t* y, uint8_t* idx, int N, int H, int W,
                             int C, int OH, int OW, int k, int s, int p, hipStream_t st) {
  const int64_t total = static_cast<int64_t>(N) * OH * OW * (C / 8);
  if (total <= 0) return;
  const int grid = stream_grid(total, 256);
  const bool i32 = total < (int64_t(1) << 31) - 2 * static_cast<int64_t>(grid) * 256;
#define PSAMD_MPF(BN, T) \
  hipLaunchKernelGGL((maxpool_nhwc_fwd_kernel<BN, T>), dim3(grid), dim3(256), 0, st, x, coef, y, idx, N, H, W, C, OH, \
                     OW, k, s, p)
  if (coef) {
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
  const int grid = stream_grid(total, 256);
  if (total < (int64_t(1) << 31) - 2 * static_cast<int64_t>(grid) * 256)
    hipLaunchKernelGGL(maxpool_nhwc_bwd_kernel<uint32_t>, dim3(grid), dim3(256), 0, st, dy, idx, dx, N, H, W, C, OH,
                       OW, k, s, p);
  else
    hipLaunchKernelGGL(maxpool_nhwc_bwd_kernel<int64_t>, dim3(grid), dim3(256), 0, st, dy, idx, dx, N, H, W, C, OH,
                       OW, k, s, p);
}

}  // namespace psamd
