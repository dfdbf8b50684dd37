// Fused BatchNorm (+ residual add) + activation for NHWC (channels_last) activations.
//
// ResNet-50 under MIOpen spends ~37 % of its step in BatchNorm and another ~17 % in the
// separate ReLU / residual-add / ReLU-backward passes (profiles/archive/r1_resnet50_ps_kernel_breakdown.txt).
// All of them are HBM-bound, so the lever is passes over memory:
//
//   forward   MIOpen: stats(read x) + norm(read x, write z) + [add(read z,r write s)] + relu(read, write)
//             here:   stats(read x) + apply(read x [+ read r], write y)
//   backward  MIOpen: relu'(read dy,y write dz) + dscale/dbias(read dz,x) + dx(read dz,x write dx)
//             here:   reduce(read dy,y,x) + apply(read dy,y,x write dx [+ write dres])
//
// Layout: x, y, dy, dx, residual are [R, C] row-major bf16 (R = N*H*W, C channels, C % 8 == 0);
// gamma/beta/stats fp32.  Every thread moves 8 channels (16 B) per access.  Channel reductions
// are two-level and deterministic: block partials [G, C] in fp32 (no atomics) + a finalize
// kernel that sums them in fixed order.  act: 0 none, 1 relu.
#include <algorithm>
#include <cstdlib>
#include <utility>

#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

// channel groups (8 channels) per reduction block: wide tensors split into 256-channel tiles
// (blockIdx.y), so ~2048 blocks stream them with [G, C] partials of ~4 MB at any C
constexpr int kRedTpr = 32;

struct RedGeom {
  int tpr;      // threads per row = C / 8 (capped at kRedTpr per channel tile)
  int rows_it;  // rows a block covers per iteration = 256 / tpr
};

__host__ __device__ inline RedGeom red_geom(int C) {
  int tpr = C / 8;
  if (tpr > kRedTpr) tpr = kRedTpr;
  // round up to a power of two so rows_it * tpr == 256 (idle lanes if C/8 is not one)
  int p = 1;
  while (p < tpr) p <<= 1;
  return {p, 256 / p};
}

int bn_red_blocks(int64_t R, int C) {
  // >= 128 rows per block keeps the [G, C] partials <= 1/32 of the data ...
  int64_t g = (R + 127) / 128;
  // ... unless that leaves the chip under-filled: wide-channel / few-row tensors (ResNet stage 3-4:
  // 25-100K rows x 1-2K channels) need ~2048 blocks in total to keep enough loads in flight, down
  // to 8 rows per block
  const int ctiles = (C / 8 + kRedTpr - 1) / kRedTpr;
  const int64_t want = (2048 + ctiles - 1) / ctiles;
  if (g < want) g = std::min<int64_t>(want, (R + 7) / 8);
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return static_cast<int>(g);
}

// Elementwise BN passes: ~2 vectors per thread (one trip of the 2-vector loop), not a
// 2048-block grid-stride sweep -- the short-lived waves keep more loads in flight per CU
// (stage-1 block output + residual + bits: 519 -> 436 us, profiles/archive/r1_stream_probe.jsonl).
inline int apply_grid(int64_t nvec) {
  int64_t g = (nvec + 511) / 512;
  if (g < 1) g = 1;
  if (g > (int64_t(1) << 22)) g = int64_t(1) << 22;
  return static_cast<int>(g);
}

// ------------------------------------------------------------------------------ stats
// Shifted sums per block: partial_s1[g, c] = sum (x - K_c), partial_s2[g, c] = sum (x - K_c)^2
// with the shift K_c = x[0, c] (a sample of the channel, so |mean - K| ~ std): robust when
// |mean| >> std, unlike raw E[x^2] - E[x]^2, and -- unlike Welford -- no division or serial
// dependency per row, so the pass streams at the HBM rate (4 rows' loads in flight/thread).
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(const uint16_t* __restrict__ x, int64_t R, int C,
                                                               float* __restrict__ ps, float* __restrict__ pq) {
  __shared__ float lds_s[256 * 8];
  __shared__ float lds_q[256 * 8];
  const RedGeom gm = red_geom(C);
  const int t = threadIdx.x;
  const int cg = t % gm.tpr + blockIdx.y * kRedTpr;  // channel group (8 channels)
  const int r0 = t / gm.tpr;
  const int ngroups = C / 8;
  const int64_t G = gridDim.x;
  const int64_t rows_per_block = (R + G - 1) / G;
  const int64_t rb = blockIdx.x * rows_per_block;
  const int64_t re = (rb + rows_per_block < R) ? rb + rows_per_block : R;
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (cg < ngroups) {
    float K[8];
    load8(x, cg * 8, K);
    auto upd = [&](const float (&v)[8]) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - K[j];
        s1[j] += d;
        s2[j] += d * d;
      }
    };
    const int64_t step = gm.rows_it;
    int64_t r = rb + r0;
    for (; r + 3 * step < re; r += 4 * step) {
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) load8(x, (r + u * step) * C + cg * 8, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) upd(v[u]);
    }
    for (; r < re; r += step) {
      float v[8];
      load8(x, r * C + cg * 8, v);
      upd(v);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    lds_s[t * 8 + j] = s1[j];
    lds_q[t * 8 + j] = s2[j];
  }
  __syncthreads();
  if (r0 == 0 && cg < ngroups) {
    for (int k = 1; k < gm.rows_it; ++k) {
      const int src = (k * gm.tpr + t) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += lds_s[src + j];
        s2[j] += lds_q[src + j];
      }
    }
    float* o1 = ps + blockIdx.x * static_cast<int64_t>(C) + cg * 8;
    float* o2 = pq + blockIdx.x * static_cast<int64_t>(C) + cg * 8;
    *reinterpret_cast<f32x4*>(o1) = f32x4{s1[0], s1[1], s1[2], s1[3]};
    *reinterpret_cast<f32x4*>(o1 + 4) = f32x4{s1[4], s1[5], s1[6], s1[7]};
    *reinterpret_cast<f32x4*>(o2) = f32x4{s2[0], s2[1], s2[2], s2[3]};
    *reinterpret_cast<f32x4*>(o2 + 4) = f32x4{s2[4], s2[5], s2[6], s2[7]};
  }
}

// Sum the [G, C] partials of one 8-channel group per block: thread t reads rows g = t, t + blockDim, ...
// (8 consecutive channels = 32 B per row), then a wave + LDS tree over the block.  Fixed
// order -> deterministic.  Returns the 8 sums in threads 0..7 (one channel each).
__device__ __forceinline__ void sum_partials8(const float* __restrict__ p, const float* __restrict__ q, int G, int C,
                                              int cg, float* lds, float& outp, float& outq) {
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // 4 rows per thread in flight at once (branch-free: clamped row, zero weight past G); a rolled
  // loop waits out one L2/HBM round trip per row (12-25 us per call at G = 2048)
  constexpr int U = 4;
  for (int g0 = threadIdx.x; g0 < G; g0 += U * blockDim.x) {
    float u[U][8], v[U][8], w[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int g = g0 + i * blockDim.x;
      w[i] = g < G ? 1.f : 0.f;
      const int64_t o = static_cast<int64_t>(g < G ? g : G - 1) * C + cg * 8;
      load8(p, o, u[i]);
      load8(q, o, v[i]);
    }
#pragma unroll
    for (int i = 0; i < U; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a[j] += w[i] * u[i][j];
        b[j] += w[i] * v[i][j];
      }
  }
  // wave reduce, then across the 4 waves through LDS
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = wave_sum(a[j]);
    b[j] = wave_sum(b[j]);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lds[wid * 16 + j] = a[j];
      lds[wid * 16 + 8 + j] = b[j];
    }
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    float sa = 0.f, sb = 0.f;
    for (int w = 0; w < static_cast<int>(blockDim.x >> 6); ++w) {
      sa += lds[w * 16 + threadIdx.x];
      sb += lds[w * 16 + 8 + threadIdx.x];
    }
    outp = sa;
    outq = sb;
  }
}

// First level for very tall partials (the per-tile partials of the non-persistent conv GEMMs,
// G ~ 12.5K rows): block (cg, s) sums rows [s * kFoldRows, (s + 1) * kFoldRows) of channel
// group cg into row s of [S][C] -- fixed order, so the two-level sum stays deterministic.
constexpr int kFoldRows = 1024;
__global__ __launch_bounds__(256) void partials_fold_kernel(const float* __restrict__ p, const float* __restrict__ q,
                                                            int G, int C, float* __restrict__ op,
                                                            float* __restrict__ oq) {
  __shared__ float lds[16 * 16];
  const int r0 = blockIdx.y * kFoldRows;
  const int rows = G - r0 < kFoldRows ? G - r0 : kFoldRows;
  float a = 0.f, b = 0.f;
  sum_partials8(p + static_cast<int64_t>(r0) * C, q + static_cast<int64_t>(r0) * C, rows, C, blockIdx.x, lds, a, b);
  if (threadIdx.x < 8) {
    const int64_t o = static_cast<int64_t>(blockIdx.y) * C + blockIdx.x * 8 + threadIdx.x;
    op[o] = a;
    oq[o] = b;
  }
}

int partials_fold_rows(int G) { return G > 2 * kFoldRows ? (G + kFoldRows - 1) / kFoldRows : 0; }

void launch_partials_fold(const float* p, const float* q, int G, int C, float* op, float* oq, hipStream_t s) {
  hipLaunchKernelGGL(partials_fold_kernel, dim3(C / 8, partials_fold_rows(G)), dim3(256), 0, s, p, q, G, C, op, oq);
}

// Threads per finalize block (one block per 8 channels): the per-tile partials of the
// non-persistent conv GEMMs reach G ~ 12.5K rows, which 256 threads walk in 25-35 us.
inline int fin_threads(int G) { return G >= 4096 ? 1024 : G >= 1024 ? 512 : 256; }

// per channel: mean, invstd, scale = gamma*invstd, shift = beta - mean*scale; running stats.
// grid = C / 8 blocks of fin_threads(G) threads.
// kshift: the shift the partial sums were taken about -- x[0, c] when null (bn_stats_partial),
// else an explicit per-channel array (producer-fused statistics, e.g. the stem convolution).
__global__ __launch_bounds__(1024) void bn_finalize_kernel(const float* __restrict__ ps, const float* __restrict__ pq,
                                                          const uint16_t* __restrict__ x,
                                                          const float* kshift /* may alias rmean */, int G, int C, int64_t R,
                                                          float eps, float momentum, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* rmean,
                                                          float* __restrict__ rvar, float* __restrict__ mean_out,
                                                          float* __restrict__ invstd_out, float* __restrict__ scale,
                                                          float* __restrict__ shift) {
  __shared__ float lds[16 * 16];  // up to 16 waves
  float s1 = 0.f, s2 = 0.f;
  sum_partials8(ps, pq, G, C, blockIdx.x, lds, s1, s2);
  if (threadIdx.x >= 8) return;
  const int c = blockIdx.x * 8 + threadIdx.x;
  const float inv_n = 1.f / static_cast<float>(R);
  const float dm = s1 * inv_n;  // mean - K
  const float mean = (kshift ? kshift[c] : bf16_to_f32(x[c])) + dm;
  float var = s2 * inv_n - dm * dm;
  if (var < 0.f) var = 0.f;
  const float invstd = rsqrtf(var + eps);
  const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
  mean_out[c] = mean;
  invstd_out[c] = invstd;
  scale[c] = ga * invstd;
  shift[c] = be - mean * ga * invstd;
  if (rmean) {
    const float unbiased = R > 1 ? var * static_cast<float>(R) / static_cast<float>(R - 1) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * unbiased;
  }
}

// eval mode: scale/shift from running stats
__global__ __launch_bounds__(256) void bn_eval_coef_kernel(int C, float eps, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ rmean,
                                                           const float* __restrict__ rvar, float* __restrict__ scale,
                                                           float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(rvar[c] + eps);
  const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
  scale[c] = ga * invstd;
  shift[c] = be - rmean[c] * ga * invstd;
}

// y = act(x * scale_c + shift_c [+ res]).  FIXED_C: the grid stride is a multiple of C/8, so
// each thread's channel group never changes -- coefficients are loaded once and the 64-bit
// modulo leaves the loop.  Two vectors per thread per iteration keep enough loads in flight.
// MASK: also store the ReLU mask of y as one bit per element (byte v <-> elements 8v..8v+7):
// the backward then reads 1/16 of the bytes it would read from y.
template <bool RES, int ACT, bool FIXED_C, bool MASK = false>
__global__ __launch_bounds__(256) void bn_apply_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, uint16_t* __restrict__ y,
                                                       int64_t nvec, int C, uint8_t* __restrict__ mb) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int cvec = C / 8;
  const int64_t v0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  float sc[8], sh[8];
  if constexpr (FIXED_C) {
    const int c = static_cast<int>(v0 % cvec) * 8;
    load8(scale, c, sc);
    load8(shift, c, sh);
  }
  auto one = [&](int64_t v, float (&a)[8], const float (&b)[8]) {
    if constexpr (!FIXED_C) {
      const int c = static_cast<int>(v % cvec) * 8;
      load8(scale, c, sc);
      load8(shift, c, sh);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = a[j] * sc[j] + sh[j];
      if constexpr (RES) o += b[j];
      if constexpr (ACT == 1) o = o > 0.f ? o : 0.f;
      a[j] = o;
    }
    store8(y, v * 8, a);
    if constexpr (MASK) {
      unsigned bits = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) bits |= (a[j] > 0.f ? 1u : 0u) << j;
      mb[v] = static_cast<uint8_t>(bits);
    }
  };
  int64_t v = v0;
  for (; v + stride < nvec; v += 2 * stride) {
    float a0[8], a1[8], b0[8], b1[8];
    load8(x, v * 8, a0);
    load8(x, (v + stride) * 8, a1);
    if constexpr (RES) {
      load8(res, v * 8, b0);
      load8(res, (v + stride) * 8, b1);
    }
    one(v, a0, b0);
    one(v + stride, a1, b1);
  }
  if (v < nvec) {
    float a0[8], b0[8];
    load8(x, v * 8, a0);
    if constexpr (RES) load8(res, v * 8, b0);
    one(v, a0, b0);
  }
}

// ------------------------------------------------------------------------------ backward
// partial_dz[g,c] = sum dz ; partial_dzx[g,c] = sum dz * (x - mean) * invstd ; dz = dy * act'(.)
// ACT: 0 identity, 1 relu mask from the saved output y, 2 relu mask recomputed from x with the
// forward's scale/shift (mc = [scale | shift]) -- no residual, so y > 0 <=> x*scale+shift > 0;
// saves one tensor read in both backward passes.
// ACT 3: relu mask from the bit mask written by the forward apply (MASK)
template <int ACT>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const uint16_t* __restrict__ dy,
                                                            const uint16_t* __restrict__ y,
                                                            const uint16_t* __restrict__ x,
                                                            const float* __restrict__ mc,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, int64_t R, int C,
                                                            float* __restrict__ pd, float* __restrict__ px,
                                                            const uint8_t* __restrict__ mb) {
  __shared__ float lds_d[256 * 8];
  __shared__ float lds_x[256 * 8];
  const RedGeom gm = red_geom(C);
  const int t = threadIdx.x;
  const int cg = t % gm.tpr + blockIdx.y * kRedTpr;
  const int r0 = t / gm.tpr;
  const int ngroups = C / 8;
  const int64_t G = gridDim.x;
  const int64_t rows_per_block = (R + G - 1) / G;
  const int64_t rb = blockIdx.x * rows_per_block;
  const int64_t re = (rb + rows_per_block < R) ? rb + rows_per_block : R;
  float sd[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (cg < ngroups) {
    float mu[8], is[8], sc[8], sh[8];
    load8(mean, cg * 8, mu);
    load8(invstd, cg * 8, is);
    if constexpr (ACT == 2) {
      load8(mc, cg * 8, sc);
      load8(mc + C, cg * 8, sh);
    }
    auto acc = [&](float (&g)[8], const float (&xv)[8], const float (&yv)[8], unsigned bits) {
      if constexpr (ACT == 3) {
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = (bits >> j) & 1u ? g[j] : 0.f;
      } else if constexpr (ACT == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
      } else if constexpr (ACT == 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = xv[j] * sc[j] + sh[j] > 0.f ? g[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sd[j] += g[j];
        sx[j] += g[j] * (xv[j] - mu[j]) * is[j];
      }
    };
    const int64_t step = gm.rows_it;
    int64_t r = rb + r0;
    constexpr int U = ACT == 1 ? 2 : 4;  // loads in flight per thread (2 or 3 tensors each)
    for (; r + (U - 1) * step < re; r += U * step) {
      float g[U][8], xv[U][8], yv[U][8];
      unsigned bits[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t o = (r + u * step) * C + cg * 8;
        load8(dy, o, g[u]);
        load8(x, o, xv[u]);
        if constexpr (ACT == 1) load8(y, o, yv[u]);
        if constexpr (ACT == 3) bits[u] = mb[o >> 3];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc(g[u], xv[u], yv[u], ACT == 3 ? bits[u] : 0u);
    }
    for (; r < re; r += step) {
      float g[8], xv[8], yv[8];
      const int64_t o = r * C + cg * 8;
      load8(dy, o, g);
      load8(x, o, xv);
      if constexpr (ACT == 1) load8(y, o, yv);
      acc(g, xv, yv, ACT == 3 ? static_cast<unsigned>(mb[o >> 3]) : 0u);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    lds_d[t * 8 + j] = sd[j];
    lds_x[t * 8 + j] = sx[j];
  }
  __syncthreads();
  if (r0 == 0 && cg < ngroups) {
    for (int k = 1; k < gm.rows_it; ++k) {
      const int src = (k * gm.tpr + t) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sd[j] += lds_d[src + j];
        sx[j] += lds_x[src + j];
      }
    }
    float* od = pd + blockIdx.x * static_cast<int64_t>(C) + cg * 8;
    float* ox = px + blockIdx.x * static_cast<int64_t>(C) + cg * 8;
    *reinterpret_cast<f32x4*>(od) = f32x4{sd[0], sd[1], sd[2], sd[3]};
    *reinterpret_cast<f32x4*>(od + 4) = f32x4{sd[4], sd[5], sd[6], sd[7]};
    *reinterpret_cast<f32x4*>(ox) = f32x4{sx[0], sx[1], sx[2], sx[3]};
    *reinterpret_cast<f32x4*>(ox + 4) = f32x4{sx[4], sx[5], sx[6], sx[7]};
  }
}

// dgamma = sum dz*xhat, dbeta = sum dz; dx = A dz + B x + Cc.  grid = C / 8 blocks.
__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(const float* __restrict__ pd,
                                                              const float* __restrict__ px, int G, int C, int64_t R,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              float* __restrict__ ca, float* __restrict__ cb,
                                                              float* __restrict__ cc) {
  __shared__ float lds[16 * 16];  // up to 16 waves
  float sd = 0.f, sx = 0.f;
  sum_partials8(pd, px, G, C, blockIdx.x, lds, sd, sx);
  if (threadIdx.x >= 8) return;
  const int c = blockIdx.x * 8 + threadIdx.x;
  if (dgamma) dgamma[c] = sx;
  if (dbeta) dbeta[c] = sd;
  const float ga = gamma ? gamma[c] : 1.f;
  const float is = invstd[c];
  const float k = ga * is;
  const float md = sd / static_cast<float>(R);
  const float mx = sx / static_cast<float>(R);
  ca[c] = k;
  cb[c] = -k * is * mx;
  cc[c] = -k * md + k * is * mx * mean[c];
}

// dz = dy * act'(.) [dres = dz]; dx = A dz + B x + Cc.  FIXED_C as in bn_apply_kernel.
template <int ACT, bool DRES, bool FIXED_C>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const uint16_t* __restrict__ dy,
                                                           const uint16_t* __restrict__ y,
                                                           const uint16_t* __restrict__ x,
                                                           const float* __restrict__ mc,
                                                           const float* __restrict__ ca,
                                                           const float* __restrict__ cb,
                                                           const float* __restrict__ cc, uint16_t* __restrict__ dx,
                                                           uint16_t* __restrict__ dres, int64_t nvec, int C,
                                                           const uint8_t* __restrict__ mb) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int cvec = C / 8;
  const int64_t v0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  float A[8], B[8], Cc[8], sc[8], sh[8];
  auto coefs = [&](int c) {
    load8(ca, c, A);
    load8(cb, c, B);
    load8(cc, c, Cc);
    if constexpr (ACT == 2) {
      load8(mc, c, sc);
      load8(mc + C, c, sh);
    }
  };
  if constexpr (FIXED_C) coefs(static_cast<int>(v0 % cvec) * 8);
  auto one = [&](int64_t v, float (&g)[8], float (&xv)[8], const float (&yv)[8]) {
    if constexpr (!FIXED_C) coefs(static_cast<int>(v % cvec) * 8);
    if constexpr (ACT == 3) {
      const unsigned bits = mb[v];
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = (bits >> j) & 1u ? g[j] : 0.f;
    } else if constexpr (ACT == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
    } else if constexpr (ACT == 2) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = xv[j] * sc[j] + sh[j] > 0.f ? g[j] : 0.f;
    }
    if constexpr (DRES) store8(dres, v * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = A[j] * g[j] + B[j] * xv[j] + Cc[j];
    store8(dx, v * 8, xv);
  };
  int64_t v = v0;
  for (; v + stride < nvec; v += 2 * stride) {
    float g0[8], g1[8], x0[8], x1[8], y0[8], y1[8];
    load8(dy, v * 8, g0);
    load8(dy, (v + stride) * 8, g1);
    load8(x, v * 8, x0);
    load8(x, (v + stride) * 8, x1);
    if constexpr (ACT == 1) {
      load8(y, v * 8, y0);
      load8(y, (v + stride) * 8, y1);
    }
    one(v, g0, x0, y0);
    one(v + stride, g1, x1, y1);
  }
  if (v < nvec) {
    float g0[8], x0[8], y0[8];
    load8(dy, v * 8, g0);
    load8(x, v * 8, x0);
    if constexpr (ACT == 1) load8(y, v * 8, y0);
    one(v, g0, x0, y0);
  }
}

// ------------------------------------------------------------------------------ launchers
void launch_bn_fwd(const BnFwdArgs& a, hipStream_t s) {
  const int C = a.C;
  const int64_t R = a.R;
  const int cblocks = (C + 255) / 256;
  if (a.training) {
    const int G = a.G;
    const int ctiles = (C / 8 + kRedTpr - 1) / kRedTpr;
    hipLaunchKernelGGL(bn_stats_partial_kernel, dim3(G, ctiles), dim3(256), 0, s, a.x, R, C, a.ws, a.ws + G * C);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(C / 8), dim3(fin_threads(G)), 0, s, a.ws, a.ws + G * C, a.x, nullptr, G, C, R,
                       a.eps,
                       a.momentum, a.gamma, a.beta, a.rmean, a.rvar, a.mean, a.invstd, a.scale, a.shift);
  } else {
    hipLaunchKernelGGL(bn_eval_coef_kernel, dim3(cblocks), dim3(256), 0, s, C, a.eps, a.gamma, a.beta, a.rmean,
                       a.rvar, a.scale, a.shift);
  }
  if (!a.y) return;  // statistics / coefficients only (the apply is fused into a consumer)
  const int64_t nvec = R * C / 8;
  const int grid = apply_grid(nvec);
  const bool fixed = (static_cast<int64_t>(grid) * 256) % (C / 8) == 0;
  uint8_t* nomask = nullptr;
#define PSAMD_BN_APPLY(RES, ACT)                                                                              \
  if (fixed)                                                                                                  \
    hipLaunchKernelGGL((bn_apply_kernel<RES, ACT, true>), dim3(grid), dim3(256), 0, s, a.x, a.res, a.scale,    \
                       a.shift, a.y, nvec, C, nomask);                                                        \
  else                                                                                                        \
    hipLaunchKernelGGL((bn_apply_kernel<RES, ACT, false>), dim3(grid), dim3(256), 0, s, a.x, a.res, a.scale,   \
                       a.shift, a.y, nvec, C, nomask)
  if (a.res) {
    if (a.act == 1) { PSAMD_BN_APPLY(true, 1); }
    else { PSAMD_BN_APPLY(true, 0); }
  } else {
    if (a.act == 1) { PSAMD_BN_APPLY(false, 1); }
    else { PSAMD_BN_APPLY(false, 0); }
  }
#undef PSAMD_BN_APPLY
}

void launch_bn_finalize_sums(const float* ps, const float* pq, const float* kshift, int G, int C, int64_t R,
                             float eps, float momentum, const float* gamma, const float* beta, float* rmean,
                             float* rvar, float* mean, float* invstd, float* scale, float* shift, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(C / 8), dim3(fin_threads(G)), 0, s, ps, pq, nullptr, kshift, G, C, R, eps,
                     momentum, gamma, beta, rmean, rvar, mean, invstd, scale, shift);
}

void launch_bn_bwd(const BnBwdArgs& a, hipStream_t s) {
  const int C = a.C;
  const int64_t R = a.R;
  const int G = a.G;
  const int ctiles = (C / 8 + kRedTpr - 1) / kRedTpr;
  const int act = a.mbits ? 3 : ((a.act == 1 && a.mask_coef && !a.dres) ? 2 : a.act);
#define PSAMD_BN_RED(ACT)                                                                                       \
  hipLaunchKernelGGL(bn_bwd_reduce_kernel<ACT>, dim3(G, ctiles), dim3(256), 0, s, a.dy, a.y, a.x, a.mask_coef, \
                     a.mean, a.invstd, R, C, a.ws, a.ws + G * C, a.mbits)
  if (act == 3) PSAMD_BN_RED(3);
  else if (act == 2) PSAMD_BN_RED(2);
  else if (act == 1) PSAMD_BN_RED(1);
  else PSAMD_BN_RED(0);
#undef PSAMD_BN_RED
  float* coef = a.ws + 2 * G * C;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C / 8), dim3(fin_threads(G)), 0, s, a.ws, a.ws + G * C, G, C, R,
                     a.gamma, a.mean, a.invstd, a.dgamma, a.dbeta, coef, coef + C, coef + 2 * C);
  const int64_t nvec = R * C / 8;
  const int grid = apply_grid(nvec);
  const bool fixed = (static_cast<int64_t>(grid) * 256) % (C / 8) == 0;
#define PSAMD_BN_BWD(ACT, DRES)                                                                                 \
  if (fixed)                                                                                                    \
    hipLaunchKernelGGL((bn_bwd_apply_kernel<ACT, DRES, true>), dim3(grid), dim3(256), 0, s, a.dy, a.y, a.x,      \
                       a.mask_coef, coef, coef + C, coef + 2 * C, a.dx, a.dres, nvec, C, a.mbits);              \
  else                                                                                                          \
    hipLaunchKernelGGL((bn_bwd_apply_kernel<ACT, DRES, false>), dim3(grid), dim3(256), 0, s, a.dy, a.y, a.x,     \
                       a.mask_coef, coef, coef + C, coef + 2 * C, a.dx, a.dres, nvec, C, a.mbits)
  if (act == 3) {
    if (a.dres) { PSAMD_BN_BWD(3, true); }
    else { PSAMD_BN_BWD(3, false); }
  } else if (a.dres) {
    if (act == 1) { PSAMD_BN_BWD(1, true); }
    else { PSAMD_BN_BWD(0, true); }
  } else {
    if (act == 2) { PSAMD_BN_BWD(2, false); }
    else if (act == 1) { PSAMD_BN_BWD(1, false); }
    else { PSAMD_BN_BWD(0, false); }
  }
#undef PSAMD_BN_BWD
}

// ------------------------------------------------------------------------------ fused-bottleneck helpers
// y = act(x * scale + shift + res * rscale + rshift): the bottleneck output when the identity
// branch is a downsample conv whose BN is applied in the same pass (its output never hits HBM).
template <int ACT, bool FIXED_C, bool MASK>
__global__ __launch_bounds__(256) void bn_apply_dual_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ r,
                                                            const float* __restrict__ coef,
                                                            const float* __restrict__ rcoef, uint16_t* __restrict__ y,
                                                            int64_t nvec, int C, uint8_t* __restrict__ mb) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int cvec = C / 8;
  const int64_t v0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  float sc[8], sh[8], rs[8], rh[8];
  auto coefs = [&](int c) {
    load8(coef, c, sc);
    load8(coef + C, c, sh);
    load8(rcoef, c, rs);
    load8(rcoef + C, c, rh);
  };
  if constexpr (FIXED_C) coefs(static_cast<int>(v0 % cvec) * 8);
  for (int64_t v = v0; v < nvec; v += stride) {
    if constexpr (!FIXED_C) coefs(static_cast<int>(v % cvec) * 8);
    float a[8], b[8];
    load8(x, v * 8, a);
    load8(r, v * 8, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = a[j] * sc[j] + sh[j] + (b[j] * rs[j] + rh[j]);
      if constexpr (ACT == 1) o = o > 0.f ? o : 0.f;
      a[j] = o;
    }
    store8(y, v * 8, a);
    if constexpr (MASK) {
      unsigned bits = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) bits |= (a[j] > 0.f ? 1u : 0u) << j;
      mb[v] = static_cast<uint8_t>(bits);
    }
  }
}

void launch_bn_apply_coef(const uint16_t* x, const uint16_t* res, const float* coef, const float* rcoef, uint16_t* y,
                          uint8_t* mbits, int64_t R, int C, int act, hipStream_t s) {
  const int64_t nvec = R * C / 8;
  if (nvec <= 0) return;
  const int grid = apply_grid(nvec);
  const bool fixed = (static_cast<int64_t>(grid) * 256) % (C / 8) == 0;
  const bool mask = mbits != nullptr;
#define PSAMD_LAUNCH(K, ...) hipLaunchKernelGGL((K<__VA_ARGS__>), dim3(grid), dim3(256), 0, s, ARGS)
#define PSAMD_FM(K, ...)                                                            \
  if (fixed) {                                                                      \
    if (mask) { PSAMD_LAUNCH(K, __VA_ARGS__, true, true); }                         \
    else { PSAMD_LAUNCH(K, __VA_ARGS__, true, false); }                             \
  } else {                                                                          \
    if (mask) { PSAMD_LAUNCH(K, __VA_ARGS__, false, true); }                        \
    else { PSAMD_LAUNCH(K, __VA_ARGS__, false, false); }                            \
  }
  if (rcoef) {
#define ARGS x, res, coef, rcoef, y, nvec, C, mbits
    if (act == 1) { PSAMD_FM(bn_apply_dual_kernel, 1) }
    else { PSAMD_FM(bn_apply_dual_kernel, 0) }
#undef ARGS
  } else {
#define ARGS x, res, coef, coef + C, y, nvec, C, mbits
    if (res) {
      if (act == 1) { PSAMD_FM(bn_apply_kernel, true, 1) }
      else { PSAMD_FM(bn_apply_kernel, true, 0) }
    } else {
      if (act == 1) { PSAMD_FM(bn_apply_kernel, false, 1) }
      else { PSAMD_FM(bn_apply_kernel, false, 0) }
    }
#undef ARGS
  }
#undef PSAMD_FM
#undef PSAMD_LAUNCH
}

void launch_bn_bwd_partials(const float* pd, const float* px, int G, const uint16_t* g, const uint16_t* x,
                            const float* gamma, const float* mean, const float* invstd, float* dgamma, float* dbeta,
                            float* coef, uint16_t* dx, int64_t R, int C, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C / 8), dim3(fin_threads(G)), 0, s, pd, px, G, C, R, gamma, mean,
                     invstd, dgamma, dbeta, coef, coef + C, coef + 2 * C);
  const int64_t nvec = R * C / 8;
  if (nvec <= 0 || dx == nullptr) return;  // dx null: coefficients only (a GEMM prologue applies them)
  const int grid = apply_grid(nvec);
  const bool fixed = (static_cast<int64_t>(grid) * 256) % (C / 8) == 0;
  const uint16_t* none = nullptr;
  const float* nomc = nullptr;
  uint16_t* nodres = nullptr;
  const uint8_t* nobits = nullptr;
  if (fixed)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<0, false, true>), dim3(grid), dim3(256), 0, s, g, none, x, nomc, coef,
                       coef + C, coef + 2 * C, dx, nodres, nvec, C, nobits);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<0, false, false>), dim3(grid), dim3(256), 0, s, g, none, x, nomc, coef,
                       coef + C, coef + 2 * C, dx, nodres, nvec, C, nobits);
}

}  // namespace psamd
