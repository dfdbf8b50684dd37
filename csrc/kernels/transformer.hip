// Fused transformer elementwise / row-normalisation kernels (bf16 activations, fp32 math) for
// the BERT-base and Llama-3 north-star configs (SURVEY §5.7 / BASELINE.json), replacing chains
// of 3-8 separate torch kernels (each a full HBM pass) measured on MI355X (profiles/):
//
//   rmsnorm        y = x * rsqrt(mean(x^2) + eps) * w        [+ fused residual s = x + r]
//   layernorm      s = x + dropout_p(o);  y = (s - mean) * rstd * gamma + beta   (BERT post-LN)
//   swiglu         h = silu(g) * u  from the fused gate/up GEMM output [g | u]
//   rope_split     q, k, v = RoPE(qkv)  with the [B, S, heads, hd] -> [B, heads, S, hd] transpose
//
// Row kernels: one wave64 per row (4 rows per 256-thread block, grid-stride over rows), 8 bf16
// (16 B) per lane-vector, VPT = D / 512 vectors per lane held in registers between the
// reductions (pure wave shuffles: no LDS, no block barrier) and the write; D <= 4096.
// Backward row kernels also accumulate the per-column weight gradients (dw / dgamma / dbeta)
// of the rows a wave owns in registers and write one fp32 partial row per wave; a second
// fixed-order kernel sums the partials (deterministic, no atomics).
//
// Dropout masks are regenerated from (seed, element index) with the same Philox stream as
// csrc/kernels/ref_ops.hip (element i uses counter i/4, lane i%4): never stored.
#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

namespace {
constexpr int kT = 256;
constexpr int kL = 64;  // lanes per row

#define PSAMD_ROW_LOOP(R)                                               \
  const int lane_ = threadIdx.x & 63;                                   \
  const int wid_ = blockIdx.x * 4 + (threadIdx.x >> 6);                 \
  for (int row = wid_; row < (R); row += gridDim.x * 4)

__device__ __forceinline__ void keep_mask8(uint64_t seed, int64_t i0, float p, float (&m)[8]) {
  // element i uses Philox(seed, i / 4)[i % 4]; i0 is a multiple of 8
  uint32_t a[4], b[4];
  Philox::gen(seed, static_cast<uint64_t>(i0 / 4), a);
  Philox::gen(seed, static_cast<uint64_t>(i0 / 4 + 1), b);
  const float sc = 1.f / (1.f - p);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m[j] = Philox::u01(a[j]) >= p ? sc : 0.f;
    m[4 + j] = Philox::u01(b[j]) >= p ? sc : 0.f;
  }
}

// Sum the 4 waves' per-column register partials (lane-vector layout vi = lane + k*64) in a
// fixed wave order through one LDS row and write the block's partial row to out[0..D).
template <int VPT>
__device__ __forceinline__ void block_fold_rows(const float (&acc)[VPT][8], float* lacc, int D, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nv = D / 8;
  for (int step = 0; step < 4; ++step) {
    if (w == step) {
#pragma unroll
      for (int k = 0; k < VPT; ++k) {
        const int vi = lane + k * kL;
        if (vi < nv) {
          float t[8];
          if (step == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) t[j] = acc[k][j];
          } else {
            load8(lacc, vi * 8, t);
#pragma unroll
            for (int j = 0; j < 8; ++j) t[j] += acc[k][j];
          }
          if (step == 3) store8(out, vi * 8, t);
          else store8(lacc, vi * 8, t);
        }
      }
    }
    __syncthreads();
  }
}

__device__ __forceinline__ void loadw8(const float* w, int64_t i, float (&o)[8]) { load8(w, i, o); }
__device__ __forceinline__ void loadw8(const uint16_t* w, int64_t i, float (&o)[8]) { load8(w, i, o); }
}  // namespace

// ------------------------------------------------------------------------------ RMSNorm
// x, r, s, y: [R, D] bf16; w: [D] (WT = float or bf16); rstd: [R] fp32.  RES: s = x + r is
// written and normalised (pre-norm residual stream).
template <int VPT, bool RES, typename WT>
__global__ __launch_bounds__(kT) void rmsnorm_fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ r,
                                                         const WT* __restrict__ w, uint16_t* __restrict__ s,
                                                         uint16_t* __restrict__ y, float* __restrict__ rstd, int R,
                                                         int D, float eps) {
  const int nv = D / 8;
  PSAMD_ROW_LOOP(R) {
    const int64_t base = static_cast<int64_t>(row) * D;
    float v[VPT][8];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int vi = lane_ + k * kL;
      if (vi < nv) {
        load8(x, base + vi * 8, v[k]);
        if constexpr (RES) {
          float q[8];
          load8(r, base + vi * 8, q);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[k][j] = bf16_to_f32(f32_to_bf16(v[k][j] + q[j]));  // stream is bf16
          store8(s, base + vi * 8, v[k]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v[k][j] * v[k][j];
      }
    }
    const float rs = rsqrtf(wave_sum(ss) / static_cast<float>(D) + eps);
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int vi = lane_ + k * kL;
      if (vi < nv) {
        float wv[8];
        loadw8(w, vi * 8, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = bf16_to_f32(f32_to_bf16(v[k][j] * rs)) * wv[j];
        store8(y, base + vi * 8, v[k]);
      }
    }
    if (lane_ == 0) rstd[row] = rs;
  }
}

// dy, s: [R, D]; ds_in: optional gradient already flowing into s (residual branch);
// dx = rstd * (g - xhat * mean(g * xhat)) [+ ds_in], g = dy * w.  wpart: [gridDim.x, D].
template <int VPT, bool ADD, typename WT, bool WG = true>
__global__ __launch_bounds__(kT) void rmsnorm_bwd_kernel(const uint16_t* __restrict__ dy,
                                                         const uint16_t* __restrict__ s,
                                                         const WT* __restrict__ w, const float* __restrict__ rstd,
                                                         const uint16_t* __restrict__ ds_in,
                                                         uint16_t* __restrict__ dx, float* __restrict__ wpart, int R,
                                                         int D) {
  const int nv = D / 8;
  float acc[VPT][8];
#pragma unroll
  for (int k = 0; k < VPT; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  PSAMD_ROW_LOOP(R) {
    const int64_t base = static_cast<int64_t>(row) * D;
    const float rs = rstd[row];
    float xh[VPT][8], g[VPT][8];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int vi = lane_ + k * kL;
      if (vi < nv) {
        float d[8], wv[8];
        load8(dy, base + vi * 8, d);
        load8(s, base + vi * 8, xh[k]);
        loadw8(w, vi * 8, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[k][j] = bf16_to_f32(f32_to_bf16(xh[k][j] * rs));  // forward's rounded xhat
          if constexpr (WG) acc[k][j] += d[j] * xh[k][j];
          g[k][j] = d[j] * wv[j];
          dot += g[k][j] * xh[k][j];
        }
      }
    }
    const float c = wave_sum(dot) / static_cast<float>(D);
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int vi = lane_ + k * kL;
      if (vi < nv) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (g[k][j] - xh[k][j] * c);
        if constexpr (ADD) {
          float q[8];
          load8(ds_in, base + vi * 8, q);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += q[j];
        }
        store8(dx, base + vi * 8, o);
      }
    }
  }
  if constexpr (WG) {
    // fold the 4 waves' column partials in LDS (fixed wave order), one partial row per block
    __shared__ __attribute__((aligned(16))) float lacc[4096];
    block_fold_rows<VPT>(acc, lacc, D, wpart + static_cast<int64_t>(blockIdx.x) * D);
  }
}

// dx only, two passes over the row (the second re-reads dy / s from L2): nothing is held across
// the row reduction, so occupancy stays high for 4096-wide rows (holding xhat and g for
// 8 vectors per lane took 256 VGPRs, one wave per SIMD and serialised the HBM loads).
template <bool ADD, typename WT>
__global__ __launch_bounds__(kT) void rmsnorm_bwd_dx2_kernel(const uint16_t* __restrict__ dy,
                                                             const uint16_t* __restrict__ s, const WT* __restrict__ w,
                                                             const float* __restrict__ rstd,
                                                             const uint16_t* __restrict__ ds_in,
                                                             uint16_t* __restrict__ dx, int R, int D) {
  const int nv = D / 8;
  PSAMD_ROW_LOOP(R) {
    const int64_t base = static_cast<int64_t>(row) * D;
    const float rs = rstd[row];
    float dot = 0.f;
#pragma unroll 4
    for (int vi = lane_; vi < nv; vi += kL) {
      float d[8], x[8], wv[8];
      load8(dy, base + vi * 8, d);
      load8(s, base + vi * 8, x);
      loadw8(w, vi * 8, wv);
#pragma unroll
      for (int j = 0; j < 8; ++j) dot += d[j] * wv[j] * bf16_to_f32(f32_to_bf16(x[j] * rs));
    }
    const float c = wave_sum(dot) / static_cast<float>(D);
#pragma unroll 4
    for (int vi = lane_; vi < nv; vi += kL) {
      float d[8], x[8], wv[8], o[8];
      load8(dy, base + vi * 8, d);
      load8(s, base + vi * 8, x);
      loadw8(w, vi * 8, wv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = rs * (d[j] * wv[j] - bf16_to_f32(f32_to_bf16(x[j] * rs)) * c);
      if constexpr (ADD) {
        float q[8];
        load8(ds_in, base + vi * 8, q);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += q[j];
      }
      store8(dx, base + vi * 8, o);
    }
  }
}

// dw partials: part[y][c] = sum over row partition y (contiguous rows) of dy[r][c] *
// bf16(s[r][c] * rstd[r]), 8 columns per thread (grid: D / 2048 column blocks x P partitions)
__global__ __launch_bounds__(kT) void rms_dw_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ s,
                                                    const float* __restrict__ rstd, float* __restrict__ part, int R,
                                                    int D) {
  const int c = (blockIdx.x * kT + threadIdx.x) * 8;
  if (c >= D) return;
  const int P = gridDim.y, per = (R + P - 1) / P;  // a contiguous row range per partition
  const int r0 = blockIdx.y * per, r1 = min(R, r0 + per);
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 4
  for (int r = r0; r < r1; ++r) {
    const int64_t o = static_cast<int64_t>(r) * D + c;
    const float rs = rstd[r];
    float d[8], x[8];
    load8(dy, o, d);
    load8(s, o, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += d[j] * bf16_to_f32(f32_to_bf16(x[j] * rs));
  }
  store8(part, static_cast<int64_t>(blockIdx.y) * D + c, a);
}

// out[y][c] = sum_{b = y, y + Y, ...} part[b][c] (Y = gridDim.y), 8 independent chains per
// thread; fixed order.  Two launches (Y = 32, then Y = 1) reduce up to ~1000 partial rows.
__global__ __launch_bounds__(kT) void colsum_kernel(const float* __restrict__ part, int G, int D,
                                                    float* __restrict__ out) {
  const int c = blockIdx.x * kT + threadIdx.x;
  if (c >= D) return;
  const int Y = gridDim.y, y = blockIdx.y;
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int b = y;
  for (; b + 7 * Y < G; b += 8 * Y) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += part[static_cast<int64_t>(b + u * Y) * D + c];
  }
  for (; b < G; b += Y) a[0] += part[static_cast<int64_t>(b) * D + c];
  out[static_cast<int64_t>(y) * D + c] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

void colsum2(const float* part, int G, int D, float* mid, float* out, hipStream_t st) {
  const int Y = G < 32 ? G : 32;
  hipLaunchKernelGGL(colsum_kernel, dim3((D + kT - 1) / kT, Y), dim3(kT), 0, st, part, G, D, mid);
  hipLaunchKernelGGL(colsum_kernel, dim3((D + kT - 1) / kT, 1), dim3(kT), 0, st, mid, Y, D, out);
}

// ------------------------------------------------------------------------------ LayerNorm
// s = x + dropout_p(o) (written), y = LN(s) * gamma + beta.  mean/rstd: [R].
template <int VPT, bool DROP, typename WT>
__global__ __launch_bounds__(kT) void layernorm_fwd_kernel(const uint16_t* __restrict__ x,
                                                           const uint16_t* __restrict__ o,
                                                           const WT* __restrict__ gamma,
                                                           const WT* __restrict__ beta, uint16_t* __restrict__ s,
                                                           uint16_t* __restrict__ y, float* __restrict__ mean_out,
                                                           float* __restrict__ rstd_out, int R, int D, float eps,
                                                           float p, uint64_t seed) {
  const int nv = D / 8;
  PSAMD_ROW_LOOP(R) {
    const int64_t base = static_cast<int64_t>(row) * D;
    float v[VPT][8];
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int vi = lane_ + k * kL;
      if (vi < nv) {
        float q[8];
        load8(x, base + vi * 8, v[k]);
        load8(o, base + vi * 8, q);
        if constexpr (DROP) {
          float m[8];
          keep_mask8(seed, base + vi * 8, p, m);
#pragma unroll
          for (int j = 0; j < 8; ++j) q[j] *= m[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[k][j] = bf16_to_f32(f32_to_bf16(v[k][j] + q[j]));
          sum += v[k][j];
        }
        store8(s, base + vi * 8, v[k]);
      }
    }
    const float mu = wave_sum(sum) / static_cast<float>(D);
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int vi = lane_ + k * kL;
      if (vi < nv) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[k][j] - mu;
          sq += d * d;
        }
      }
    }
    const float rs = rsqrtf(wave_sum(sq) / static_cast<float>(D) + eps);
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int vi = lane_ + k * kL;
      if (vi < nv) {
        float ga[8], be[8];
        loadw8(gamma, vi * 8, ga);
        loadw8(beta, vi * 8, be);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = (v[k][j] - mu) * rs * ga[j] + be[j];
        store8(y, base + vi * 8, v[k]);
      }
    }
    if (lane_ == 0) {
      mean_out[row] = mu;
      rstd_out[row] = rs;
    }
  }
}

// ds = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma; dx = ds (residual input),
// do = ds * mask (dropout input).  part: [2, gridDim.x, D] (dgamma, dbeta).
template <int VPT, bool DROP, typename WT>
__global__ __launch_bounds__(kT) void layernorm_bwd_kernel(const uint16_t* __restrict__ dy,
                                                           const uint16_t* __restrict__ s,
                                                           const WT* __restrict__ gamma,
                                                           const float* __restrict__ mean_in,
                                                           const float* __restrict__ rstd_in,
                                                           uint16_t* __restrict__ dx, uint16_t* __restrict__ dout,
                                                           float* __restrict__ part, int64_t part_rows, int R, int D,
                                                           float p, uint64_t seed) {
  const int nv = D / 8;
  float ag[VPT][8], ab[VPT][8];
#pragma unroll
  for (int k = 0; k < VPT; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) ag[k][j] = ab[k][j] = 0.f;
  PSAMD_ROW_LOOP(R) {
    const int64_t base = static_cast<int64_t>(row) * D;
    const float mu = mean_in[row], rs = rstd_in[row];
    float xh[VPT][8], g[VPT][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int vi = lane_ + k * kL;
      if (vi < nv) {
        float d[8], ga[8];
        load8(dy, base + vi * 8, d);
        load8(s, base + vi * 8, xh[k]);
        loadw8(gamma, vi * 8, ga);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[k][j] = (xh[k][j] - mu) * rs;
          ag[k][j] += d[j] * xh[k][j];
          ab[k][j] += d[j];
          g[k][j] = d[j] * ga[j];
          s1 += g[k][j];
          s2 += g[k][j] * xh[k][j];
        }
      }
    }
    const float m1 = wave_sum(s1) / static_cast<float>(D);
    const float m2 = wave_sum(s2) / static_cast<float>(D);
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int vi = lane_ + k * kL;
      if (vi < nv) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (g[k][j] - m1 - xh[k][j] * m2);
        store8(dx, base + vi * 8, o);
        if constexpr (DROP) {
          float m[8];
          keep_mask8(seed, base + vi * 8, p, m);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] *= m[j];
        }
        store8(dout, base + vi * 8, o);
      }
    }
  }
  __shared__ __attribute__((aligned(16))) float lacc[4096];
  block_fold_rows<VPT>(ag, lacc, D, part + static_cast<int64_t>(blockIdx.x) * D);
  block_fold_rows<VPT>(ab, lacc, D, part + (part_rows + blockIdx.x) * D);
}

// ------------------------------------------------------------------------------ SwiGLU
// gu: [R, 2F] = [g | u]; h: [R, F] = silu(g) * u.  Backward: dg = dh * u * silu'(g),
// du = dh * silu(g), written into dgu [R, 2F].
__global__ __launch_bounds__(kT) void swiglu_fwd_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ h,
                                                        int64_t R, int F) {
  const int fv = F / 8;
  const int64_t n = R * fv;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kT;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x; i < n; i += stride) {
    const int64_t r = i / fv;
    const int c = static_cast<int>(i - r * fv) * 8;
    float g[8], u[8];
    load8(gu, r * 2 * F + c, g);
    load8(gu, r * 2 * F + F + c, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = g[j] / (1.f + __expf(-g[j])) * u[j];
    store8(h, r * F + c, g);
  }
}

__global__ __launch_bounds__(kT) void swiglu_bwd_kernel(const uint16_t* __restrict__ dh,
                                                        const uint16_t* __restrict__ gu,
                                                        uint16_t* __restrict__ dgu, int64_t R, int F) {
  const int fv = F / 8;
  const int64_t n = R * fv;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kT;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x; i < n; i += stride) {
    const int64_t r = i / fv;
    const int c = static_cast<int>(i - r * fv) * 8;
    float d[8], g[8], u[8];
    load8(dh, r * F + c, d);
    load8(gu, r * 2 * F + c, g);
    load8(gu, r * 2 * F + F + c, u);
    float dg[8], du[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = 1.f / (1.f + __expf(-g[j]));
      const float si = g[j] * sg;
      du[j] = d[j] * si;
      dg[j] = d[j] * u[j] * sg * (1.f + g[j] * (1.f - sg));
    }
    store8(dgu, r * 2 * F + c, dg);
    store8(dgu, r * 2 * F + F + c, du);
  }
}

// ------------------------------------------------------------------------------ RoPE + split
// qkv: [B, S, NH, hd] with NH = H + 2 KV (the fused QKV GEMM output); cs: [S, hd/2, 2] fp32
// (cos, sin).  q: [B, H, S, hd], k/v: [B, KV, S, hd].  Rotate-halves convention (Llama/HF):
// (x1, x2) -> (x1 c - x2 s, x2 c + x1 s) on the first H + KV heads, v copied.  One thread = 8
// dims of the first half and their 8 partners.
__global__ __launch_bounds__(kT) void rope_split_fwd_kernel(const uint16_t* __restrict__ qkv,
                                                            const float* __restrict__ cs, uint16_t* __restrict__ q,
                                                            uint16_t* __restrict__ k, uint16_t* __restrict__ v,
                                                            int B, int S, int H, int KV, int hd) {
  const int NH = H + 2 * KV, half = hd / 2, hv = half / 8;
  const int64_t n = static_cast<int64_t>(B) * S * NH * hv;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kT;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x; i < n; i += stride) {
    const int c = static_cast<int>(i % hv) * 8;
    int64_t t = i / hv;
    const int hh = static_cast<int>(t % NH);
    t /= NH;
    const int s = static_cast<int>(t % S);
    const int b = static_cast<int>(t / S);
    const uint16_t* src = qkv + ((static_cast<int64_t>(b) * S + s) * NH + hh) * hd;
    float x1[8], x2[8];
    load8(src, c, x1);
    load8(src, half + c, x2);
    uint16_t* dst;
    if (hh < H) dst = q + ((static_cast<int64_t>(b) * H + hh) * S + s) * hd;
    else if (hh < H + KV) dst = k + ((static_cast<int64_t>(b) * KV + (hh - H)) * S + s) * hd;
    else dst = v + ((static_cast<int64_t>(b) * KV + (hh - H - KV)) * S + s) * hd;
    if (hh < H + KV) {
      const float* cp = cs + (static_cast<int64_t>(s) * half + c) * 2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float co = cp[2 * j], si = cp[2 * j + 1];
        const float a = x1[j], bb = x2[j];
        x1[j] = a * co - bb * si;
        x2[j] = bb * co + a * si;
      }
    }
    store8(dst, c, x1);
    store8(dst, half + c, x2);
  }
}

__global__ __launch_bounds__(kT) void rope_split_bwd_kernel(const uint16_t* __restrict__ dq,
                                                            const uint16_t* __restrict__ dk,
                                                            const uint16_t* __restrict__ dv,
                                                            const float* __restrict__ cs,
                                                            uint16_t* __restrict__ dqkv, int B, int S, int H, int KV,
                                                            int hd) {
  const int NH = H + 2 * KV, half = hd / 2, hv = half / 8;
  const int64_t n = static_cast<int64_t>(B) * S * NH * hv;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kT;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x; i < n; i += stride) {
    const int c = static_cast<int>(i % hv) * 8;
    int64_t t = i / hv;
    const int hh = static_cast<int>(t % NH);
    t /= NH;
    const int s = static_cast<int>(t % S);
    const int b = static_cast<int>(t / S);
    const uint16_t* src;
    if (hh < H) src = dq + ((static_cast<int64_t>(b) * H + hh) * S + s) * hd;
    else if (hh < H + KV) src = dk + ((static_cast<int64_t>(b) * KV + (hh - H)) * S + s) * hd;
    else src = dv + ((static_cast<int64_t>(b) * KV + (hh - H - KV)) * S + s) * hd;
    float y1[8], y2[8];
    load8(src, c, y1);
    load8(src, half + c, y2);
    if (hh < H + KV) {  // transpose of the rotation
      const float* cp = cs + (static_cast<int64_t>(s) * half + c) * 2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float co = cp[2 * j], si = cp[2 * j + 1];
        const float a = y1[j], bb = y2[j];
        y1[j] = a * co + bb * si;
        y2[j] = bb * co - a * si;
      }
    }
    uint16_t* dst = dqkv + ((static_cast<int64_t>(b) * S + s) * NH + hh) * hd;
    store8(dst, c, y1);
    store8(dst, half + c, y2);
  }
}

// ------------------------------------------------------------------------------ launchers
namespace {
int row_grid(int R) { const int b = (R + 3) / 4; return b < 2048 ? b : 2048; }
int part_grid(int R) { const int b = (R + 3) / 4; return b < 1024 ? b : 1024; }  // one partial row per block
}  // namespace

#define PSAMD_VPT_SWITCH(D, BODY)                                  \
  do {                                                             \
    const int vpt_ = ((D) / 8 + kL - 1) / kL;                      \
    if (vpt_ <= 1) { constexpr int VPT = 1; BODY; }                \
    else if (vpt_ <= 2) { constexpr int VPT = 2; BODY; }           \
    else if (vpt_ <= 4) { constexpr int VPT = 4; BODY; }           \
    else { constexpr int VPT = 8; BODY; }                          \
  } while (0)

void launch_rmsnorm_fwd(const uint16_t* x, const uint16_t* r, const void* w, bool w_bf16, uint16_t* s, uint16_t* y,
                        float* rstd, int R, int D, float eps, hipStream_t st) {
  if (R <= 0) return;
  const int g = row_grid(R);
  PSAMD_VPT_SWITCH(D, {
    if (w_bf16) {
      if (r) hipLaunchKernelGGL((rmsnorm_fwd_kernel<VPT, true, uint16_t>), dim3(g), dim3(kT), 0, st, x, r,
                                static_cast<const uint16_t*>(w), s, y, rstd, R, D, eps);
      else hipLaunchKernelGGL((rmsnorm_fwd_kernel<VPT, false, uint16_t>), dim3(g), dim3(kT), 0, st, x, r,
                              static_cast<const uint16_t*>(w), s, y, rstd, R, D, eps);
    } else {
      if (r) hipLaunchKernelGGL((rmsnorm_fwd_kernel<VPT, true, float>), dim3(g), dim3(kT), 0, st, x, r,
                                static_cast<const float*>(w), s, y, rstd, R, D, eps);
      else hipLaunchKernelGGL((rmsnorm_fwd_kernel<VPT, false, float>), dim3(g), dim3(kT), 0, st, x, r,
                              static_cast<const float*>(w), s, y, rstd, R, D, eps);
    }
  });
}

int rmsnorm_bwd_parts(int R) { return part_grid(R) + 32; }  // + colsum scratch rows

void launch_rmsnorm_bwd(const uint16_t* dy, const uint16_t* s, const void* w, bool w_bf16, const float* rstd,
                        const uint16_t* ds_in, uint16_t* dx, float* wpart, float* dw, int R, int D, hipStream_t st) {
  if (R <= 0) return;
  if (D > 2048) {  // dx row kernel without weight-gradient registers + a row-partitioned dw reduction
    const int g = row_grid(R), P = part_grid(R) < 512 ? part_grid(R) : 512;
#define PSAMD_RMS_DX(ADDV, WTV) \
  hipLaunchKernelGGL((rmsnorm_bwd_dx2_kernel<ADDV, WTV>), dim3(g), dim3(kT), 0, st, dy, s, static_cast<const WTV*>(w), \
                     rstd, ds_in, dx, R, D)
    if (w_bf16) {
      if (ds_in) PSAMD_RMS_DX(true, uint16_t); else PSAMD_RMS_DX(false, uint16_t);
    } else {
      if (ds_in) PSAMD_RMS_DX(true, float); else PSAMD_RMS_DX(false, float);
    }
#undef PSAMD_RMS_DX
    hipLaunchKernelGGL(rms_dw_kernel, dim3((D / 8 + kT - 1) / kT, P), dim3(kT), 0, st, dy, s, rstd, wpart, R, D);
    colsum2(wpart, P, D, wpart + static_cast<int64_t>(P) * D, dw, st);
    return;
  }
  const int g = part_grid(R);
  PSAMD_VPT_SWITCH(D, {
    if (w_bf16) {
      if (ds_in) hipLaunchKernelGGL((rmsnorm_bwd_kernel<VPT, true, uint16_t>), dim3(g), dim3(kT), 0, st, dy, s,
                                    static_cast<const uint16_t*>(w), rstd, ds_in, dx, wpart, R, D);
      else hipLaunchKernelGGL((rmsnorm_bwd_kernel<VPT, false, uint16_t>), dim3(g), dim3(kT), 0, st, dy, s,
                              static_cast<const uint16_t*>(w), rstd, ds_in, dx, wpart, R, D);
    } else {
      if (ds_in) hipLaunchKernelGGL((rmsnorm_bwd_kernel<VPT, true, float>), dim3(g), dim3(kT), 0, st, dy, s,
                                    static_cast<const float*>(w), rstd, ds_in, dx, wpart, R, D);
      else hipLaunchKernelGGL((rmsnorm_bwd_kernel<VPT, false, float>), dim3(g), dim3(kT), 0, st, dy, s,
                              static_cast<const float*>(w), rstd, ds_in, dx, wpart, R, D);
    }
  });
  colsum2(wpart, g, D, wpart + static_cast<int64_t>(g) * D, dw, st);
}

void launch_layernorm_fwd(const uint16_t* x, const uint16_t* o, const void* gamma, const void* beta, bool w_bf16,
                          uint16_t* s, uint16_t* y, float* mean, float* rstd, int R, int D, float eps, float p,
                          uint64_t seed, hipStream_t st) {
  if (R <= 0) return;
  const int g = row_grid(R);
#define PSAMD_LN_F(DROP, WT)                                                                                      \
  hipLaunchKernelGGL((layernorm_fwd_kernel<VPT, DROP, WT>), dim3(g), dim3(kT), 0, st, x, o,                        \
                     static_cast<const WT*>(gamma), static_cast<const WT*>(beta), s, y, mean, rstd, R, D, eps, p, seed)
  PSAMD_VPT_SWITCH(D, {
    if (w_bf16) {
      if (p > 0.f) PSAMD_LN_F(true, uint16_t);
      else PSAMD_LN_F(false, uint16_t);
    } else {
      if (p > 0.f) PSAMD_LN_F(true, float);
      else PSAMD_LN_F(false, float);
    }
  });
#undef PSAMD_LN_F
}

int layernorm_bwd_parts(int R) { return part_grid(R) + 32; }

void launch_layernorm_bwd(const uint16_t* dy, const uint16_t* s, const void* gamma, bool w_bf16, const float* mean,
                          const float* rstd, uint16_t* dx, uint16_t* dout, float* part, float* dgamma, float* dbeta,
                          int R, int D, float p, uint64_t seed, hipStream_t st) {
  if (R <= 0) return;
  const int g = part_grid(R);
  const int64_t P = static_cast<int64_t>(g) + 32;  // rows per partial array (g partials + colsum scratch)
#define PSAMD_LN_B(DROP, WT)                                                                                    \
  hipLaunchKernelGGL((layernorm_bwd_kernel<VPT, DROP, WT>), dim3(g), dim3(kT), 0, st, dy, s,                     \
                     static_cast<const WT*>(gamma), mean, rstd, dx, dout, part, P, R, D, p, seed)
  PSAMD_VPT_SWITCH(D, {
    if (w_bf16) {
      if (p > 0.f) PSAMD_LN_B(true, uint16_t);
      else PSAMD_LN_B(false, uint16_t);
    } else {
      if (p > 0.f) PSAMD_LN_B(true, float);
      else PSAMD_LN_B(false, float);
    }
  });
#undef PSAMD_LN_B
  colsum2(part, g, D, part + static_cast<int64_t>(g) * D, dgamma, st);
  colsum2(part + P * D, g, D, part + (P + g) * D, dbeta, st);
}

void launch_swiglu_fwd(const uint16_t* gu, uint16_t* h, int64_t R, int F, hipStream_t st) {
  if (R <= 0) return;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(stream_grid(R * (F / 8), kT)), dim3(kT), 0, st, gu, h, R, F);
}

void launch_swiglu_bwd(const uint16_t* dh, const uint16_t* gu, uint16_t* dgu, int64_t R, int F, hipStream_t st) {
  if (R <= 0) return;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(stream_grid(R * (F / 8), kT)), dim3(kT), 0, st, dh, gu, dgu, R, F);
}

void launch_rope_split_fwd(const uint16_t* qkv, const float* cs, uint16_t* q, uint16_t* k, uint16_t* v, int B, int S,
                           int H, int KV, int hd, hipStream_t st) {
  const int64_t n = static_cast<int64_t>(B) * S * (H + 2 * KV) * (hd / 16);
  if (n <= 0) return;
  hipLaunchKernelGGL(rope_split_fwd_kernel, dim3(stream_grid(n, kT)), dim3(kT), 0, st, qkv, cs, q, k, v, B, S, H, KV,
                     hd);
}

void launch_rope_split_bwd(const uint16_t* dq, const uint16_t* dk, const uint16_t* dv, const float* cs,
                           uint16_t* dqkv, int B, int S, int H, int KV, int hd, hipStream_t st) {
  const int64_t n = static_cast<int64_t>(B) * S * (H + 2 * KV) * (hd / 16);
  if (n <= 0) return;
  hipLaunchKernelGGL(rope_split_bwd_kernel, dim3(stream_grid(n, kT)), dim3(kT), 0, st, dq, dk, dv, cs, dqkv, B, S, H,
                     KV, hd);
}

#undef PSAMD_VPT_SWITCH

}  // namespace psamd
