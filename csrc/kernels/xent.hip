// Fused softmax cross-entropy over bf16 logits (the LM heads of BERT-MLM and Llama): vocab rows of
// 30522 / 128256 logits are the largest activations of those steps, and the unfused path (cast to
// fp32, log-softmax, NLL, their backward) makes ~8 fp32 passes over them.  Here:
//   forward   one pass per row: online max / sum-exp over 16-B pieces -> lse[r]; loss[r] =
//             lse - x[label] (0 for ignored rows); the caller sums loss rows (fixed order).
//   backward  one pass: dx = (exp(x - lse) - [j == label]) * go / count, bf16, 0 for ignored rows.
// One 256-thread block per row; the row stays L2-resident between the two passes of nothing --
// each pass reads it once.  Reference role: the SoftmaxLoss / CrossEntropy of the reference models
// (loss/SoftmaxLoss.java:9-28) at LM-head scale.
#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {
namespace {

__device__ __forceinline__ void block_max_sum(float& m, float& s, float* red) {
  // combine (m, s) pairs: s is a sum of exp(x - m)
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
    m = mn;
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    red[2 * w] = m;
    red[2 * w + 1] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = red[0], S = red[1];
    for (int i = 1; i < static_cast<int>(blockDim.x >> 6); ++i) {
      const float m2 = red[2 * i], s2 = red[2 * i + 1], mn = fmaxf(M, m2);
      S = (M == -INFINITY ? 0.f : S * __expf(M - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
      M = mn;
    }
    red[0] = M;
    red[1] = S;
  }
  __syncthreads();
  m = red[0];
  s = red[1];
}

__global__ __launch_bounds__(256) void xent_fwd_kernel(const uint16_t* __restrict__ x, const int64_t* __restrict__ lab,
                                                       int64_t R, int V, int64_t ignore, float* __restrict__ lse,
                                                       float* __restrict__ loss) {
  __shared__ float red[8];
  const int64_t r = blockIdx.x;
  const uint16_t* row = x + r * V;
  float m = -INFINITY, s = 0.f;
  const bool vec = (V & 7) == 0;
  auto acc = [&](float v) {
    if (v > m) {
      s = s * __expf(m - v) + 1.f;
      m = v;
    } else {
      s += __expf(v - m);
    }
  };
  if (vec) {
    for (int i = threadIdx.x * 8; i < V; i += blockDim.x * 8) {
      const u16x8 q = *reinterpret_cast<const u16x8*>(row + i);
      float f[8], lm = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f[j] = bf16_to_f32(q[j]);
        lm = fmaxf(lm, f[j]);
      }
      // one rescale per 8 values
      if (lm > m) {
        s *= __expf(m - lm);
        m = lm;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(f[j] - m);
    }
  } else {
    for (int i = threadIdx.x; i < V; i += blockDim.x) acc(bf16_to_f32(row[i]));
  }
  block_max_sum(m, s, red);
  if (threadIdx.x == 0) {
    const float l = m + __logf(s);
    lse[r] = l;
    const int64_t y = lab[r];
    loss[r] = (y == ignore || y < 0 || y >= V) ? 0.f : l - bf16_to_f32(row[y]);
  }
}

__global__ __launch_bounds__(256) void xent_bwd_kernel(const uint16_t* __restrict__ x, const int64_t* __restrict__ lab,
                                                       const float* __restrict__ lse, int V, int64_t ignore,
                                                       const float* __restrict__ go, const float* __restrict__ count,
                                                       uint16_t* __restrict__ dx) {
  const int64_t r = blockIdx.x;
  const uint16_t* row = x + r * V;
  uint16_t* out = dx + r * V;
  const int64_t y = lab[r];
  const bool skip = y == ignore || y < 0 || y >= V;
  const float k = skip ? 0.f : go[0] / fmaxf(count[0], 1.f);
  const float l = lse[r];
  if ((V & 7) == 0) {
    for (int i = threadIdx.x * 8; i < V; i += blockDim.x * 8) {
      u16x8 o;
      if (skip) {
        o = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      } else {
        const u16x8 q = *reinterpret_cast<const u16x8*>(row + i);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float p = __expf(bf16_to_f32(q[j]) - l) - (i + j == y ? 1.f : 0.f);
          o[j] = f32_to_bf16(p * k);
        }
      }
      *reinterpret_cast<u16x8*>(out + i) = o;
    }
  } else {
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const float p = skip ? 0.f : (__expf(bf16_to_f32(row[i]) - l) - (i == y ? 1.f : 0.f)) * k;
      out[i] = f32_to_bf16(p);
    }
  }
}

}  // namespace

void launch_xent_fwd(const uint16_t* x, const int64_t* lab, int64_t R, int V, int64_t ignore, float* lse, float* loss,
                     hipStream_t s) {
  if (R <= 0) return;
  hipLaunchKernelGGL(xent_fwd_kernel, dim3(static_cast<unsigned>(R)), dim3(256), 0, s, x, lab, R, V, ignore, lse, loss);
}

void launch_xent_bwd(const uint16_t* x, const int64_t* lab, const float* lse, int64_t R, int V, int64_t ignore,
                     const float* go, const float* count, uint16_t* dx, hipStream_t s) {
  if (R <= 0) return;
  hipLaunchKernelGGL(xent_bwd_kernel, dim3(static_cast<unsigned>(R)), dim3(256), 0, s, x, lab, lse, V, ignore, go,
                     count, dx);
}

}  // namespace psamd
