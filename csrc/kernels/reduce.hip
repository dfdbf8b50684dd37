// Bucket / reduction kernels (K19, K20, K25, K27 in SURVEY §2.5).
//
//  * sumsq_partial + sumsq_finish: deterministic two-pass global squared L2 norm of a flat
//    gradient shard (reference has no clipping; north-star K25). Each block writes one
//    partial; the finisher sums partials in a fixed order, so the result is bitwise
//    reproducible run to run (no float atomics).
//  * clip_factor: min(1, max_norm / (sqrt(sumsq) + 1e-6)) written to device memory so the
//    optimizer kernel reads it without a host sync.
//  * cast / axpy / reduce_n: bucket accumulation (store/KVStore.java:192-200 `sum` and the
//    divide-by-count at :253) and the server-side N-way reduce of worker pushes
//    (net/PServer.java:178,186).
//  * lerp: loss-surface interpolation w = s*w0 + (1-s)*w (store/KVStore.java:153-155).
#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

template <typename T>
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const T* __restrict__ x, int64_t n,
                                                             float* __restrict__ partial) {
  __shared__ float scratch[4];
  float acc = 0.f;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x * 8;
  const int64_t nv = (n / 8) * 8;
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 8; i < nv; i += stride) {
    float v[8];
    load8(x, i, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j] * v[j];
  }
  if (blockIdx.x == 0)
    for (int64_t i = nv + threadIdx.x; i < n; i += blockDim.x) {
      const float v = Elem<T>::load(x, i);
      acc += v * v;
    }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

template <typename T>
__global__ __launch_bounds__(256) void sumsq_partial_scalar_kernel(const T* __restrict__ x, int64_t n,
                                                                    float* __restrict__ partial) {
  __shared__ float scratch[4];
  float acc = 0.f;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = Elem<T>::load(x, i);
    acc += v * v;
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

int sumsq_blocks(int64_t n) { return stream_grid((n + 7) / 8, 256) > 1024 ? 1024 : stream_grid((n + 7) / 8, 256); }

void launch_sumsq_partial(const void* x, int dtype, int64_t n, float* partial, int nblocks, hipStream_t s) {
  const bool aligned = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  if (dtype == 1) {
    if (aligned)
      hipLaunchKernelGGL(sumsq_partial_kernel<uint16_t>, dim3(nblocks), dim3(256), 0, s,
                         static_cast<const uint16_t*>(x), n, partial);
    else
      hipLaunchKernelGGL(sumsq_partial_scalar_kernel<uint16_t>, dim3(nblocks), dim3(256), 0, s,
                         static_cast<const uint16_t*>(x), n, partial);
  } else {
    if (aligned)
      hipLaunchKernelGGL(sumsq_partial_kernel<float>, dim3(nblocks), dim3(256), 0, s, static_cast<const float*>(x),
                         n, partial);
    else
      hipLaunchKernelGGL(sumsq_partial_scalar_kernel<float>, dim3(nblocks), dim3(256), 0, s,
                         static_cast<const float*>(x), n, partial);
  }
}

__global__ __launch_bounds__(256) void sumsq_finish_kernel(const float* __restrict__ partial, int nblocks,
                                                            float* __restrict__ out, int accumulate) {
  __shared__ float scratch[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nblocks; i += blockDim.x) acc += partial[i];
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) *out = accumulate ? (*out + acc) : acc;
}

void launch_sumsq_finish(const float* partial, int nblocks, float* out, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(sumsq_finish_kernel, dim3(1), dim3(256), 0, s, partial, nblocks, out, accumulate);
}

__global__ void clip_factor_kernel(const float* __restrict__ sumsq, float max_norm, float* __restrict__ factor) {
  if (threadIdx.x == 0) {
    const float norm = sqrtf(*sumsq);
    const float f = max_norm / (norm + 1e-6f);
    *factor = f < 1.f ? f : 1.f;
  }
}

void launch_clip_factor(const float* sumsq, float max_norm, float* factor, hipStream_t s) {
  hipLaunchKernelGGL(clip_factor_kernel, dim3(1), dim3(64), 0, s, sumsq, max_norm, factor);
}

// ------------------------------------------------------------------- elementwise family
template <typename X, typename Y>
__global__ __launch_bounds__(256) void cast_kernel(const X* __restrict__ x, Y* __restrict__ y, int64_t n, float scale,
                                                   bool vec) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (vec) {
    const int64_t nv = n / 8;
    for (int64_t v = tid; v < nv; v += stride) {
      float r[8];
      load8(x, v * 8, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] *= scale;
      store8(y, v * 8, r);
    }
    for (int64_t i = nv * 8 + tid; i < n; i += stride) Elem<Y>::store(y, i, Elem<X>::load(x, i) * scale);
  } else {
    for (int64_t i = tid; i < n; i += stride) Elem<Y>::store(y, i, Elem<X>::load(x, i) * scale);
  }
}

template <typename X, typename Y>
__global__ __launch_bounds__(256) void axpy_kernel(float a, const X* __restrict__ x, Y* __restrict__ y, int64_t n,
                                                   bool vec) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (vec) {
    const int64_t nv = n / 8;
    for (int64_t v = tid; v < nv; v += stride) {
      float xr[8], yr[8];
      load8(x, v * 8, xr);
      load8(y, v * 8, yr);
#pragma unroll
      for (int j = 0; j < 8; ++j) yr[j] += a * xr[j];
      store8(y, v * 8, yr);
    }
    for (int64_t i = nv * 8 + tid; i < n; i += stride) Elem<Y>::store(y, i, Elem<Y>::load(y, i) + a * Elem<X>::load(x, i));
  } else {
    for (int64_t i = tid; i < n; i += stride) Elem<Y>::store(y, i, Elem<Y>::load(y, i) + a * Elem<X>::load(x, i));
  }
}

// y[i] = scale * sum_k x[k*n + i]   (k worker buffers laid out contiguously; fixed order)
template <typename X, typename Y>
__global__ __launch_bounds__(256) void reduce_n_kernel(const X* __restrict__ x, int k, int64_t n, Y* __restrict__ y,
                                                       float scale, bool vec) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (vec) {
    const int64_t nv = n / 8;
    for (int64_t v = tid; v < nv; v += stride) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int w = 0; w < k; ++w) {
        float r[8];
        load8(x + static_cast<int64_t>(w) * n, v * 8, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += r[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= scale;
      store8(y, v * 8, acc);
    }
    for (int64_t i = nv * 8 + tid; i < n; i += stride) {
      float acc = 0.f;
      for (int w = 0; w < k; ++w) acc += Elem<X>::load(x + static_cast<int64_t>(w) * n, i);
      Elem<Y>::store(y, i, acc * scale);
    }
  } else {
    for (int64_t i = tid; i < n; i += stride) {
      float acc = 0.f;
      for (int w = 0; w < k; ++w) acc += Elem<X>::load(x + static_cast<int64_t>(w) * n, i);
      Elem<Y>::store(y, i, acc * scale);
    }
  }
}

template <typename Y>
__global__ __launch_bounds__(256) void lerp_kernel(const float* __restrict__ w0, const float* __restrict__ w, float sc,
                                                   Y* __restrict__ out, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    Elem<Y>::store(out, i, sc * w0[i] + (1.f - sc) * w[i]);
}

static inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

#define PSAMD_DT2(xd, yd, FN)                          \
  if ((xd) == 1 && (yd) == 1) FN(uint16_t, uint16_t)   \
  else if ((xd) == 1 && (yd) == 0) FN(uint16_t, float) \
  else if ((xd) == 0 && (yd) == 1) FN(float, uint16_t) \
  else FN(float, float)

void launch_cast(const void* x, int xdtype, void* y, int ydtype, int64_t n, float scale, hipStream_t s) {
  if (n <= 0) return;
  const bool vec = al16(x) && al16(y);
  const int grid = stream_grid(vec ? (n + 7) / 8 : n, 256);
#define PSAMD_CAST(X, Y) \
  hipLaunchKernelGGL((cast_kernel<X, Y>), dim3(grid), dim3(256), 0, s, static_cast<const X*>(x), static_cast<Y*>(y), n, scale, vec);
  PSAMD_DT2(xdtype, ydtype, PSAMD_CAST)
#undef PSAMD_CAST
}

void launch_axpy(float a, const void* x, int xdtype, void* y, int ydtype, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  const bool vec = al16(x) && al16(y);
  const int grid = stream_grid(vec ? (n + 7) / 8 : n, 256);
#define PSAMD_AXPY(X, Y) \
  hipLaunchKernelGGL((axpy_kernel<X, Y>), dim3(grid), dim3(256), 0, s, a, static_cast<const X*>(x), static_cast<Y*>(y), n, vec);
  PSAMD_DT2(xdtype, ydtype, PSAMD_AXPY)
#undef PSAMD_AXPY
}

void launch_reduce_n(const void* x, int xdtype, int k, int64_t n, void* y, int ydtype, float scale, hipStream_t s) {
  if (n <= 0) return;
  const bool vec = al16(x) && al16(y) && (n % 8 == 0);
  const int grid = stream_grid(vec ? (n + 7) / 8 : n, 256);
#define PSAMD_RED(X, Y) \
  hipLaunchKernelGGL((reduce_n_kernel<X, Y>), dim3(grid), dim3(256), 0, s, static_cast<const X*>(x), k, n, static_cast<Y*>(y), scale, vec);
  PSAMD_DT2(xdtype, ydtype, PSAMD_RED)
#undef PSAMD_RED
}

void launch_lerp(const float* w0, const float* w, float sc, void* out, int odtype, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  const int grid = stream_grid(n, 256);
  if (odtype == 1)
    hipLaunchKernelGGL(lerp_kernel<uint16_t>, dim3(grid), dim3(256), 0, s, w0, w, sc, static_cast<uint16_t*>(out), n);
  else
    hipLaunchKernelGGL(lerp_kernel<float>, dim3(grid), dim3(256), 0, s, w0, w, sc, static_cast<float*>(out), n);
}

}  // namespace psamd
