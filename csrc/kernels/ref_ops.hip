// Reference-model ops (K3, K4, K11, K12, K15, K17, K18, K28 in SURVEY §2.5).
//
//  softmax_temp_fwd   softmax(x / T) per row with the reference's clamps
//                     (activations/Softmax.java:11-40: subtract max, T = 10000, 0 -> 0.001,
//                     1 -> 0.999).  One wave per row; rows = samples (batch-major layout).
//  softmax_xent       fused -log p[label] and dL/dp for SoftmaxLoss (loss/SoftmaxLoss.java:9-28)
//                     plus the batch-mean loss (single atomic per block).
//  bce                mean BCE + grad (p - y)/(p(1-p)) (loss/CrossEntropy.java:10-28)
//  maxpool2d          2D max pool with the argmax stored per output (layer/PoolingLayer.java:62-101)
//                     and an ACCUMULATING backward (fixes Q9: reference overwrites, :129)
//  im2col / col2im    (layer/Conv2DLayer.java:94-127, 185-217); col2im is a gather over the
//                     output positions that touch each input pixel: no atomics.
//  dropout            philox mask regenerated from (seed, offset) in backward: the mask is
//                     never stored (layer/DropoutLayer.java:23-53; keep-prob semantics fixed, Q10)
//  uniform_init       U(lo, hi) keyed by (seed, offset + i) (util/MatrixUtil.java:62-74)
#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

__global__ __launch_bounds__(256) void softmax_temp_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                               int64_t rows, int cols, float inv_temp, float clamp_lo,
                                                               float clamp_hi) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t r = wave; r < rows; r += nwaves) {
    const float* xr = x + r * cols;
    float m = -INFINITY;
    for (int c = lane; c < cols; c += 64) m = fmaxf(m, xr[c] * inv_temp);
    m = wave_max(m);
    float s = 0.f;
    for (int c = lane; c < cols; c += 64) s += __expf(xr[c] * inv_temp - m);
    s = wave_sum(s);
    const float inv = 1.f / s;
    for (int c = lane; c < cols; c += 64) {
      float p = __expf(xr[c] * inv_temp - m) * inv;
      if (clamp_lo > 0.f && p <= 0.f) p = clamp_lo;
      if (clamp_hi < 1.f && p >= 1.f) p = clamp_hi;
      y[r * cols + c] = p;
    }
  }
}

void launch_softmax_temp_fwd(const float* x, float* y, int64_t rows, int cols, float inv_temp, float clamp_lo,
                             float clamp_hi, hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(softmax_temp_fwd_kernel, dim3(stream_grid(rows * 64, 256)), dim3(256), 0, s, x, y, rows, cols,
                     inv_temp, clamp_lo, clamp_hi);
}

// Softmax backward (Jacobian-vector product, activations/Softmax.java:45-67): one wave per row,
// dx = scale * p * (dy - sum_c dy_c p_c); scale = 1 reproduces the reference (which omits the
// 1/T of the temperature, Q15), scale = 1/T is the exact gradient.
__global__ __launch_bounds__(256) void softmax_temp_bwd_kernel(const float* __restrict__ p, const float* __restrict__ dy,
                                                               float* __restrict__ dx, int64_t rows, int cols,
                                                               float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t r = wave; r < rows; r += nwaves) {
    const float* pr = p + r * cols;
    const float* gr = dy + r * cols;
    float d = 0.f;
    for (int c = lane; c < cols; c += 64) d += gr[c] * pr[c];
    d = wave_sum(d);
    for (int c = lane; c < cols; c += 64) dx[r * cols + c] = scale * pr[c] * (gr[c] - d);
  }
}

void launch_softmax_temp_bwd(const float* p, const float* dy, float* dx, int64_t rows, int cols, float scale,
                             hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(softmax_temp_bwd_kernel, dim3(stream_grid(rows * 64, 256)), dim3(256), 0, s, p, dy, dx, rows,
                     cols, scale);
}

// loss (scalar, pre-zeroed) += -mean log p[label]; grad[r, c] = (c == label) ? -1/p / rows : 0
__global__ __launch_bounds__(256) void softmax_xent_kernel(const float* __restrict__ p, const int64_t* __restrict__ labels,
                                                           int64_t rows, int cols, float* __restrict__ loss,
                                                           float* __restrict__ grad) {
  __shared__ float scratch[4];
  float acc = 0.f;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t total = rows * cols;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t r = i / cols;
    const int c = static_cast<int>(i - r * cols);
    const bool hot = labels[r] == c;
    const float pv = p[i];
    if (hot) acc += -__logf(pv);
    if (grad) grad[i] = hot ? (-1.f / pv) / static_cast<float>(rows) : 0.f;
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0 && loss) atomicAdd(loss, acc / static_cast<float>(rows));
}

void launch_softmax_xent(const float* p, const int64_t* labels, int64_t rows, int cols, float* loss, float* grad,
                         hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(stream_grid(rows * cols, 256)), dim3(256), 0, s, p, labels, rows, cols,
                     loss, grad);
}

__global__ __launch_bounds__(256) void bce_kernel(const float* __restrict__ p, const float* __restrict__ y, int64_t n,
                                                  float* __restrict__ loss, float* __restrict__ grad) {
  __shared__ float scratch[4];
  float acc = 0.f;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float pv = p[i], yv = y[i];
    acc += -(yv * __logf(pv) + (1.f - yv) * __logf(1.f - pv));
    if (grad) grad[i] = (pv - yv) / (pv * (1.f - pv)) / static_cast<float>(n);
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0 && loss) atomicAdd(loss, acc / static_cast<float>(n));
}

void launch_bce(const float* p, const float* y, int64_t n, float* loss, float* grad, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(bce_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, s, p, y, n, loss, grad);
}

// NCHW max pool; padding positions are -inf (fixes Q9's index-0 padding).  argmax is the flat
// h*w index inside the (n, c) plane, -1 if the window is entirely padding.
template <typename T>
__global__ __launch_bounds__(256) void maxpool2d_fwd_kernel(const T* __restrict__ x, int64_t nc, int h, int w, int k,
                                                            int stride, int pad, T* __restrict__ y,
                                                            int32_t* __restrict__ argmax, int oh, int ow) {
  const int64_t total = nc * oh * ow;
  const int64_t gs = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += gs) {
    const int64_t plane = i / (oh * ow);
    const int rem = static_cast<int>(i - plane * oh * ow);
    const int oy = rem / ow, ox = rem - (rem / ow) * ow;
    const T* xp = x + plane * h * w;
    float best = -INFINITY;
    int bi = -1;
    for (int ky = 0; ky < k; ++ky) {
      const int iy = oy * stride - pad + ky;
      if (iy < 0 || iy >= h) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int ix = ox * stride - pad + kx;
        if (ix < 0 || ix >= w) continue;
        const float v = Elem<T>::load(xp, iy * w + ix);
        if (v > best || bi < 0) { best = v; bi = iy * w + ix; }
      }
    }
    Elem<T>::store(y, i, bi < 0 ? 0.f : best);
    argmax[i] = bi;
  }
}

// gather formulation: each input pixel sums dy over the outputs whose argmax points at it
template <typename T>
__global__ __launch_bounds__(256) void maxpool2d_bwd_kernel(const T* __restrict__ dy, const int32_t* __restrict__ argmax,
                                                            int64_t nc, int h, int w, int oh, int ow, int k, int stride,
                                                            int pad, T* __restrict__ dx) {
  const int64_t total = nc * h * w;
  const int64_t gs = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += gs) {
    const int64_t plane = i / (h * w);
    const int pix = static_cast<int>(i - plane * h * w);
    const int iy = pix / w, ix = pix - (pix / w) * w;
    // outputs whose window covers (iy, ix): oy in [ceil((iy+pad-k+1)/stride), (iy+pad)/stride]
    const int oy0 = max(0, (iy + pad - k + stride) / stride), oy1 = min(oh - 1, (iy + pad) / stride);
    const int ox0 = max(0, (ix + pad - k + stride) / stride), ox1 = min(ow - 1, (ix + pad) / stride);
    float acc = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy)
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int64_t o = plane * oh * ow + oy * ow + ox;
        if (argmax[o] == pix) acc += Elem<T>::load(dy, o);
      }
    Elem<T>::store(dx, i, acc);
  }
}

void launch_maxpool2d_fwd(const void* x, int dtype, int64_t nc, int h, int w, int k, int stride, int pad, void* y,
                          int32_t* argmax, int oh, int ow, hipStream_t s) {
  const int64_t total = nc * oh * ow;
  if (total <= 0) return;
  const int grid = stream_grid(total, 256);
  if (dtype == 1)
    hipLaunchKernelGGL(maxpool2d_fwd_kernel<uint16_t>, dim3(grid), dim3(256), 0, s, static_cast<const uint16_t*>(x), nc,
                       h, w, k, stride, pad, static_cast<uint16_t*>(y), argmax, oh, ow);
  else
    hipLaunchKernelGGL(maxpool2d_fwd_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<const float*>(x), nc, h, w,
                       k, stride, pad, static_cast<float*>(y), argmax, oh, ow);
}

void launch_maxpool2d_bwd(const void* dy, int dtype, const int32_t* argmax, int64_t nc, int h, int w, int oh, int ow,
                          int k, int stride, int pad, void* dx, hipStream_t s) {
  const int64_t total = nc * h * w;
  if (total <= 0) return;
  const int grid = stream_grid(total, 256);
  if (dtype == 1)
    hipLaunchKernelGGL(maxpool2d_bwd_kernel<uint16_t>, dim3(grid), dim3(256), 0, s, static_cast<const uint16_t*>(dy),
                       argmax, nc, h, w, oh, ow, k, stride, pad, static_cast<uint16_t*>(dx));
  else
    hipLaunchKernelGGL(maxpool2d_bwd_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<const float*>(dy), argmax,
                       nc, h, w, oh, ow, k, stride, pad, static_cast<float*>(dx));
}

// col layout: [n, oh*ow, c*k*k]  (rows = output positions, cols = patch) -> GEMM-ready
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ x, int64_t n, int c, int h, int w, int k,
                                                     int stride, int pad, int oh, int ow, float* __restrict__ col) {
  const int64_t patch = static_cast<int64_t>(c) * k * k;
  const int64_t total = n * oh * ow * patch;
  const int64_t gs = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += gs) {
    const int64_t row = i / patch;
    const int pc = static_cast<int>(i - row * patch);
    const int64_t b = row / (oh * ow);
    const int pos = static_cast<int>(row - b * oh * ow);
    const int oy = pos / ow, ox = pos - (pos / ow) * ow;
    const int ch = pc / (k * k), kk = pc - (pc / (k * k)) * k * k;
    const int ky = kk / k, kx = kk - (kk / k) * k;
    const int iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
    float v = 0.f;
    if (iy >= 0 && iy < h && ix >= 0 && ix < w) v = x[((b * c + ch) * h + iy) * w + ix];
    col[i] = v;
  }
}

__global__ __launch_bounds__(256) void col2im_kernel(const float* __restrict__ col, int64_t n, int c, int h, int w, int k,
                                                     int stride, int pad, int oh, int ow, float* __restrict__ x) {
  const int64_t total = n * c * h * w;
  const int64_t patch = static_cast<int64_t>(c) * k * k;
  const int64_t gs = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += gs) {
    const int64_t b = i / (static_cast<int64_t>(c) * h * w);
    int rem = static_cast<int>(i - b * c * h * w);
    const int ch = rem / (h * w);
    rem -= ch * h * w;
    const int iy = rem / w, ix = rem - (rem / w) * w;
    float acc = 0.f;
    for (int ky = 0; ky < k; ++ky) {
      const int ty = iy + pad - ky;
      if (ty < 0 || ty % stride) continue;
      const int oy = ty / stride;
      if (oy >= oh) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int tx = ix + pad - kx;
        if (tx < 0 || tx % stride) continue;
        const int ox = tx / stride;
        if (ox >= ow) continue;
        acc += col[(b * oh * ow + oy * ow + ox) * patch + (ch * k + ky) * k + kx];
      }
    }
    x[i] = acc;
  }
}

void launch_im2col(const float* x, int64_t n, int c, int h, int w, int k, int stride, int pad, int oh, int ow,
                   float* col, hipStream_t s) {
  const int64_t total = n * oh * ow * c * k * k;
  if (total <= 0) return;
  hipLaunchKernelGGL(im2col_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, s, x, n, c, h, w, k, stride, pad, oh,
                     ow, col);
}

void launch_col2im(const float* col, int64_t n, int c, int h, int w, int k, int stride, int pad, int oh, int ow,
                   float* x, hipStream_t s) {
  const int64_t total = n * c * h * w;
  if (total <= 0) return;
  hipLaunchKernelGGL(col2im_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, s, col, n, c, h, w, k, stride, pad, oh,
                     ow, x);
}

// keep with probability (1 - p_drop), scale kept values by 1/(1 - p_drop)
template <typename T>
__global__ __launch_bounds__(256) void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                      float p_drop, uint64_t seed, uint64_t offset) {
  const float keep_scale = 1.f / (1.f - p_drop);
  const int64_t gs = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; q * 4 < n; q += gs) {
    uint32_t r[4];
    Philox::gen(seed, offset + static_cast<uint64_t>(q), r);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t i = q * 4 + j;
      if (i < n) {
        const bool keep = Philox::u01(r[j]) >= p_drop;
        Elem<T>::store(y, i, keep ? Elem<T>::load(x, i) * keep_scale : 0.f);
      }
    }
  }
}

void launch_dropout_fwd(const void* x, int dtype, void* y, int64_t n, float p_drop, uint64_t seed, uint64_t offset,
                        hipStream_t s) {
  if (n <= 0) return;
  const int grid = stream_grid((n + 3) / 4, 256);
  if (dtype == 1)
    hipLaunchKernelGGL(dropout_kernel<uint16_t>, dim3(grid), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                       static_cast<uint16_t*>(y), n, p_drop, seed, offset);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<const float*>(x),
                       static_cast<float*>(y), n, p_drop, seed, offset);
}

void launch_dropout_bwd(const void* dy, int dtype, void* dx, int64_t n, float p_drop, uint64_t seed, uint64_t offset,
                        hipStream_t s) {
  // identical mask & scale: backward of y = m * x / (1-p) is dx = m * dy / (1-p)
  launch_dropout_fwd(dy, dtype, dx, n, p_drop, seed, offset, s);
}

__global__ __launch_bounds__(256) void uniform_init_kernel(float* __restrict__ w, int64_t n, uint64_t seed,
                                                           uint64_t offset, float lo, float hi) {
  const int64_t gs = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; q * 4 < n; q += gs) {
    uint32_t r[4];
    Philox::gen(seed, offset + static_cast<uint64_t>(q), r);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (q * 4 + j < n) w[q * 4 + j] = lo + (hi - lo) * Philox::u01(r[j]);
  }
}

void launch_uniform_init(float* w, int64_t n, uint64_t seed, uint64_t offset, float lo, float hi, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(uniform_init_kernel, dim3(stream_grid((n + 3) / 4, 256)), dim3(256), 0, s, w, n, seed, offset, lo,
                     hi);
}

}  // namespace psamd
