// Fused server-side optimizers for the parameter-server shards (K21-K24 in SURVEY §2.5).
//
// Every kernel is one pass over a flat, range-partitioned shard: fp32 master weights and
// fp32 optimizer state live on the owning rank, the pushed gradient arrives as bf16 or fp32
// (reduce-scatter output), and the kernel optionally writes the updated weights straight
// into the bf16/fp32 "pull" buffer that the following all-gather broadcasts.  One read of
// each operand and one write of each result: these kernels are HBM-bound, so the only
// levers are 16-byte-per-lane accesses, a grid that fills 256 CUs, and fusing the gradient
// scale (1/world, clip coefficient) into the same pass.
//
// Reference semantics (file:line in /root/reference/src/main/java):
//   SGD          update/SimpleUpdater.java:20-22        w += -eta * dw
//   Adam         update/AdamUpdater.java:57-70          bias correction by the CONSTANT (1-beta)
//                                                        (Q5) -> bias_mode = 2; standard (1-beta^t) = 1
//   FTRL         update/FtrlUpdater.java:51-76           reference ordering/sigma (Q6) -> ftrl_mode = 1;
//                                                        canonical McMahan FTRL-proximal -> ftrl_mode = 0
//   Adagrad      (north-star, DLRM tables)
#include <cstdlib>

#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

// Dense optimizer grid: stream_grid (a cap on the grid, to leave CUs to an overlapping backward,
// measured no better: profiles/r4_llama_serve_overlap.txt).
static int opt_grid(int64_t work_items, int block) { return stream_grid(work_items, block); }

enum OptKind : int { kSGD = 0, kAdam = 1, kAdagrad = 2, kFtrl = 3 };

struct OptParams {
  float lr;
  float beta1, beta2, eps;
  float wd;
  float momentum, dampening;
  int nesterov;
  int adamw;
  float bc1, bc2;      // multipliers applied to m and v (bias correction), host-computed
  float l1, l2, fbeta; // FTRL
  int ftrl_mode;       // 0 canonical, 1 reference
  int skip_zero;       // FTRL: skip the update when the first grad element of the key is 0 (reference)
  float gscale;        // host gradient multiplier
  const float* gscale_ptr;  // optional device multiplier (global-norm clip factor)
};

template <int KIND>
__device__ __forceinline__ void opt_apply(float& w, float g, float& s0, float& s1, const OptParams& p) {
  if constexpr (KIND == kSGD) {
    if (p.wd != 0.f) g += p.wd * w;
    if (p.momentum != 0.f) {
      s0 = p.momentum * s0 + (1.f - p.dampening) * g;
      g = p.nesterov ? g + p.momentum * s0 : s0;
    }
    w -= p.lr * g;
  } else if constexpr (KIND == kAdam) {
    if (p.wd != 0.f && !p.adamw) g += p.wd * w;
    s0 = p.beta1 * s0 + (1.f - p.beta1) * g;
    s1 = p.beta2 * s1 + (1.f - p.beta2) * g * g;
    const float mh = s0 * p.bc1;
    const float vh = s1 * p.bc2;
    float upd = mh / (sqrtf(vh) + p.eps);
    if (p.wd != 0.f && p.adamw) upd += p.wd * w;
    w -= p.lr * upd;
  } else if constexpr (KIND == kAdagrad) {
    if (p.wd != 0.f) g += p.wd * w;
    s0 += g * g;
    w -= p.lr * g / (sqrtf(s0) + p.eps);
  } else {  // FTRL; s0 = z, s1 = n ; lr = alpha
    const float z = s0, n = s1;
    if (p.ftrl_mode == 1) {
      // reference: w from (z, n_old), then sigma = sqrt(n+g^2) - sqrt(n/alpha), z += g - sigma*w
      float wn;
      if (fabsf(z) <= p.l1) wn = 0.f;
      else {
        const float sgn = z >= 0.f ? 1.f : -1.f;
        wn = -(z - sgn * p.l1) / ((p.l2 + (p.fbeta + sqrtf(n))) / p.lr);
      }
      const float sigma = sqrtf(n + g * g) - sqrtf(n / p.lr);
      s0 = z + (g - sigma * wn);
      s1 = n + g * g;
      w = wn;
    } else {
      const float nn = n + g * g;
      const float sigma = (sqrtf(nn) - sqrtf(n)) / p.lr;
      const float zn = z + g - sigma * w;
      s0 = zn;
      s1 = nn;
      if (fabsf(zn) <= p.l1) w = 0.f;
      else {
        const float sgn = zn >= 0.f ? 1.f : -1.f;
        w = -(zn - sgn * p.l1) / ((p.fbeta + sqrtf(nn)) / p.lr + p.l2);
      }
    }
  }
}

template <int KIND> struct NState { static constexpr int v = (KIND == kAdam || KIND == kFtrl) ? 2 : ((KIND == kSGD) ? 1 : 1); };

// OUT: 0 = no copy-out, 1 = bf16 copy-out, 2 = fp32 copy-out.
template <int KIND, typename G, int OUT, bool VEC>
__global__ __launch_bounds__(256) void fused_opt_kernel(float* __restrict__ w, float* __restrict__ st0,
                                                         float* __restrict__ st1, const G* __restrict__ g,
                                                         void* __restrict__ wout, int64_t n, OptParams p) {
  float scale = p.gscale;
  if (p.gscale_ptr) scale *= *p.gscale_ptr;
  const bool use_st0 = st0 != nullptr;
  const bool use_st1 = st1 != nullptr;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  if constexpr (VEC) {
    const int64_t nv = n / 8;
    for (int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; v < nv; v += stride) {
      const int64_t i = v * 8;
      float wr[8], gr[8], a[8], b[8];
      load8(w, i, wr);
      load8(g, i, gr);
      if (use_st0) load8(st0, i, a); else {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = 0.f;
      }
      if (use_st1) load8(st1, i, b); else {
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) opt_apply<KIND>(wr[j], gr[j] * scale, a[j], b[j], p);
      store8(w, i, wr);
      if (use_st0) store8(st0, i, a);
      if (use_st1) store8(st1, i, b);
      if constexpr (OUT == 1) store8(static_cast<uint16_t*>(wout), i, wr);
      if constexpr (OUT == 2) store8(static_cast<float*>(wout), i, wr);
    }
    // tail (n % 8) handled by block 0
    if (blockIdx.x == 0) {
      for (int64_t i = nv * 8 + threadIdx.x; i < n; i += blockDim.x) {
        float wr = w[i], a = use_st0 ? st0[i] : 0.f, b = use_st1 ? st1[i] : 0.f;
        opt_apply<KIND>(wr, Elem<G>::load(g, i) * scale, a, b, p);
        w[i] = wr;
        if (use_st0) st0[i] = a;
        if (use_st1) st1[i] = b;
        if constexpr (OUT == 1) static_cast<uint16_t*>(wout)[i] = f32_to_bf16(wr);
        if constexpr (OUT == 2) static_cast<float*>(wout)[i] = wr;
      }
    }
  } else {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
      float wr = w[i], a = use_st0 ? st0[i] : 0.f, b = use_st1 ? st1[i] : 0.f;
      opt_apply<KIND>(wr, Elem<G>::load(g, i) * scale, a, b, p);
      w[i] = wr;
      if (use_st0) st0[i] = a;
      if (use_st1) st1[i] = b;
      if constexpr (OUT == 1) static_cast<uint16_t*>(wout)[i] = f32_to_bf16(wr);
      if constexpr (OUT == 2) static_cast<float*>(wout)[i] = wr;
    }
  }
}

template <int KIND, typename G, int OUT>
static void dispatch_vec(const FusedOptArgs& a, const OptParams& p, hipStream_t s) {
  const bool aligned = ((reinterpret_cast<uintptr_t>(a.w) | reinterpret_cast<uintptr_t>(a.st0) |
                         reinterpret_cast<uintptr_t>(a.st1) | reinterpret_cast<uintptr_t>(a.g) |
                         reinterpret_cast<uintptr_t>(a.wout)) & 15) == 0 &&
                       (sizeof(G) == 4 || (reinterpret_cast<uintptr_t>(a.g) & 15) == 0);
  const int block = 256;
  if (aligned) {
    const int grid = opt_grid((a.n + 7) / 8, block);
    hipLaunchKernelGGL((fused_opt_kernel<KIND, G, OUT, true>), dim3(grid), dim3(block), 0, s, a.w, a.st0, a.st1,
                       static_cast<const G*>(a.g), a.wout, a.n, p);
  } else {
    const int grid = opt_grid(a.n, block);
    hipLaunchKernelGGL((fused_opt_kernel<KIND, G, OUT, false>), dim3(grid), dim3(block), 0, s, a.w, a.st0, a.st1,
                       static_cast<const G*>(a.g), a.wout, a.n, p);
  }
}

template <int KIND, typename G>
static void dispatch_out(const FusedOptArgs& a, const OptParams& p, hipStream_t s) {
  if (a.wout == nullptr) dispatch_vec<KIND, G, 0>(a, p, s);
  else if (a.wout_bf16) dispatch_vec<KIND, G, 1>(a, p, s);
  else dispatch_vec<KIND, G, 2>(a, p, s);
}

template <int KIND>
static void dispatch_grad(const FusedOptArgs& a, const OptParams& p, hipStream_t s) {
  if (a.g_bf16) dispatch_out<KIND, uint16_t>(a, p, s);
  else dispatch_out<KIND, float>(a, p, s);
}

static OptParams opt_params(const FusedOptArgs& a) {
  OptParams p;
  p.lr = a.lr; p.beta1 = a.beta1; p.beta2 = a.beta2; p.eps = a.eps; p.wd = a.wd;
  p.momentum = a.momentum; p.dampening = a.dampening; p.nesterov = a.nesterov; p.adamw = a.adamw;
  p.bc1 = a.bc1; p.bc2 = a.bc2; p.l1 = a.l1; p.l2 = a.l2; p.fbeta = a.fbeta; p.ftrl_mode = a.ftrl_mode;
  p.skip_zero = 0; p.gscale = a.gscale; p.gscale_ptr = a.gscale_ptr;
  return p;
}

void launch_fused_opt(const FusedOptArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  const OptParams p = opt_params(a);
  switch (a.kind) {
    case kSGD: dispatch_grad<kSGD>(a, p, s); break;
    case kAdam: dispatch_grad<kAdam>(a, p, s); break;
    case kAdagrad: dispatch_grad<kAdagrad>(a, p, s); break;
    case kFtrl: dispatch_grad<kFtrl>(a, p, s); break;
    default: break;
  }
}

// ---------------------------------------------------------------------------------------
// Owner-side "reduce + serve" of the xGMI parameter-server plane (ps_amd/parallel/plane.py,
// csrc/plane.cpp): the gradient of every element is the sum, in fixed rank order, of the W
// workers' pushed values read straight out of their IPC-mapped gradient buckets (or decoded
// from their 1-bit packed pushes), accumulated in fp32 and fed to the fused optimizer in the
// same pass.  One kernel replaces reduce-scatter + owner optimizer: the reduced gradient never
// round-trips through HBM, and each lane keeps W 16-B loads in flight -- one per peer -- so all
// of a GPU's xGMI links stream concurrently.
//
// Segments start at an arbitrary chunk element ``off`` (key boundaries inside a bucket): block
// 0 handles the unaligned head and the tail element by element, everything else moves 8
// elements (16 B of bf16) per lane per source.
//
// Coherence: the producers' data is published by a HIP event (system-scope release) that the
// host observed before launching this kernel; the system-scope acquire at entry makes sure no
// stale line of a peer's buffer is served from this GPU's caches.
// ---------------------------------------------------------------------------------------
template <int ONEBIT, typename G>
__device__ __forceinline__ float multi_load1(const MultiGrad& m, int64_t q) {
  float acc = 0.f;
  for (int s = 0; s < m.nsrc; ++s) {
    if constexpr (ONEBIT) {
      const uint64_t wd = m.words[s][q >> 6];
      const float sc = m.scales[s][q / kOnebitChunk];
      acc += ((wd >> (q & 63)) & 1ull) ? sc : -sc;
    } else {
      acc += Elem<G>::load(static_cast<const G*>(m.g[s]), q);
    }
  }
  return acc;
}

template <int ONEBIT, typename G>
__device__ __forceinline__ void multi_load8(const MultiGrad& m, int64_t q0, float (&acc)[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  if constexpr (ONEBIT) {
    const int sh = static_cast<int>(q0 & 63);
    for (int s = 0; s < m.nsrc; ++s) {
      const uint32_t byte = static_cast<uint32_t>(m.words[s][q0 >> 6] >> sh) & 0xFFu;
      const float sc = m.scales[s][q0 / kOnebitChunk];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += ((byte >> k) & 1u) ? sc : -sc;
    }
  } else {
    // issue every source's 16-B load before the first add: W loads in flight per lane
    float v[kPlaneMaxSrc][8];
#pragma unroll
    for (int s = 0; s < kPlaneMaxSrc; ++s)
      if (s < m.nsrc) load8(static_cast<const G*>(m.g[s]), q0, v[s]);
#pragma unroll
    for (int s = 0; s < kPlaneMaxSrc; ++s)
      if (s < m.nsrc) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += v[s][k];
      }
  }
}

template <int KIND, int ONEBIT, typename G, int OUT>
__global__ __launch_bounds__(256) void fused_opt_multi_kernel(float* __restrict__ w, float* __restrict__ st0,
                                                               float* __restrict__ st1, const MultiGrad m,
                                                               void* __restrict__ wout, int64_t n, int64_t head,
                                                               OptParams p) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  float scale = p.gscale;
  if (p.gscale_ptr) scale *= *p.gscale_ptr;
  const bool use_st0 = st0 != nullptr;
  const bool use_st1 = st1 != nullptr;
  const int64_t nv = (n - head) / 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const int64_t i = head + v * 8;
    float wr[8], gr[8], a[8], b[8];
    multi_load8<ONEBIT, G>(m, m.off + i, gr);
    load8(w, i, wr);
    if (use_st0) load8(st0, i, a);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = 0.f;
    }
    if (use_st1) load8(st1, i, b);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) opt_apply<KIND>(wr[j], gr[j] * scale, a[j], b[j], p);
    store8(w, i, wr);
    if (use_st0) store8(st0, i, a);
    if (use_st1) store8(st1, i, b);
    if constexpr (OUT == 1) store8(static_cast<uint16_t*>(wout), i, wr);
    if constexpr (OUT == 2) store8(static_cast<float*>(wout), i, wr);
  }
  if (blockIdx.x == 0) {  // unaligned head [0, head) and tail [head + 8 nv, n)
    const int64_t tail0 = head + nv * 8;
    const int64_t ntail = n - tail0;
    for (int64_t t = threadIdx.x; t < head + ntail; t += blockDim.x) {
      const int64_t i = t < head ? t : tail0 + (t - head);
      float wr = w[i], a = use_st0 ? st0[i] : 0.f, b = use_st1 ? st1[i] : 0.f;
      opt_apply<KIND>(wr, multi_load1<ONEBIT, G>(m, m.off + i) * scale, a, b, p);
      w[i] = wr;
      if (use_st0) st0[i] = a;
      if (use_st1) st1[i] = b;
      if constexpr (OUT == 1) static_cast<uint16_t*>(wout)[i] = f32_to_bf16(wr);
      if constexpr (OUT == 2) static_cast<float*>(wout)[i] = wr;
    }
  }
}

template <int KIND, int ONEBIT, typename G>
static void launch_multi_out(const FusedOptArgs& a, const MultiGrad& m, const OptParams& p, int64_t head,
                             hipStream_t s) {
  const int grid = opt_grid((a.n - head + 7) / 8, 256);
  if (a.wout == nullptr)
    hipLaunchKernelGGL((fused_opt_multi_kernel<KIND, ONEBIT, G, 0>), dim3(grid), dim3(256), 0, s, a.w, a.st0, a.st1,
                       m, a.wout, a.n, head, p);
  else if (a.wout_bf16)
    hipLaunchKernelGGL((fused_opt_multi_kernel<KIND, ONEBIT, G, 1>), dim3(grid), dim3(256), 0, s, a.w, a.st0, a.st1,
                       m, a.wout, a.n, head, p);
  else
    hipLaunchKernelGGL((fused_opt_multi_kernel<KIND, ONEBIT, G, 2>), dim3(grid), dim3(256), 0, s, a.w, a.st0, a.st1,
                       m, a.wout, a.n, head, p);
}

template <int KIND>
static void launch_multi_kind(const FusedOptArgs& a, const MultiGrad& m, const OptParams& p, int64_t head,
                              hipStream_t s) {
  if (m.onebit) launch_multi_out<KIND, 1, float>(a, m, p, head, s);
  else if (a.g_bf16) launch_multi_out<KIND, 0, uint16_t>(a, m, p, head, s);
  else launch_multi_out<KIND, 0, float>(a, m, p, head, s);
}

void launch_fused_opt_multi(const FusedOptArgs& a, const MultiGrad& m, hipStream_t s) {
  if (a.n <= 0) return;
  const OptParams p = opt_params(a);
  // elements before the first 8-aligned chunk index are done element-wise (every array of the
  // segment shares the phase of m.off: masters / states / wout start at the segment too)
  int64_t head = (8 - (m.off & 7)) & 7;
  if (head > a.n) head = a.n;
  switch (a.kind) {
    case kSGD: launch_multi_kind<kSGD>(a, m, p, head, s); break;
    case kAdam: launch_multi_kind<kAdam>(a, m, p, head, s); break;
    case kAdagrad: launch_multi_kind<kAdagrad>(a, m, p, head, s); break;
    case kFtrl: launch_multi_kind<kFtrl>(a, m, p, head, s); break;
    default: break;
  }
}

// Reduce-only form (global-norm clipping needs the whole reduced gradient before any update):
// out[i] = sum over sources, fp32, in rank order.
template <int ONEBIT, typename G>
__global__ __launch_bounds__(256) void reduce_multi_kernel(const MultiGrad m, int64_t n, int64_t head,
                                                            float* __restrict__ out) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const int64_t nv = (n - head) / 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const int64_t i = head + v * 8;
    float gr[8];
    multi_load8<ONEBIT, G>(m, m.off + i, gr);
    store8(out, i, gr);
  }
  if (blockIdx.x == 0) {
    const int64_t tail0 = head + nv * 8;
    const int64_t ntail = n - tail0;
    for (int64_t t = threadIdx.x; t < head + ntail; t += blockDim.x) {
      const int64_t i = t < head ? t : tail0 + (t - head);
      out[i] = multi_load1<ONEBIT, G>(m, m.off + i);
    }
  }
}

void launch_reduce_multi(const MultiGrad& m, int g_bf16, int64_t n, float* out, hipStream_t s) {
  if (n <= 0) return;
  int64_t head = (8 - (m.off & 7)) & 7;
  if (head > n) head = n;
  const int grid = opt_grid((n - head + 7) / 8, 256);
  if (m.onebit)
    hipLaunchKernelGGL((reduce_multi_kernel<1, float>), dim3(grid), dim3(256), 0, s, m, n, head, out);
  else if (g_bf16)
    hipLaunchKernelGGL((reduce_multi_kernel<0, uint16_t>), dim3(grid), dim3(256), 0, s, m, n, head, out);
  else
    hipLaunchKernelGGL((reduce_multi_kernel<0, float>), dim3(grid), dim3(256), 0, s, m, n, head, out);
}

// ---------------------------------------------------------------------------------------
// Row-sparse variants (sparse embedding tables, K24): apply the optimizer only to the rows
// named in `rows` (owner-local row indices), with `grad` laid out [n, dim].  One wave per row
// entry.  Row-wise Adagrad keeps ONE accumulator per row (mean of g^2 over the row), the DLRM
// convention.
//
// Two input forms:
//  * perm == nullptr: `rows` are unique, grad row r belongs to rows[r].
//  * perm != nullptr: `rows` is SORTED and may repeat (several workers pushed the same row,
//    or several micro-batches of one round); grad row perm[j] belongs to rows[j].  The wave
//    at the head of each run sums the run's gradient rows in order (deterministic, no atomics)
//    and applies ONE update -- the owner-side "sum the W pushes, then step" of a BSP round
//    without a host-side unique (which would need a device->host sync for its size).
// Negative rows (unresolved keys) are skipped.
// ---------------------------------------------------------------------------------------
template <typename G>
__device__ __forceinline__ float run_grad(const G* __restrict__ grad, const int64_t* __restrict__ perm, int64_t r,
                                          int64_t e, int dim, int c) {
  if (perm == nullptr) return Elem<G>::load(grad + r * dim, c);
  float acc = 0.f;
  for (int64_t j = r; j < e; ++j) acc += Elem<G>::load(grad + perm[j] * dim, c);
  return acc;
}

template <int KIND, typename G>
__global__ __launch_bounds__(256) void sparse_opt_kernel(float* __restrict__ table, float* __restrict__ st0,
                                                          float* __restrict__ st1, const int64_t* __restrict__ rows,
                                                          const int64_t* __restrict__ perm,
                                                          const G* __restrict__ grad, int64_t nrows, int dim,
                                                          OptParams p, int rowwise, const int32_t* __restrict__ ncount) {
  if (ncount) nrows = min(nrows, static_cast<int64_t>(*ncount));
  float scale = p.gscale;
  if (p.gscale_ptr) scale *= *p.gscale_ptr;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * blockDim.x / 64;
  for (int64_t r = wave; r < nrows; r += nwaves) {
    const int64_t row = rows[r];
    if (row < 0) continue;
    int64_t e = r + 1;
    if (perm != nullptr) {
      if (r > 0 && rows[r - 1] == row) continue;  // not the head of its run
      while (e < nrows && rows[e] == row) ++e;
    }
    float* wrow = table + row * dim;
    if (KIND == kAdagrad && rowwise) {
      float ss = 0.f;
      for (int c = lane; c < dim; c += 64) {
        const float gv = run_grad(grad, perm, r, e, dim, c) * scale;
        ss += gv * gv;
      }
      ss = wave_sum(ss) / static_cast<float>(dim);
      const float h = st0[row] + ss;
      if (lane == 0) st0[row] = h;
      const float denom = sqrtf(h) + p.eps;
      for (int c = lane; c < dim; c += 64) {
        const float gv = run_grad(grad, perm, r, e, dim, c) * scale;
        wrow[c] -= p.lr * gv / denom;
      }
    } else {
      // skip_zero reproduces FtrlUpdater.java:52-54 (per key == per row).
      if (p.skip_zero && run_grad(grad, perm, r, e, dim, 0) == 0.f) continue;
      for (int c = lane; c < dim; c += 64) {
        float wr = wrow[c];
        float a = st0 ? st0[row * dim + c] : 0.f;
        float b = st1 ? st1[row * dim + c] : 0.f;
        opt_apply<KIND>(wr, run_grad(grad, perm, r, e, dim, c) * scale, a, b, p);
        wrow[c] = wr;
        if (st0) st0[row * dim + c] = a;
        if (st1) st1[row * dim + c] = b;
      }
    }
  }
}

// Vectorised form for dim = 4 * 2^k <= 256: 2^lg lanes share a row, each lane owns 4 adjacent
// elements (16-B loads / stores), a wave updates 64 >> lg rows at once and a run's summed
// gradient stays in registers (one pass over the pushed rows, none re-read).
template <int KIND, typename G>
__global__ __launch_bounds__(256) void sparse_opt_vec_kernel(float* __restrict__ table, float* __restrict__ st0,
                                                              float* __restrict__ st1, const int64_t* __restrict__ rows,
                                                              const int64_t* __restrict__ perm,
                                                              const G* __restrict__ grad, int64_t nrows, int dim,
                                                              int lg, OptParams p, int rowwise,
                                                              const int32_t* __restrict__ ncount) {
  if (ncount) nrows = min(nrows, static_cast<int64_t>(*ncount));
  float scale = p.gscale;
  if (p.gscale_ptr) scale *= *p.gscale_ptr;
  const int lane = threadIdx.x & 63;
  const int sub = lane >> lg;                  // row slot within the wave
  const int c = (lane & ((1 << lg) - 1)) * 4;  // first element of this lane
  const int per_wave = 64 >> lg;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * blockDim.x / 64;
  for (int64_t rb = wave * per_wave; rb < nrows; rb += nwaves * per_wave) {  // wave-uniform loop
    const int64_t r = rb + sub;
    int64_t row = r < nrows ? rows[r] : -1;
    if (row >= 0 && perm != nullptr && r > 0 && rows[r - 1] == row) row = -1;  // not a run head
    f32x4 g = {0.f, 0.f, 0.f, 0.f};
    if (row >= 0) {
      if (perm == nullptr) {
        g = load4(grad, r * dim + c);
      } else {
        // the run's next row id and this entry's perm are independent loads: issue both, then
        // the gradient row; runs are short (one entry per pushing worker / micro-batch)
        int64_t j = r;
        int64_t pj = perm[j];
        int64_t nx = j + 1 < nrows ? rows[j + 1] : -1;
        g = load4(grad, pj * dim + c);
        while (nx == row) {
          ++j;
          pj = perm[j];
          nx = j + 1 < nrows ? rows[j + 1] : -1;
          g += load4(grad, pj * dim + c);
        }
      }
      g *= scale;
    }
    if (KIND == kAdagrad && rowwise) {
      const float ss = group_sum(g.x * g.x + g.y * g.y + g.z * g.z + g.w * g.w, lg) / static_cast<float>(dim);
      if (row < 0) continue;
      const float h = st0[row] + ss;
      if (c == 0) st0[row] = h;
      const float k = p.lr / (sqrtf(h) + p.eps);
      f32x4 w = load4(table, row * dim + c);
      w -= k * g;
      store4(table, row * dim + c, w);
    } else {
      // skip_zero (FtrlUpdater.java:52-54): the row's first gradient element, from its lane 0
      const float g0 = __shfl(g.x, lane & ~((1 << lg) - 1), kWave);
      if (row < 0 || (p.skip_zero && g0 == 0.f)) continue;
      const int64_t o = row * dim + c;
      f32x4 w = load4(table, o);
      f32x4 a = st0 ? load4(st0, o) : f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 b = st1 ? load4(st1, o) : f32x4{0.f, 0.f, 0.f, 0.f};
      float wv[4] = {w.x, w.y, w.z, w.w}, av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
      const float gv[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) opt_apply<KIND>(wv[k], gv[k], av[k], bv[k], p);
      store4(table, o, f32x4{wv[0], wv[1], wv[2], wv[3]});
      if (st0) store4(st0, o, f32x4{av[0], av[1], av[2], av[3]});
      if (st1) store4(st1, o, f32x4{bv[0], bv[1], bv[2], bv[3]});
    }
  }
}

static int vec_lanes_log2(int dim) {  // lanes per row for the vectorised kernels, -1 = scalar path
  if (dim % 4 != 0 || dim > 256) return -1;
  const int l = dim / 4;
  if ((l & (l - 1)) != 0) return -1;
  int lg = 0;
  while ((1 << lg) < l) ++lg;
  return lg;
}

void launch_sparse_opt(const SparseOptArgs& a, hipStream_t s) {
  if (a.nrows <= 0) return;
  OptParams p;
  p.lr = a.lr; p.beta1 = a.beta1; p.beta2 = a.beta2; p.eps = a.eps; p.wd = a.wd;
  p.momentum = a.momentum; p.dampening = a.dampening; p.nesterov = a.nesterov; p.adamw = a.adamw;
  p.bc1 = a.bc1; p.bc2 = a.bc2; p.l1 = a.l1; p.l2 = a.l2; p.fbeta = a.fbeta; p.ftrl_mode = a.ftrl_mode;
  p.skip_zero = a.skip_zero; p.gscale = a.gscale; p.gscale_ptr = nullptr;
  const int block = 256;
  const int lg = vec_lanes_log2(a.dim);
  const bool aligned = ((reinterpret_cast<uintptr_t>(a.table) | reinterpret_cast<uintptr_t>(a.st0) |
                         reinterpret_cast<uintptr_t>(a.st1) | reinterpret_cast<uintptr_t>(a.grad)) & 15) == 0;
  if (lg >= 0 && aligned) {
    const int grid = stream_grid(((a.nrows << lg) + 63) / 64 * 64, block);
#define PSAMD_SPARSE_VEC(K)                                                                                      \
  if (a.g_bf16)                                                                                                  \
    hipLaunchKernelGGL((sparse_opt_vec_kernel<K, uint16_t>), dim3(grid), dim3(block), 0, s, a.table, a.st0,      \
                       a.st1, a.rows, a.perm, static_cast<const uint16_t*>(a.grad), a.nrows, a.dim, lg, p,     \
                       a.rowwise, a.ncount);                                                                     \
  else                                                                                                           \
    hipLaunchKernelGGL((sparse_opt_vec_kernel<K, float>), dim3(grid), dim3(block), 0, s, a.table, a.st0, a.st1, \
                       a.rows, a.perm, static_cast<const float*>(a.grad), a.nrows, a.dim, lg, p, a.rowwise,    \
                       a.ncount);
    switch (a.kind) {
      case kSGD: PSAMD_SPARSE_VEC(kSGD); break;
      case kAdam: PSAMD_SPARSE_VEC(kAdam); break;
      case kAdagrad: PSAMD_SPARSE_VEC(kAdagrad); break;
      case kFtrl: PSAMD_SPARSE_VEC(kFtrl); break;
      default: break;
    }
#undef PSAMD_SPARSE_VEC
    return;
  }
  const int grid = stream_grid(a.nrows * 64, block);
#define PSAMD_SPARSE_LAUNCH(K)                                                                                  \
  if (a.g_bf16)                                                                                                 \
    hipLaunchKernelGGL((sparse_opt_kernel<K, uint16_t>), dim3(grid), dim3(block), 0, s, a.table, a.st0, a.st1,  \
                       a.rows, a.perm, static_cast<const uint16_t*>(a.grad), a.nrows, a.dim, p, a.rowwise,      \
                       a.ncount);                                                                               \
  else                                                                                                          \
    hipLaunchKernelGGL((sparse_opt_kernel<K, float>), dim3(grid), dim3(block), 0, s, a.table, a.st0, a.st1,     \
                       a.rows, a.perm, static_cast<const float*>(a.grad), a.nrows, a.dim, p, a.rowwise, a.ncount);
  switch (a.kind) {
    case kSGD: PSAMD_SPARSE_LAUNCH(kSGD); break;
    case kAdam: PSAMD_SPARSE_LAUNCH(kAdam); break;
    case kAdagrad: PSAMD_SPARSE_LAUNCH(kAdagrad); break;
    case kFtrl: PSAMD_SPARSE_LAUNCH(kFtrl); break;
    default: break;
  }
#undef PSAMD_SPARSE_LAUNCH
}

}  // namespace psamd
