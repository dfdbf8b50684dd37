// Data-movement kernels of the xGMI parameter-server plane (ps_amd/parallel/plane.py,
// csrc/plane.cpp).
//
// Reference: a worker pulls every dense key from the server that owns it after the barrier
// (store/KVStore.java:136-159 get -> net/PSRouterClient.java:55-58 -> net/PServer.java:78-99),
// one RPC per key and server.  Here the pull of a bucket is ONE kernel on the reading GPU that
// copies every other owner's freshly updated chunk out of that owner's IPC-mapped weight
// buffer into the local replica.  Blocks are dealt round-robin over the owners (block k reads
// owner k mod nseg), so the W-1 source GPUs -- W-1 different xGMI links -- stream at once;
// within an owner each lane moves 16 B per access.
//
// The owner wrote its chunk in an earlier kernel whose completion event (system-scope release)
// the host observed before launching this one; the system-scope acquire at entry keeps this
// GPU's caches from serving a stale line of the peer buffer.
#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

__global__ __launch_bounds__(256) void plane_gather_kernel(const PlaneCopies c, int blocks_per_seg) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const int seg = blockIdx.x % c.nseg;
  const int lb = blockIdx.x / c.nseg;
  const int64_t nbytes = c.nbytes[seg];
  const f32x4* __restrict__ src = static_cast<const f32x4*>(c.src[seg]);
  f32x4* __restrict__ dst = static_cast<f32x4*>(c.dst[seg]);
  const int64_t n16 = nbytes / 16;
  const int64_t stride = static_cast<int64_t>(blocks_per_seg) * blockDim.x;
  int64_t i = static_cast<int64_t>(lb) * blockDim.x + threadIdx.x;
  // 4 independent 16-B loads in flight per lane before the first store
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const f32x4 a = src[i], b = src[i + stride], d = src[i + 2 * stride], e = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = d;
    dst[i + 3 * stride] = e;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
  if (lb == 0) {  // byte tail (chunks are multiples of 128 B in practice)
    const uint8_t* s8 = static_cast<const uint8_t*>(c.src[seg]);
    uint8_t* d8 = static_cast<uint8_t*>(c.dst[seg]);
    for (int64_t t = n16 * 16 + threadIdx.x; t < nbytes; t += blockDim.x) d8[t] = s8[t];
  }
}

void launch_plane_copy(const PlaneCopies& c, hipStream_t s) {
  if (c.nseg <= 0) return;
  int64_t mx = 0;
  for (int k = 0; k < c.nseg; ++k) mx = c.nbytes[k] > mx ? c.nbytes[k] : mx;
  if (mx <= 0) return;
  // ~8 blocks per CU over the whole launch; at least one block per segment
  int64_t per = (mx / 16 + 255) / 256;
  int64_t cap = (2048 + c.nseg - 1) / c.nseg;
  if (per > cap) per = cap;
  if (per < 1) per = 1;
  hipLaunchKernelGGL(plane_gather_kernel, dim3(static_cast<unsigned>(per * c.nseg)), dim3(256), 0, s, c,
                     static_cast<int>(per));
}

void launch_plane_gather(const PlaneCopies& c, int64_t nbytes, hipStream_t s) {
  PlaneCopies e = c;
  for (int k = 0; k < e.nseg; ++k) e.nbytes[k] = nbytes;
  launch_plane_copy(e, s);
}

// Global-norm clip factor from every rank's partial sum of squares (read from the peers'
// IPC-mapped slots, summed in rank order so every rank computes the identical factor).
__global__ void plane_clip_factor_kernel(const PlaneCopies c, float max_norm, float* __restrict__ total,
                                         float* __restrict__ factor) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  if (threadIdx.x == 0) {
    float acc = 0.f;
    for (int r = 0; r < c.nseg; ++r) acc += *static_cast<const float*>(c.src[r]);
    *total = acc;
    const float f = max_norm / (sqrtf(acc) + 1e-6f);
    *factor = f < 1.f ? f : 1.f;
  }
}

void launch_plane_clip_factor(const PlaneCopies& c, float max_norm, float* total, float* factor, hipStream_t s) {
  hipLaunchKernelGGL(plane_clip_factor_kernel, dim3(1), dim3(64), 0, s, c, max_norm, total, factor);
}

// Fill n floats (small plane scratch: the self-test probe, zeroed norm slots).
__global__ void plane_fill_kernel(float* __restrict__ p, int64_t n, float v) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    p[i] = v;
}

void launch_plane_fill(float* p, int64_t n, float v, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(plane_fill_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, s, p, n, v);
}

}  // namespace psamd
