// 1-bit gradient compression with error feedback (K26 in SURVEY §2.5).
//
// The reference gzips every float payload on the wire (net/PSClient.java:37,
// visual/UiClient.java:31) and lists quantized transfer as TODO (README.md:233).  Here the
// push is compressed on device before it is sent:
//
//   c      = g + e                       (error feedback)
//   scale  = mean(|c|) over a 1024-element chunk
//   bit    = c >= 0                      packed 64 per word with a wave64 __ballot
//   e      = c - (bit ? scale : -scale)
//
// Layout: element i lives in word i/64, bit i%64; the chunk scale for element i is
// scales[i/1024].  A 256-thread block owns one chunk: thread t handles elements
// t, t+256, t+512, t+768, so each wave's ballot produces one contiguous 64-element word.
// unpack_reduce sums W workers' packed pushes in a fixed worker order (deterministic) and
// optionally accumulates into the destination.
#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

template <typename G>
__global__ __launch_bounds__(256) void onebit_pack_kernel(const G* __restrict__ g, float* __restrict__ err, int64_t n,
                                                          uint64_t* __restrict__ words, float* __restrict__ scales) {
  __shared__ float scratch[4];
  const int64_t chunk = blockIdx.x;
  const int64_t base = chunk * kOnebitChunk;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  float c[4];
  float asum = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t i = base + j * 256 + threadIdx.x;
    float v = 0.f;
    if (i < n) v = Elem<G>::load(g, i) + err[i];
    c[j] = v;
    asum += fabsf(v);
  }
  const int64_t valid = (n - base) < kOnebitChunk ? (n - base) : kOnebitChunk;
  asum = block_sum(asum, scratch);
  const float scale = asum / static_cast<float>(valid);
  if (threadIdx.x == 0) scales[chunk] = scale;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t i = base + j * 256 + threadIdx.x;
    const bool pos = (i < n) && c[j] >= 0.f;  // padded lanes contribute 0 bits
    const uint64_t m = __ballot(pos);
    if (i < n) err[i] = c[j] - (pos ? scale : -scale);
    const int64_t wbase = base + j * 256 + wid * 64;
    if (lane == 0 && wbase < n) words[wbase / 64] = m;
  }
}

// 8 consecutive elements per thread (one byte of a packed word, one 16-B / 32-B output store):
// a wave covers 512 elements = 8 words inside one 1024-element scale chunk, so per worker it
// issues one 64-B coalesced word load and one broadcast scale load for 512 outputs.
template <typename O>
__global__ __launch_bounds__(256) void onebit_unpack_reduce_kernel(const uint64_t* __restrict__ words,
                                                                   const float* __restrict__ scales, int nworkers,
                                                                   int64_t n, int64_t wstride, int64_t sstride,
                                                                   O* __restrict__ out, float mult, int accumulate,
                                                                   int vec) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t n8 = (n + 7) / 8;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < n8; t += stride) {
    const int64_t i0 = t * 8;
    const int64_t wi = i0 >> 6;
    const int sh = static_cast<int>(i0 & 63);
    const int64_t si = i0 / kOnebitChunk;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < nworkers; ++w) {
      const uint32_t byte = static_cast<uint32_t>(words[w * wstride + wi] >> sh) & 0xFFu;
      const float sc = scales[w * sstride + si];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += ((byte >> k) & 1u) ? sc : -sc;
    }
    if (vec && i0 + 8 <= n) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] *= mult;
      if (accumulate) {
        float o[8];
        load8(out, i0, o);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += o[k];
      }
      store8(out, i0, acc);
    } else {
      for (int k = 0; k < 8 && i0 + k < n; ++k) {
        float v = acc[k] * mult;
        if (accumulate) v += Elem<O>::load(out, i0 + k);
        Elem<O>::store(out, i0 + k, v);
      }
    }
  }
}

void launch_onebit_pack(const void* g, int gdtype, float* err, int64_t n, uint64_t* words, float* scales,
                        hipStream_t s) {
  if (n <= 0) return;
  const int64_t nchunks = (n + kOnebitChunk - 1) / kOnebitChunk;
  if (gdtype == 1)
    hipLaunchKernelGGL(onebit_pack_kernel<uint16_t>, dim3(nchunks), dim3(256), 0, s, static_cast<const uint16_t*>(g),
                       err, n, words, scales);
  else
    hipLaunchKernelGGL(onebit_pack_kernel<float>, dim3(nchunks), dim3(256), 0, s, static_cast<const float*>(g), err,
                       n, words, scales);
}

void launch_onebit_unpack_reduce(const uint64_t* words, const float* scales, int nworkers, int64_t n,
                                 int64_t words_stride, int64_t scales_stride, void* out, int odtype, float mult,
                                 int accumulate, hipStream_t s) {
  if (n <= 0) return;
  // 8-element vector stores need a 16-B aligned destination (else element stores)
  const int vec = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  const int grid = stream_grid((n + 7) / 8, 256);
  if (odtype == 1)
    hipLaunchKernelGGL(onebit_unpack_reduce_kernel<uint16_t>, dim3(grid), dim3(256), 0, s, words, scales, nworkers, n,
                       words_stride, scales_stride, static_cast<uint16_t*>(out), mult, accumulate, vec);
  else
    hipLaunchKernelGGL(onebit_unpack_reduce_kernel<float>, dim3(grid), dim3(256), 0, s, words, scales, nworkers, n,
                       words_stride, scales_stride, static_cast<float*>(out), mult, accumulate, vec);
}

}  // namespace psamd
