// 1-bit gradient compression with error feedback (K26 in SURVEY §2.5).
//
// The reference gzips every float payload on the wire (net/PSClient.java:37,
// visual/UiClient.java:31) and lists quantized transfer as TODO (README.md:233).  Here the
// push is compressed on device before it is sent:
//
//   c      = g + e                       (error feedback)
//   scale  = mean(|c|) over a 1024-element chunk
//   bit    = c >= 0                      packed 64 per word
//   e      = c - (bit ? scale : -scale)
//
// Layout: element i lives in word i/64, bit i%64 (= byte i/8, bit i%8); the chunk scale for
// element i is scales[i/1024].
// unpack_reduce sums W workers' packed pushes in a fixed worker order (deterministic) and
// optionally accumulates into the destination.
#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

// E: the error-feedback buffer's element type -- fp32, or bf16 (uint16_t) to halve its footprint
// on large models (Llama-3-8B: 16 GB instead of 32 GB per rank); c is formed in fp32 either way.
// Vector layout: thread t of a 256-thread block owns 8 CONSECUTIVE elements of one of the block's
// two 1024-element chunks (128 threads = 2 waves per chunk): 16-B loads / stores of g and e, and
// its 8 sign bits are exactly one byte of the packed words (element i -> word i / 64, bit i % 64
// == byte i / 8, bit i % 8 in little-endian memory), stored as a byte -- a wave writes 64
// consecutive bytes.  The chunk's mean |c| is a 2-wave reduction through LDS.  (The previous
// element-strided kernel with a wave64 ballot per word ran at ~0.4 TB/s: 0.49 ms per 64 MB
// bf16 bucket, profiles/r5_llama_width_onebit.txt.)
// MOM (1-bit Adam, compressing the worker's MOMENTUM instead of its gradient): m = beta1 m + (1 - beta1) g
// first (m in E, stored back), then c = m + e; the owner runs Adam with beta1 = 0 and a frozen variance
// on the decoded momenta (parallel/updaters.py OneBitAdamUpdater).
template <typename G, typename E, bool MOM>
__global__ __launch_bounds__(256) void onebit_pack_kernel(const G* __restrict__ g, E* __restrict__ err, int64_t n,
                                                          uint8_t* __restrict__ wbytes, float* __restrict__ scales,
                                                          E* __restrict__ mom, float beta1) {
  __shared__ float part[4];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int64_t chunk = static_cast<int64_t>(blockIdx.x) * 2 + (t >> 7);
  const int64_t base = chunk * kOnebitChunk;
  const int64_t i0 = base + static_cast<int64_t>(t & 127) * 8;
  float c[8];
  float asum = 0.f;
  const bool full = i0 + 8 <= n;
  if (full) {
    float gv[8], ev[8];
    load8(g, i0, gv);
    load8(err, i0, ev);
    if constexpr (MOM) {
      float mv[8];
      load8(mom, i0, mv);
#pragma unroll
      for (int k = 0; k < 8; ++k) gv[k] = beta1 * mv[k] + (1.f - beta1) * gv[k];
      store8(mom, i0, gv);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      c[k] = gv[k] + ev[k];
      asum += fabsf(c[k]);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t i = i0 + k;
      float gk = 0.f;
      if (i < n) {
        gk = Elem<G>::load(g, i);
        if constexpr (MOM) {
          gk = beta1 * Elem<E>::load(mom, i) + (1.f - beta1) * gk;
          Elem<E>::store(mom, i, gk);
        }
      }
      c[k] = i < n ? gk + Elem<E>::load(err, i) : 0.f;
      asum += fabsf(c[k]);
    }
  }
  asum = wave_sum(asum);
  if (lane == 0) part[wid] = asum;
  __syncthreads();
  if (base >= n) return;  // (a block's second chunk past the end: after the barrier)
  const float tot = part[(wid & ~1)] + part[(wid & ~1) + 1];
  const int64_t valid = (n - base) < kOnebitChunk ? (n - base) : kOnebitChunk;
  const float scale = tot / static_cast<float>(valid);
  if ((t & 127) == 0) scales[chunk] = scale;
  if (i0 >= n) {  // past the end inside the last word: zero bits, as the host layout pads
    if (i0 < ((n + 63) & ~int64_t(63))) wbytes[i0 >> 3] = 0;
    return;
  }
  unsigned byte = 0;
  float e[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool pos = (i0 + k < n) && c[k] >= 0.f;  // padded elements contribute 0 bits
    byte |= (pos ? 1u : 0u) << k;
    e[k] = c[k] - (pos ? scale : -scale);
  }
  if (full) {
    store8(err, i0, e);
  } else {
    for (int k = 0; k < 8 && i0 + k < n; ++k) Elem<E>::store(err, i0 + k, e[k]);
  }
  wbytes[i0 >> 3] = static_cast<uint8_t>(byte);
}

// m = beta1 m + (1 - beta1) g: the worker momentum of 1-bit Adam during the full-precision warm-up
// rounds (the push itself is the uncompressed gradient then), so the compressed phase starts from it.
template <typename G, typename E>
__global__ __launch_bounds__(256) void onebit_momentum_kernel(const G* __restrict__ g, E* __restrict__ mom, int64_t n,
                                                              float beta1) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t * 8 < n; t += stride) {
    const int64_t i0 = t * 8;
    if (i0 + 8 <= n) {
      float gv[8], mv[8];
      load8(g, i0, gv);
      load8(mom, i0, mv);
#pragma unroll
      for (int k = 0; k < 8; ++k) mv[k] = beta1 * mv[k] + (1.f - beta1) * gv[k];
      store8(mom, i0, mv);
    } else {
      for (int64_t i = i0; i < n; ++i)
        Elem<E>::store(mom, i, beta1 * Elem<E>::load(mom, i) + (1.f - beta1) * Elem<G>::load(g, i));
    }
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

void launch_onebit_pack(const void* g, int gdtype, void* err, int edtype, int64_t n, uint64_t* words, float* scales,
                        hipStream_t s, void* mom, float beta1) {
  if (n <= 0) return;
  const int64_t nchunks = (n + kOnebitChunk - 1) / kOnebitChunk;
  const int64_t nblk = (nchunks + 1) / 2;
  uint8_t* wb = reinterpret_cast<uint8_t*>(words);
#define PSAMD_PACK(G, E)                                                                                             \
  if (mom != nullptr)                                                                                                \
    hipLaunchKernelGGL((onebit_pack_kernel<G, E, true>), dim3(nblk), dim3(256), 0, s, static_cast<const G*>(g),      \
                       static_cast<E*>(err), n, wb, scales, static_cast<E*>(mom), beta1);                            \
  else                                                                                                               \
    hipLaunchKernelGGL((onebit_pack_kernel<G, E, false>), dim3(nblk), dim3(256), 0, s, static_cast<const G*>(g),     \
                       static_cast<E*>(err), n, wb, scales, static_cast<E*>(nullptr), 0.f)
  if (gdtype == 1 && edtype == 1) PSAMD_PACK(uint16_t, uint16_t);
  else if (gdtype == 1) PSAMD_PACK(uint16_t, float);
  else if (edtype == 1) PSAMD_PACK(float, uint16_t);
  else PSAMD_PACK(float, float);
#undef PSAMD_PACK
}

void launch_onebit_momentum(const void* g, int gdtype, void* mom, int mdtype, int64_t n, float beta1, hipStream_t s) {
  if (n <= 0) return;
  const int grid = stream_grid((n + 7) / 8, 256);
#define PSAMD_MOM(G, E)                                                                                       \
  hipLaunchKernelGGL((onebit_momentum_kernel<G, E>), dim3(grid), dim3(256), 0, s, static_cast<const G*>(g), \
                     static_cast<E*>(mom), n, beta1)
  if (gdtype == 1 && mdtype == 1) PSAMD_MOM(uint16_t, uint16_t);
  else if (gdtype == 1) PSAMD_MOM(uint16_t, float);
  else if (mdtype == 1) PSAMD_MOM(float, uint16_t);
  else PSAMD_MOM(float, float);
#undef PSAMD_MOM
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
