// Sparse-row kernels for embedding / wide tables (K5-K8, K24, K28, K29 in SURVEY §2.5).
//
// Reference: each embedding row is its own PS key "<field>.<id>" pulled and pushed one RPC
// at a time (layer/EmbeddingField.java:57-104, store/KVStore.java:74-127); each wide weight
// is a 1x1 key "wide.weights.<id>" (layer/LRLayer.java:62-120).  Here a table is one dense
// fp32 [rows, dim] array on its owner rank and rows move as batches:
//
//  gather_rows          owner side of pull_rows: out[r] = act(table[rows[r]])  (one wave/row,
//                       16-B loads; writes into an arbitrary column slice of a wider output
//                       buffer so the reference ConcatLayer copy is free, K9)
//  segment_reduce_rows  worker side of push_rows: per unique id, sum (or mean) of its
//                       occurrence rows, read through a sorted permutation; deterministic,
//                       no atomics (cdna_hip_programming.md Appendix B, store-and-sum form)
//  scatter_add_rows     owner side apply for plain accumulate (unique rows => no conflicts)
//  embedding_bag_fwd    fused per-field lookup for the reference EmbeddingLayer: ids[b, f]
//                       -> out[b, off + f*dim : off + (f+1)*dim] with ReLU (layer/EmbeddingLayer.java:36-46)
//  sparse_lr_fwd        z[b] = sum_f w[ids[b,f] mod H] + bias (layer/LRLayer.java:62-98 with
//                       the hash of util/MatrixUtil.java:27-33 fused in)
//  lazy_init_rows       deterministic first-touch row init keyed by (seed, global key) with an
//                       "initialized" byte map; replaces the upsert(replace=false) round trip
//                       (store/KVStore.java:86-107, net/PServer.java:143-162)
//  hash_slots           device-resident id -> slot map (open addressing, CAS insert) for
//                       tables keyed by unbounded ids; no host round trip per lookup
#include <algorithm>

#include "psamd_device.h"
#include "psamd_launch.h"

namespace psamd {

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == 1) return v > 0.f ? v : 0.f;
  if (act == 2) return v > 0.f ? v : 0.01f * v;
  if (act == 3) return 0.001f + 0.998f / (1.f + __expf(-v));
  return v;
}

template <typename T, typename O>
__global__ __launch_bounds__(256) void gather_rows_kernel(const T* __restrict__ table, const int64_t* __restrict__ rows,
                                                          int64_t nrows, int dim, O* __restrict__ out, int64_t out_ld,
                                                          int64_t out_off, int act) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t r = wave; r < nrows; r += nwaves) {
    const int64_t row = rows[r];
    O* dst = out + r * out_ld + out_off;
    if (row < 0) {  // unresolved key (map overflow): zero row, wave-uniform branch
      for (int c = lane; c < dim; c += 64) Elem<O>::store(dst, c, 0.f);
      continue;
    }
    const T* src = table + row * dim;
    for (int c = lane; c < dim; c += 64) Elem<O>::store(dst, c, apply_act(Elem<T>::load(src, c), act));
  }
}

// vectorized: dim % 4 == 0, fp32 table, fp32 out, 16-B aligned rows
__global__ __launch_bounds__(256) void gather_rows_vec4_kernel(const float* __restrict__ table,
                                                               const int64_t* __restrict__ rows, int64_t nrows,
                                                               int dim, float* __restrict__ out, int64_t out_ld,
                                                               int64_t out_off, int act) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  const int d4 = dim >> 2;
  for (int64_t r = wave; r < nrows; r += nwaves) {
    const int64_t row = rows[r];
    f32x4* dst = reinterpret_cast<f32x4*>(out + r * out_ld + out_off);
    if (row < 0) {
      for (int c = lane; c < d4; c += 64) dst[c] = f32x4{0.f, 0.f, 0.f, 0.f};
      continue;
    }
    const f32x4* src = reinterpret_cast<const f32x4*>(table + row * dim);
    for (int c = lane; c < d4; c += 64) {
      f32x4 v = src[c];
      v.x = apply_act(v.x, act); v.y = apply_act(v.y, act); v.z = apply_act(v.z, act); v.w = apply_act(v.w, act);
      dst[c] = v;
    }
  }
}

// dim = 4 * 2^lg <= 256, fp32 table, fp32 or bf16 out: 2^lg lanes per row, 16-B loads, 64 >> lg
// rows per wave in flight
template <typename O>
__global__ __launch_bounds__(256) void gather_rows_lg_kernel(const float* __restrict__ table,
                                                             const int64_t* __restrict__ rows, int64_t nrows,
                                                             int dim, int lg, O* __restrict__ out, int64_t out_ld,
                                                             int64_t out_off, int act) {
  const int lane = threadIdx.x & 63;
  const int sub = lane >> lg;
  const int c = (lane & ((1 << lg) - 1)) * 4;
  const int per_wave = 64 >> lg;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t rb = wave * per_wave; rb < nrows; rb += nwaves * per_wave) {
    const int64_t r = rb + sub;
    if (r >= nrows) continue;
    const int64_t row = rows[r];
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (row >= 0) {
      v = load4(table, row * dim + c);
      v.x = apply_act(v.x, act); v.y = apply_act(v.y, act); v.z = apply_act(v.z, act); v.w = apply_act(v.w, act);
    }
    store4(out, r * out_ld + out_off + c, v);
  }
}

static int lg_of(int dim) {
  if (dim % 4 != 0 || dim > 256) return -1;
  const int l = dim / 4;
  if ((l & (l - 1)) != 0) return -1;
  int lg = 0;
  while ((1 << lg) < l) ++lg;
  return lg;
}

void launch_gather_rows(const void* table, int tdtype, const int64_t* rows, int64_t nrows, int dim, void* out,
                        int odtype, int64_t out_ld, int64_t out_off, int act, hipStream_t s) {
  if (nrows <= 0) return;
  const int lg = lg_of(dim);
  const int oes = odtype == 1 ? 2 : 4;
  if (tdtype == 0 && lg >= 0 && out_ld % 4 == 0 && out_off % 4 == 0 &&
      ((reinterpret_cast<uintptr_t>(table) & 15) | (reinterpret_cast<uintptr_t>(out) & (oes * 4 - 1))) == 0) {
    const int g = stream_grid(((nrows << lg) + 63) / 64 * 64, 256);
    if (odtype == 1)
      hipLaunchKernelGGL(gather_rows_lg_kernel<uint16_t>, dim3(g), dim3(256), 0, s, static_cast<const float*>(table),
                         rows, nrows, dim, lg, static_cast<uint16_t*>(out), out_ld, out_off, act);
    else
      hipLaunchKernelGGL(gather_rows_lg_kernel<float>, dim3(g), dim3(256), 0, s, static_cast<const float*>(table),
                         rows, nrows, dim, lg, static_cast<float*>(out), out_ld, out_off, act);
    return;
  }
  const int grid = stream_grid(nrows * 64, 256);
  const bool vec = tdtype == 0 && odtype == 0 && dim % 4 == 0 && out_ld % 4 == 0 && out_off % 4 == 0 &&
                   ((reinterpret_cast<uintptr_t>(table) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  if (vec) {
    hipLaunchKernelGGL(gather_rows_vec4_kernel, dim3(grid), dim3(256), 0, s, static_cast<const float*>(table), rows,
                       nrows, dim, static_cast<float*>(out), out_ld, out_off, act);
    return;
  }
#define PSAMD_G(T, O)                                                                                                \
  hipLaunchKernelGGL((gather_rows_kernel<T, O>), dim3(grid), dim3(256), 0, s, static_cast<const T*>(table), rows, \
                     nrows, dim, static_cast<O*>(out), out_ld, out_off, act);
  if (tdtype == 1 && odtype == 1) PSAMD_G(uint16_t, uint16_t)
  else if (tdtype == 1) PSAMD_G(uint16_t, float)
  else if (odtype == 1) PSAMD_G(float, uint16_t)
  else PSAMD_G(float, float)
#undef PSAMD_G
}

// out[u] = (mean ? 1/cnt : 1) * sum_{j in [seg_off[u], seg_off[u+1])} src[perm[j]]
template <typename S, typename O>
__global__ __launch_bounds__(256) void segment_reduce_rows_kernel(const S* __restrict__ src,
                                                                  const int64_t* __restrict__ perm,
                                                                  const int64_t* __restrict__ seg_off, int64_t nseg,
                                                                  int dim, O* __restrict__ out, int mean) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t u = wave; u < nseg; u += nwaves) {
    const int64_t b = seg_off[u], e = seg_off[u + 1];
    const float inv = mean ? 1.f / static_cast<float>(e - b) : 1.f;
    for (int c = lane; c < dim; c += 64) {
      float acc = 0.f;
      for (int64_t j = b; j < e; ++j) acc += Elem<S>::load(src + perm[j] * dim, c);
      Elem<O>::store(out + u * dim, c, acc * inv);
    }
  }
}

// vectorised: dim = 4 * 2^lg <= 256, 2^lg lanes per segment, 4 elements (16 B) per lane, the
// segment's running sum in registers
template <typename S, typename O>
__global__ __launch_bounds__(256) void segment_reduce_rows_vec_kernel(const S* __restrict__ src,
                                                                      const int64_t* __restrict__ perm,
                                                                      const int64_t* __restrict__ seg_off,
                                                                      int64_t nseg, int dim, int lg,
                                                                      O* __restrict__ out, int mean) {
  const int lane = threadIdx.x & 63;
  const int sub = lane >> lg;
  const int c = (lane & ((1 << lg) - 1)) * 4;
  const int per_wave = 64 >> lg;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t ub = wave * per_wave; ub < nseg; ub += nwaves * per_wave) {
    const int64_t u = ub + sub;
    if (u >= nseg) continue;
    const int64_t b = seg_off[u], e = seg_off[u + 1];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int64_t j = b;
    // 4 independent row loads in flight: hot ids (long segments) are latency chains otherwise
    for (; j + 4 <= e; j += 4) {
      const int64_t p0 = perm[j], p1 = perm[j + 1], p2 = perm[j + 2], p3 = perm[j + 3];
      const f32x4 v0 = load4(src, p0 * dim + c), v1 = load4(src, p1 * dim + c);
      const f32x4 v2 = load4(src, p2 * dim + c), v3 = load4(src, p3 * dim + c);
      acc += (v0 + v1) + (v2 + v3);
    }
    for (; j < e; ++j) acc += load4(src, perm[j] * dim + c);
    if (mean) acc *= 1.f / static_cast<float>(e - b > 0 ? e - b : 1);
    store4(out, u * dim + c, acc);
  }
}

static int vec_lg(int dim) {
  if (dim % 4 != 0 || dim > 256) return -1;
  const int l = dim / 4;
  if ((l & (l - 1)) != 0) return -1;
  int lg = 0;
  while ((1 << lg) < l) ++lg;
  return lg;
}

void launch_segment_reduce_rows(const void* src, int sdtype, const int64_t* perm, const int64_t* seg_off,
                                int64_t nseg, int dim, void* out, int odtype, int mean, hipStream_t s) {
  if (nseg <= 0) return;
  const int lg = vec_lg(dim);
  if (lg >= 0 && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(out)) & 15) == 0) {
    const int grid = stream_grid(((nseg << lg) + 63) / 64 * 64, 256);
#define PSAMD_SV(S, O)                                                                                              \
  hipLaunchKernelGGL((segment_reduce_rows_vec_kernel<S, O>), dim3(grid), dim3(256), 0, s, static_cast<const S*>(src), \
                     perm, seg_off, nseg, dim, lg, static_cast<O*>(out), mean);
    if (sdtype == 1 && odtype == 1) PSAMD_SV(uint16_t, uint16_t)
    else if (sdtype == 1) PSAMD_SV(uint16_t, float)
    else if (odtype == 1) PSAMD_SV(float, uint16_t)
    else PSAMD_SV(float, float)
#undef PSAMD_SV
    return;
  }
  const int grid = stream_grid(nseg * 64, 256);
#define PSAMD_S(S, O)                                                                                           \
  hipLaunchKernelGGL((segment_reduce_rows_kernel<S, O>), dim3(grid), dim3(256), 0, s, static_cast<const S*>(src), \
                     perm, seg_off, nseg, dim, static_cast<O*>(out), mean);
  if (sdtype == 1 && odtype == 1) PSAMD_S(uint16_t, uint16_t)
  else if (sdtype == 1) PSAMD_S(uint16_t, float)
  else if (odtype == 1) PSAMD_S(float, uint16_t)
  else PSAMD_S(float, float)
#undef PSAMD_S
}

template <typename S>
__global__ __launch_bounds__(256) void scatter_add_rows_kernel(const S* __restrict__ src,
                                                               const int64_t* __restrict__ rows, int64_t nrows,
                                                               int dim, float* __restrict__ table) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t r = wave; r < nrows; r += nwaves) {
    float* dst = table + rows[r] * dim;
    for (int c = lane; c < dim; c += 64) dst[c] += Elem<S>::load(src + r * dim, c);
  }
}

void launch_scatter_add_rows(const void* src, int sdtype, const int64_t* rows, int64_t nrows, int dim, float* table,
                             hipStream_t s) {
  if (nrows <= 0) return;
  const int grid = stream_grid(nrows * 64, 256);
  if (sdtype == 1)
    hipLaunchKernelGGL(scatter_add_rows_kernel<uint16_t>, dim3(grid), dim3(256), 0, s,
                       static_cast<const uint16_t*>(src), rows, nrows, dim, table);
  else
    hipLaunchKernelGGL(scatter_add_rows_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<const float*>(src),
                       rows, nrows, dim, table);
}

// ids[b, f] are owner-local row indices into table (per-field offsets already applied)
template <typename O>
__global__ __launch_bounds__(256) void embedding_bag_fwd_kernel(const float* __restrict__ table,
                                                                const int64_t* __restrict__ ids, int64_t batch,
                                                                int fields, int dim, O* __restrict__ out,
                                                                int64_t out_ld, int64_t out_off, int act) {
  const int64_t total = batch * fields * dim;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t b = i / (static_cast<int64_t>(fields) * dim);
    const int64_t rem = i - b * fields * dim;
    const int f = static_cast<int>(rem / dim);
    const int d = static_cast<int>(rem - static_cast<int64_t>(f) * dim);
    const float v = table[ids[b * fields + f] * dim + d];
    Elem<O>::store(out, b * out_ld + out_off + rem, apply_act(v, act));
  }
}

void launch_embedding_bag_fwd(const float* table, const int64_t* ids, int64_t batch, int fields, int dim, void* out,
                              int odtype, int64_t out_ld, int64_t out_off, int act, hipStream_t s) {
  const int64_t total = batch * fields * dim;
  if (total <= 0) return;
  const int grid = stream_grid(total, 256);
  if (odtype == 1)
    hipLaunchKernelGGL(embedding_bag_fwd_kernel<uint16_t>, dim3(grid), dim3(256), 0, s, table, ids, batch, fields, dim,
                       static_cast<uint16_t*>(out), out_ld, out_off, act);
  else
    hipLaunchKernelGGL(embedding_bag_fwd_kernel<float>, dim3(grid), dim3(256), 0, s, table, ids, batch, fields, dim,
                       static_cast<float*>(out), out_ld, out_off, act);
}

// one wave per sample; lanes stride over fields
__global__ __launch_bounds__(256) void sparse_lr_fwd_kernel(const float* __restrict__ w, const int64_t* __restrict__ ids,
                                                            int64_t batch, int fields, int64_t hash_size,
                                                            const float* __restrict__ bias, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t b = wave; b < batch; b += nwaves) {
    float acc = 0.f;
    for (int f = lane; f < fields; f += 64) {
      int64_t id = ids[b * fields + f] % hash_size;
      if (id < 0) id += hash_size;
      acc += w[id];
    }
    acc = wave_sum(acc);
    if (lane == 0) out[b] = acc + (bias ? bias[0] : 0.f);
  }
}

void launch_sparse_lr_fwd(const float* w, const int64_t* ids, int64_t batch, int fields, int64_t hash_size,
                          const float* bias, float* out, hipStream_t s) {
  if (batch <= 0) return;
  const int grid = stream_grid(batch * 64, 256);
  hipLaunchKernelGGL(sparse_lr_fwd_kernel, dim3(grid), dim3(256), 0, s, w, ids, batch, fields, hash_size, bias, out);
}

__device__ __forceinline__ int vec_lanes_log2_dev(int dim) {  // lanes per row: dim = 4 * 2^lg <= 256
  if (dim % 4 != 0 || dim > 256) return -1;
  const int l = dim / 4;
  if ((l & (l - 1)) != 0) return -1;
  return __builtin_ctz(l);
}

// rows: owner-local indices (negative = unresolved, skipped).  The RNG is keyed by the row's
// GLOBAL key -- keys[r] when given (hash-mapped tables: the raw id), else row + row_base (range
// partitioned tables: the global row) -- so a row's initial value does not depend on which rank
// owns it, which slot it landed in, or when it is first touched (first-writer-wins for free).
__global__ __launch_bounds__(256) void lazy_init_rows_kernel(float* __restrict__ table, const int64_t* __restrict__ rows,
                                                             const int64_t* __restrict__ keys, int64_t nrows, int dim,
                                                             uint8_t* __restrict__ flags, uint64_t seed,
                                                             int64_t row_base, float lo, float hi) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  const float span = hi - lo;
  // 64 rows per wave step: every lane checks one row's flag, the rows still to be created are
  // ballotted and then initialised P = 64 / L at a time, L = dim / 4 lanes per row when dim is
  // 4 * 2^k <= 256 (each lane one Philox call -> one 16-B store), else one row at a time by the
  // whole wave.  Steady state: almost every row exists, so the kernel is one coalesced flag probe
  // per 64 rows; a fresh batch keeps every lane busy.
  const int lg = vec_lanes_log2_dev(dim);
  const int L = lg >= 0 ? (1 << lg) : 64, P = 64 / L, sub = lane / L, ql = lane % L;
  for (int64_t base = wave * 64; base < nrows; base += nwaves * 64) {
    const int64_t r = base + lane;
    const int64_t row = r < nrows ? rows[r] : -1;
    const bool need = row >= 0 && flags[row] == 0;
    const int64_t key = need ? (keys ? keys[r] : row + row_base) : 0;
    uint64_t todo = __ballot(need);
    while (todo) {
      uint64_t t = todo;  // this lane group's row: the sub-th remaining set bit
      for (int k = 0; k < sub; ++k) t &= t - 1;
      for (int k = 0; k < P; ++k) todo &= todo - 1;
      const int l = t ? __ffsll(static_cast<unsigned long long>(t)) - 1 : 0;
      const int64_t rr = __shfl(row, l, 64);
      const uint64_t grow = static_cast<uint64_t>(__shfl(key, l, 64));
      if (!t) continue;
      // one Philox call yields the 4 values of elements 4q .. 4q+3: 128-bit counter (q, key), so
      // map-mode keys (field << 44 | id) keep their field bits and every field gets its own rows
      for (int q = ql; q * 4 < dim; q += L) {
        uint32_t rnd[4];
        Philox::gen(seed, static_cast<uint64_t>(q), rnd, grow);
        float* dst = table + rr * dim + q * 4;
        if (q * 4 + 4 <= dim && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0)) {
          store4(dst, 0, f32x4{lo + span * Philox::u01(rnd[0]), lo + span * Philox::u01(rnd[1]),
                               lo + span * Philox::u01(rnd[2]), lo + span * Philox::u01(rnd[3])});
        } else {
          for (int k = 0; k < 4 && q * 4 + k < dim; ++k) dst[k] = lo + span * Philox::u01(rnd[k]);
        }
      }
    }
    // duplicates inside one launch re-initialise identically; flags go up after the rows
    if (need) flags[row] = 1;
  }
}

void launch_lazy_init_rows(float* table, const int64_t* rows, const int64_t* keys, int64_t nrows, int dim,
                           uint8_t* init_flags, uint64_t seed, int64_t row_base, float lo, float hi, hipStream_t s) {
  if (nrows <= 0) return;
  const int grid = stream_grid((nrows + 63) / 64 * 64, 256);
  hipLaunchKernelGGL(lazy_init_rows_kernel, dim3(grid), dim3(256), 0, s, table, rows, keys, nrows, dim, init_flags,
                     seed, row_base, lo, hi);
}

// ---------------------------------------------------------------------------------------
// Device-resident id -> slot map for hash-mapped ("map" mode) sparse tables: open addressing
// with linear probing over a power-of-two key array initialised to -1.  The slot of a key IS
// its probe position, so creation needs no counter and no second pass: the lane whose 64-bit
// compare-and-swap claims an empty position owns it, a lane that loses the race to the SAME
// key (another worker asked for it in this launch) reads that key back and shares the slot.
// This replaces the reference's upsert(replace=false) round trip for rows that do not exist
// yet (store/KVStore.java:86-107, net/PServer.java:143-162) without a host lookup.  A key
// that finds the table full (or is absent with insert=0) gets slot -1; ``status`` is set to 1
// with a plain store so the host can check it at its next sync point.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix_key(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__global__ __launch_bounds__(256) void hash_slots_kernel(unsigned long long* __restrict__ hkeys, int64_t cap_mask,
                                                         const int64_t* __restrict__ ids, int64_t n,
                                                         int64_t* __restrict__ out, int insert,
                                                         int32_t* __restrict__ status) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const unsigned long long kEmpty = ~0ull;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const unsigned long long key = static_cast<unsigned long long>(ids[i]);
    int64_t slot = -1;
    if (ids[i] >= 0) {
      uint64_t h = mix_key(key) & static_cast<uint64_t>(cap_mask);
      for (int64_t probe = 0; probe <= cap_mask; ++probe) {
        unsigned long long cur = __hip_atomic_load(&hkeys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == key) { slot = static_cast<int64_t>(h); break; }
        if (cur == kEmpty) {
          if (!insert) break;
          const unsigned long long prev = atomicCAS(&hkeys[h], kEmpty, key);
          if (prev == kEmpty || prev == key) { slot = static_cast<int64_t>(h); break; }
        }
        h = (h + 1) & static_cast<uint64_t>(cap_mask);
      }
    }
    out[i] = slot;
    if (slot < 0 && insert && ids[i] >= 0) status[0] = 1;  // negative ids = pad keys (no row)
  }
}

void launch_hash_slots(int64_t* hkeys, int64_t capacity, const int64_t* ids, int64_t n, int64_t* out, int insert,
                       int32_t* status, hipStream_t s) {
  if (n <= 0) return;
  const int grid = stream_grid(n, 256);
  hipLaunchKernelGGL(hash_slots_kernel, dim3(grid), dim3(256), 0, s, reinterpret_cast<unsigned long long*>(hkeys),
                     capacity - 1, ids, n, out, insert, status);
}

// Compaction of sorted keys: for every run head i (i == 0 or srt[i] != srt[i-1]) with unique
// index uidx[i] (inclusive scan of the head flags, minus 1): ukeys[u] = srt[i] & mask,
// seg[u] = i, and seg[nu] = n -- the (unique keys, segment offsets) of a pull plan without the
// host needing nu first (outputs are sized n and n + 1).
__global__ __launch_bounds__(256) void unique_runs_kernel(const int64_t* __restrict__ srt,
                                                          const int64_t* __restrict__ uidx, int64_t n, int64_t mask,
                                                          int64_t* __restrict__ ukeys, int64_t* __restrict__ seg) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t u = uidx[i];
    if (i == 0 || srt[i] != srt[i - 1]) {
      ukeys[u] = srt[i] & mask;
      seg[u] = i;
    }
    if (i == n - 1) seg[u + 1] = n;
  }
}

void launch_unique_runs(const int64_t* srt, const int64_t* uidx, int64_t n, int64_t mask, int64_t* ukeys,
                        int64_t* seg, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(unique_runs_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, s, srt, uidx, n, mask, ukeys, seg);
}

// ---------------------------------------------------------------------------------------
// One-node row exchange over IPC-mapped arenas (parallel/row_plane.py): every rank publishes its
// unique keys sorted by owner, with [offset | count] per owner, in its own arena; owners read
// their segments straight from the peers' arenas and write the rows straight back; pushes are
// read the same way.  Counts stay in device memory -- no split sizes on the host.  Entry e of
// the owner's [W][cap] view is worker e / cap's key e % cap (pads: key -1 / slot -1).
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void row_plane_recv_kernel(const RowPeers P, int me, int64_t cap,
                                                             int64_t* __restrict__ rkeys, int64_t* __restrict__ pmeta) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // peers' keys / counts: no stale lines (system scope)
  const int64_t total = static_cast<int64_t>(P.W) * cap;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < total; e += stride) {
    const int w = static_cast<int>(e / cap);
    const int64_t j = e - w * cap;
    const int64_t off = P.meta[w][me], cnt = P.meta[w][P.W + me];
    rkeys[e] = j < cnt ? P.skeys[w][off + j] : -1;
    if (j == 0) {
      pmeta[2 * w] = off;
      pmeta[2 * w + 1] = cnt;
    }
  }
}

// rows of the owner's slots -> worker w's arena rows at its offset (slot < 0: zero row).
// Blocks never straddle two workers (cap % (entries per block) == 0) and skip pad blocks whole.
template <int V>
__global__ __launch_bounds__(256) void row_plane_send_kernel(const float* __restrict__ table,
                                                             const int64_t* __restrict__ rslots,
                                                             const int64_t* __restrict__ pmeta, const RowPeers P,
                                                             int64_t cap, int dim, int lpe) {
  // lpe lanes per entry (each V floats per step), 256 / lpe entries per block-step
  const int epb = 256 / lpe;
  const int64_t nblocks = static_cast<int64_t>(P.W) * cap / epb;
  const int sub = threadIdx.x / lpe, ql = threadIdx.x % lpe;
  for (int64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
    const int64_t e0 = b * epb;
    const int w = static_cast<int>(e0 / cap);
    const int64_t j0 = e0 - w * cap;
    const int64_t cnt = pmeta[2 * w + 1];
    if (j0 >= cnt) continue;  // block-uniform: a block of pads
    const int64_t j = j0 + sub;
    if (j >= cnt) continue;
    const int64_t slot = rslots[e0 + sub];
    float* dst = P.rows[w] + (pmeta[2 * w] + j) * dim;
    for (int c = ql * V; c < dim; c += lpe * V) {
      if constexpr (V == 4) {
        const f32x4 v = slot >= 0 ? load4(table, slot * dim + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        store4(dst, c, v);
      } else {
        dst[c] = slot >= 0 ? table[slot * dim + c] : 0.f;
      }
    }
  }
}

// one worker's pushed rows into the owner's fp32 accumulator (pass w of W, launched in rank
// order: deterministic sums, no atomics on the data).  A slot first seen this round (tflag !=
// tag) is appended to the touched list and its accumulator row overwritten instead of added to.
// Each block owns a contiguous chunk of kAccChunk entries and collects its first-touched slots in
// LDS (LDS atomics), then reserves their range of the touched list with ONE global atomic: a
// global atomic per first touch (one address, ~1M times per DLRM push) had serialised the kernel
// at ~0.3 TB/s (profiles/r5_dlrm_w2_row_plane_stages_before.json).  The list order is arbitrary;
// the apply updates each listed row once, so the result does not depend on it.
constexpr int kAccChunk = 1024;
template <int V>
__global__ __launch_bounds__(256) void row_plane_accum_kernel(const RowPeers P, int w, const int64_t* __restrict__ rslots,
                                                              const int64_t* __restrict__ pmeta, float* __restrict__ acc,
                                                              int32_t* __restrict__ tflag, int32_t tag,
                                                              int64_t* __restrict__ touched, int32_t* __restrict__ tcount,
                                                              int64_t cap, int dim, int lpe) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // worker w's pushed rows (system scope)
  __shared__ int64_t lslots[kAccChunk];
  __shared__ int lcount, lbase;
  const int epb = 256 / lpe;
  const int64_t cnt = pmeta[2 * w + 1], off = pmeta[2 * w];
  const int64_t j0 = static_cast<int64_t>(blockIdx.x) * kAccChunk;
  if (j0 >= cnt) return;  // block-uniform
  if (threadIdx.x == 0) lcount = 0;
  __syncthreads();
  const int64_t j1 = min(cnt, j0 + kAccChunk);
  const int sub = threadIdx.x / lpe, ql = threadIdx.x % lpe;
  const float* src = P.grads[w];
  for (int64_t jb = j0; jb < j1; jb += epb) {
    const int64_t j = jb + sub;
    const int64_t slot = j < j1 ? rslots[static_cast<int64_t>(w) * cap + j] : -1;
    // every lane of the entry reads the flag before its first lane writes it (one wave, in order)
    const bool first = slot >= 0 && tflag[slot] != tag;
    if (slot >= 0 && ql == 0 && first) {
      tflag[slot] = tag;
      lslots[atomicAdd(&lcount, 1)] = slot;
    }
    if (slot < 0) continue;
    const float* g = src + (off + j) * dim;
    float* a = acc + slot * dim;
    for (int c = ql * V; c < dim; c += lpe * V) {
      if constexpr (V == 4) {
        f32x4 v = load4(g, c);
        if (!first) v += load4(a, c);
        store4(a, c, v);
      } else {
        a[c] = first ? g[c] : a[c] + g[c];
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) lbase = lcount ? atomicAdd(tcount, lcount) : 0;
  __syncthreads();
  for (int i = threadIdx.x; i < lcount; i += blockDim.x) touched[lbase + i] = lslots[i];
}

static int row_lanes(int dim, int V) {  // lanes per entry: a power of two <= 64 covering dim / V
  int need = (dim + V - 1) / V, l = 1;
  while (l < need && l < 64) l <<= 1;
  return l;
}

void launch_row_plane_recv(const RowPeers& P, int me, int64_t cap, int64_t* rkeys, int64_t* pmeta, hipStream_t s) {
  const int64_t total = static_cast<int64_t>(P.W) * cap;
  if (total <= 0) return;
  hipLaunchKernelGGL(row_plane_recv_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, s, P, me, cap, rkeys, pmeta);
}

void launch_row_plane_send(const float* table, const int64_t* rslots, const int64_t* pmeta, const RowPeers& P,
                           int64_t cap, int dim, hipStream_t s) {
  const bool v4 = dim % 4 == 0;
  const int lpe = row_lanes(dim, v4 ? 4 : 1);
  const int64_t nblocks = static_cast<int64_t>(P.W) * cap / (256 / lpe);
  if (nblocks <= 0) return;
  const int grid = static_cast<int>(std::min<int64_t>(nblocks, 65536));
  if (v4) hipLaunchKernelGGL(row_plane_send_kernel<4>, dim3(grid), dim3(256), 0, s, table, rslots, pmeta, P, cap, dim, lpe);
  else hipLaunchKernelGGL(row_plane_send_kernel<1>, dim3(grid), dim3(256), 0, s, table, rslots, pmeta, P, cap, dim, lpe);
}

void launch_row_plane_accum(const RowPeers& P, const int64_t* rslots, const int64_t* pmeta, float* acc, int32_t* tflag,
                            int32_t tag, int64_t* touched, int32_t* tcount, int64_t cap, int dim, hipStream_t s) {
  const bool v4 = dim % 4 == 0;
  const int lpe = row_lanes(dim, v4 ? 4 : 1);
  const int grid = static_cast<int>(std::max<int64_t>(1, (cap + kAccChunk - 1) / kAccChunk));
  for (int w = 0; w < P.W; ++w) {  // rank order
    if (v4)
      hipLaunchKernelGGL(row_plane_accum_kernel<4>, dim3(grid), dim3(256), 0, s, P, w, rslots, pmeta, acc, tflag, tag,
                         touched, tcount, cap, dim, lpe);
    else
      hipLaunchKernelGGL(row_plane_accum_kernel<1>, dim3(grid), dim3(256), 0, s, P, w, rslots, pmeta, acc, tflag, tag,
                         touched, tcount, cap, dim, lpe);
  }
}

// ---------------------------------------------------------------------------------------
// Device-side segment moves between a worker and its owners' mailboxes (async rows,
// parallel/async_rows.py): owner o's piece is [meta[o], meta[o] + meta[W + o]) of the worker's
// owner-sorted buffer; counts stay in device memory (each mailbox carries its count in the word
// after its cap entries).  blockIdx.y = owner; a block stride loop over that owner's piece only.
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void segs_to_peers_kernel(const T* __restrict__ src, const int64_t* __restrict__ meta,
                                                            const PeerSegs P, int64_t width) {
  const int o = blockIdx.y;
  const int64_t off = meta[o], cnt = meta[P.W + o];
  T* dst = static_cast<T*>(P.ptr[o]);
  const int64_t total = cnt * width;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    dst[i] = src[off * width + i];
  if (blockIdx.x == 0 && threadIdx.x == 0 && P.cnt[o] != nullptr) *P.cnt[o] = cnt;
}

template <typename T>
__global__ __launch_bounds__(256) void segs_from_peers_kernel(T* __restrict__ dst, const int64_t* __restrict__ meta,
                                                              const PeerSegs P, int64_t width) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the owners' response rows (system scope)
  const int o = blockIdx.y;
  const int64_t off = meta[o], cnt = meta[P.W + o];
  const T* src = static_cast<const T*>(P.ptr[o]);
  const int64_t total = cnt * width;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    dst[off * width + i] = src[i];
}

void launch_segs_peers(bool to_peers, const void* local, int esize, const int64_t* meta, const PeerSegs& P,
                       int64_t width, int64_t cap, hipStream_t s) {
  if (P.W <= 0 || cap <= 0) return;
  const int gx = static_cast<int>(std::min<int64_t>(std::max<int64_t>(1, (cap * width + 255) / 256), 1024));
  const dim3 grid(gx, P.W);
  if (esize == 8) {
    if (to_peers)
      hipLaunchKernelGGL(segs_to_peers_kernel<int64_t>, grid, dim3(256), 0, s, static_cast<const int64_t*>(local), meta, P,
                         width);
    else
      hipLaunchKernelGGL(segs_from_peers_kernel<int64_t>, grid, dim3(256), 0, s,
                         static_cast<int64_t*>(const_cast<void*>(local)), meta, P, width);
  } else {
    if (to_peers)
      hipLaunchKernelGGL(segs_to_peers_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(local), meta, P,
                         width);
    else
      hipLaunchKernelGGL(segs_from_peers_kernel<float>, grid, dim3(256), 0, s,
                         static_cast<float*>(const_cast<void*>(local)), meta, P, width);
  }
}

// owner-local rows of range-partitioned keys: rows[i] = keys[i] - base (negative keys stay negative)
__global__ __launch_bounds__(256) void keys_to_rows_kernel(const int64_t* __restrict__ keys, int64_t n, int64_t base,
                                                           int64_t* __restrict__ rows) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    rows[i] = keys[i] < 0 ? -1 : keys[i] - base;
}

// a system-scope acquire on every CU (one block each): later kernels of the stream read memory
// peers wrote (over xGMI, after the host saw their completion) without stale cached lines
__global__ __launch_bounds__(64) void system_acquire_kernel() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }

void launch_system_acquire(hipStream_t s) { hipLaunchKernelGGL(system_acquire_kernel, dim3(256), dim3(64), 0, s); }

void launch_keys_to_rows(const int64_t* keys, int64_t n, int64_t base, int64_t* rows, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(keys_to_rows_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, s, keys, n, base, rows);
}

}  // namespace psamd
