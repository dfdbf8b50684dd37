// Host-side launcher declarations for the ps_amd HIP kernels.
//
// The kernels live in csrc/kernels/*.hip (compiled by hipcc for gfx950 only); the torch
// bindings in csrc/bindings.cpp validate tensors and call these launchers on the current
// HIP stream.  Keeping this header free of torch lets the kernel TUs build in seconds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psamd {

// ---------------------------------------------------------------- optim.hip
struct FusedOptArgs {
  int kind;  // 0 sgd, 1 adam, 2 adagrad, 3 ftrl
  float* w;  // fp32 master shard (in/out)
  float* st0;  // momentum / adam m / adagrad h / ftrl z (nullable for plain sgd)
  float* st1;  // adam v / ftrl n (nullable)
  const void* g;  // gradient, bf16 (g_bf16) or fp32
  int g_bf16;
  void* wout;  // optional weight copy-out (pull buffer), bf16 (wout_bf16) or fp32
  int wout_bf16;
  int64_t n;
  float lr, beta1, beta2, eps, wd, momentum, dampening;
  int nesterov, adamw;
  float bc1, bc2;
  float l1, l2, fbeta;
  int ftrl_mode;
  float gscale;
  const float* gscale_ptr;
};
void launch_fused_opt(const FusedOptArgs& a, hipStream_t s);

// Multi-source gradient of the xGMI plane (optim.hip): element q of the gradient is the sum over
// s < nsrc, in order, of source s's value at chunk element off + q -- read from g[s] (bf16 when
// the FusedOptArgs say g_bf16, else fp32), or decoded from 1-bit words[s] / scales[s] (onebit;
// word q >> 6, scale q / kOnebitChunk, pointers at chunk element 0).
constexpr int kPlaneMaxSrc = 16;
struct MultiGrad {
  const void* g[kPlaneMaxSrc];
  const uint64_t* words[kPlaneMaxSrc];
  const float* scales[kPlaneMaxSrc];
  int nsrc;
  int onebit;
  int64_t off;
};
// fused optimizer over a segment (a.w / st / wout at the segment's first element; a.g unused)
void launch_fused_opt_multi(const FusedOptArgs& a, const MultiGrad& m, hipStream_t s);
// reduce only: out[0, n) fp32 = the multi-source gradient of the segment
void launch_reduce_multi(const MultiGrad& m, int g_bf16, int64_t n, float* out, hipStream_t s);

// ---------------------------------------------------------------- plane.hip
// up to kPlaneMaxSrc (src -> dst) copies issued as one launch (16-B aligned, sizes in bytes)
struct PlaneCopies {
  const void* src[kPlaneMaxSrc];
  void* dst[kPlaneMaxSrc];
  int64_t nbytes[kPlaneMaxSrc];
  int nseg;
};
// every segment ``nbytes`` long
void launch_plane_gather(const PlaneCopies& c, int64_t nbytes, hipStream_t s);
// one-node row exchange (sparse.hip, parallel/row_plane.py): every rank's arena pointers
struct RowPeers {
  const int64_t* skeys[kPlaneMaxSrc];  // unique keys sorted by owner
  const int64_t* meta[kPlaneMaxSrc];   // [2W]: offset of owner o's segment, then its count
  float* rows[kPlaneMaxSrc];           // [cap, dim] rows for skeys (written by the owners)
  const float* grads[kPlaneMaxSrc];    // [cap, dim] pushed gradient rows for skeys
  int W;
};
// worker <-> owner mailboxes of the asynchronous row tables: owner o's piece of a worker's
// owner-sorted buffer is [meta[o], meta[o] + meta[W + o]); cnt[o] (nullable) receives the count
struct PeerSegs {
  void* ptr[kPlaneMaxSrc];
  int64_t* cnt[kPlaneMaxSrc];
  int W;
};
void launch_segs_peers(bool to_peers, const void* local, int esize, const int64_t* meta, const PeerSegs& P,
                       int64_t width, int64_t cap, hipStream_t s);
void launch_keys_to_rows(const int64_t* keys, int64_t n, int64_t base, int64_t* rows, hipStream_t s);
void launch_system_acquire(hipStream_t s);
void launch_row_plane_recv(const RowPeers& P, int me, int64_t cap, int64_t* rkeys, int64_t* pmeta, hipStream_t s);
void launch_row_plane_send(const float* table, const int64_t* rslots, const int64_t* pmeta, const RowPeers& P,
                           int64_t cap, int dim, hipStream_t s);
void launch_row_plane_accum(const RowPeers& P, const int64_t* rslots, const int64_t* pmeta, float* acc, int32_t* tflag,
                            int32_t tag, int64_t* touched, int32_t* tcount, int64_t cap, int dim, hipStream_t s);
// segment sizes from c.nbytes
void launch_plane_copy(const PlaneCopies& c, hipStream_t s);
// total = sum_r *(float*)c.src[r] (rank order); factor = min(1, max_norm / (sqrt(total) + 1e-6))
void launch_plane_clip_factor(const PlaneCopies& c, float max_norm, float* total, float* factor, hipStream_t s);
void launch_plane_fill(float* p, int64_t n, float v, hipStream_t s);

struct SparseOptArgs {
  int kind;
  float* table;  // [rows_total, dim] owner-local fp32 table
  float* st0;
  float* st1;
  const int64_t* rows;  // [nrows] owner-local rows: unique (perm null) or sorted with repeats
  const int64_t* perm;  // nullable: grad row of sorted entry j is perm[j] (runs are summed)
  const void* grad;     // [nrows, dim]
  int g_bf16;
  int64_t nrows;
  int dim;
  int rowwise;  // adagrad: one accumulator per row
  int skip_zero;
  float lr, beta1, beta2, eps, wd, momentum, dampening;
  int nesterov, adamw;
  float bc1, bc2, l1, l2, fbeta;
  int ftrl_mode;
  float gscale;
  const int32_t* ncount = nullptr;  // nullable device count: only rows [0, min(nrows, *ncount)) are live
};
void launch_sparse_opt(const SparseOptArgs& a, hipStream_t s);

// ---------------------------------------------------------------- reduce.hip
// dtype codes: 0 = fp32, 1 = bf16
void launch_sumsq_partial(const void* x, int dtype, int64_t n, float* partial, int nblocks, hipStream_t s);
void launch_sumsq_finish(const float* partial, int nblocks, float* out, int accumulate, hipStream_t s);
void launch_clip_factor(const float* sumsq, float max_norm, float* factor, hipStream_t s);
void launch_cast(const void* x, int xdtype, void* y, int ydtype, int64_t n, float scale, hipStream_t s);
void launch_axpy(float a, const void* x, int xdtype, void* y, int ydtype, int64_t n, hipStream_t s);
void launch_reduce_n(const void* x, int xdtype, int k, int64_t n, void* y, int ydtype, float scale, hipStream_t s);
void launch_lerp(const float* w0, const float* w, float sc, void* out, int odtype, int64_t n, hipStream_t s);
int sumsq_blocks(int64_t n);

// ---------------------------------------------------------------- compress.hip
// 1-bit sign compression with per-chunk scale and error feedback (K26).
constexpr int kOnebitChunk = 1024;
// mom (nullable, err's dtype): 1-bit Adam -- compress the worker momentum beta1 m + (1 - beta1) g
void launch_onebit_pack(const void* g, int gdtype, void* err, int edtype, int64_t n, uint64_t* words, float* scales,
                        hipStream_t s, void* mom = nullptr, float beta1 = 0.f);
void launch_onebit_momentum(const void* g, int gdtype, void* mom, int mdtype, int64_t n, float beta1, hipStream_t s);
void launch_onebit_unpack_reduce(const uint64_t* words, const float* scales, int nworkers, int64_t n,
                                 int64_t words_stride, int64_t scales_stride, void* out, int odtype, float mult,
                                 int accumulate, hipStream_t s);

// ---------------------------------------------------------------- sparse.hip
void launch_gather_rows(const void* table, int tdtype, const int64_t* rows, int64_t nrows, int dim, void* out,
                        int odtype, int64_t out_ld, int64_t out_off, int act, hipStream_t s);
void launch_segment_reduce_rows(const void* src, int sdtype, const int64_t* perm, const int64_t* seg_off,
                                int64_t nseg, int dim, void* out, int odtype, int mean, hipStream_t s);
void launch_scatter_add_rows(const void* src, int sdtype, const int64_t* rows, int64_t nrows, int dim, float* table,
                             hipStream_t s);
void launch_embedding_bag_fwd(const float* table, const int64_t* ids, int64_t batch, int fields, int dim,
                              void* out, int odtype, int64_t out_ld, int64_t out_off, int act, hipStream_t s);
void launch_sparse_lr_fwd(const float* w, const int64_t* ids, int64_t batch, int fields, int64_t hash_size,
                          const float* bias, float* out, hipStream_t s);
void launch_lazy_init_rows(float* table, const int64_t* rows, const int64_t* keys, int64_t nrows, int dim,
                           uint8_t* init_flags, uint64_t seed, int64_t row_base, float lo, float hi, hipStream_t s);
void launch_unique_runs(const int64_t* srt, const int64_t* uidx, int64_t n, int64_t mask, int64_t* ukeys,
                        int64_t* seg, hipStream_t s);
void launch_hash_slots(int64_t* hkeys, int64_t capacity, const int64_t* ids, int64_t n, int64_t* out, int insert,
                       int32_t* status, hipStream_t s);

// ---------------------------------------------------------------- fc.hip
// fused FC backward: dW = (act'(y) * dy)^T x (+ db = column sums), dX = (act'(y) * dy) W;
// dtype 0 fp32 / 1 bf16 for every operand; dw / db / dx nullable
void launch_fc_bwd(const void* dy, const void* y, const void* x, const void* w, void* dw, float* db, void* dx,
                   int dtype, int M, int N, int K, int act, float* ws, hipStream_t s);
// fp32 workspace (floats) of the split-reduction dW path, 0 = unsplit
int64_t fc_bwd_ws_floats(int M, int N, int K);
void launch_fc_fwd_f32(const float* x, const float* w, const float* b, float* y, int M, int N, int K, int act,
                       hipStream_t s);

// ---------------------------------------------------------------- ref_ops.hip
void launch_softmax_temp_fwd(const float* x, float* y, int64_t rows, int cols, float inv_temp, float clamp_lo,
                             float clamp_hi, hipStream_t s);
void launch_softmax_temp_bwd(const float* p, const float* dy, float* dx, int64_t rows, int cols, float scale,
                             hipStream_t s);
void launch_softmax_xent(const float* p, const int64_t* labels, int64_t rows, int cols, float* loss,
                         float* grad, hipStream_t s);
void launch_bce(const float* p, const float* y, int64_t n, float* loss, float* grad, hipStream_t s);
void launch_maxpool2d_fwd(const void* x, int dtype, int64_t nc, int h, int w, int k, int stride, int pad,
                          void* y, int32_t* argmax, int oh, int ow, hipStream_t s);
void launch_maxpool2d_bwd(const void* dy, int dtype, const int32_t* argmax, int64_t nc, int h, int w, int oh,
                          int ow, int k, int stride, int pad, void* dx, hipStream_t s);
void launch_im2col(const float* x, int64_t n, int c, int h, int w, int k, int stride, int pad, int oh, int ow,
                   float* col, hipStream_t s);
void launch_col2im(const float* col, int64_t n, int c, int h, int w, int k, int stride, int pad, int oh, int ow,
                   float* x, hipStream_t s);
void launch_dropout_fwd(const void* x, int dtype, void* y, int64_t n, float p_drop, uint64_t seed,
                        uint64_t offset, hipStream_t s);
void launch_dropout_bwd(const void* dy, int dtype, void* dx, int64_t n, float p_drop, uint64_t seed,
                        uint64_t offset, hipStream_t s);
void launch_uniform_init(float* w, int64_t n, uint64_t seed, uint64_t offset, float lo, float hi, hipStream_t s);

// ---------------------------------------------------------------- bn_act.hip
// NHWC BatchNorm (+residual) + activation; x/y/dy/dx/res bf16 [R, C]; params/stats fp32 [C].
struct BnFwdArgs {
  const uint16_t* x;
  const uint16_t* res;  // nullable
  uint16_t* y;
  const float* gamma;   // nullable (affine=False)
  const float* beta;
  float* rmean;         // nullable (no running stats)
  float* rvar;
  float* mean;          // [C] saved for backward
  float* invstd;        // [C]
  float* scale;         // [C] scratch
  float* shift;         // [C] scratch
  float* ws;            // [2, G, C] partials
  int64_t R;
  int C;
  int G;
  int act;
  int training;
  float eps, momentum;
};
void launch_bn_fwd(const BnFwdArgs& a, hipStream_t s);

void launch_maxpool_nhwc_fwd(const uint16_t* x, const float* coef, uint16_t* y, uint8_t* idx, int N, int H, int W,
                             int C, int OH, int OW, int k, int s, int p, hipStream_t st);
void launch_maxpool_nhwc_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int H, int W, int C, int OH,
                             int OW, int k, int s, int p, hipStream_t st);
// stem backward: maxpool 3x3/2/1 scatter fused into the BN(+ReLU) backward of its input z
// (mc = the forward's [scale | shift]); ws: [2 G C + 3 C] fp32, G = pool_bn_bwd_blocks(...);
// dz == nullptr: the statistics pass only (dgamma, dbeta and the coefficients at ws + 2 G C)
int pool_bn_bwd_blocks(int64_t N, int H, int W, int C);
void launch_pool_bn_bwd(const uint16_t* dy, const uint8_t* idx, const uint16_t* z, const float* mc, const float* mean,
                        const float* invstd, const float* gamma, float* ws, int G, float* dgamma, float* dbeta,
                        uint16_t* dz, int N, int H, int W, int C, int OH, int OW, hipStream_t st);

// ---------------------------------------------------------------- stem.hip (ResNet 7x7/2 stem, MFMA)
// x: [N, H, W, cin] bf16, cin 3 or 4 (channel 3 meets zero weights); wp: [64][224] packed
// bf16 (k' = kh*32 + kw*4 + c); z: [N, OH, OW, 64] bf16; OW <= 128.
// kshift/part optional: per-block BN partial sums of z about kshift -> part[2][blocks][64]
void launch_stem_conv_fwd(const uint16_t* x, int cin, const uint16_t* wp, uint16_t* z, int N, int H, int W, int OH,
                          int OW, const float* kshift, float* part, hipStream_t s);
int stem_fwd_blocks(int N);
int stem_wrw_blocks(int N, int OH);
// Tall [G][C] partial pairs: rows S = partials_fold_rows(G) (0: no fold needed) of a first-level
// fixed-order sum into op/oq [S][C]
int partials_fold_rows(int G);
void launch_partials_fold(const float* p, const float* q, int G, int C, float* op, float* oq, hipStream_t s);
// BN finalize from producer-fused partial sums ps/pq: [G][C] of sum(x - k), sum((x - k)^2)
void launch_bn_finalize_sums(const float* ps, const float* pq, const float* kshift, int G, int C, int64_t R,
                             float eps, float momentum, const float* gamma, const float* beta, float* rmean,
                             float* rvar, float* mean, float* invstd, float* scale, float* shift, hipStream_t s);
// ws: (stem_wrw_blocks + 32) * 64 * 224 floats; dwp: [64][224] fp32 packed weight gradient
// pool_dy != nullptr: FUSED -- dz is z (the stem BN's input) and each dz row is computed in the
// kernel from the pooled gradient pool_dy / pool_idx ([N, OH/2, OW/2, 64]), mc ([2 * 64] scale |
// shift) and coef ([3 * 64] bn backward ca | cb | cc; pool.hip launch_pool_bn_bwd with dz null)
void launch_stem_conv_wrw(const uint16_t* x, int cin, const uint16_t* dz, float* ws, float* dwp, int N, int H, int W,
                          int OH, int OW, hipStream_t s, const uint16_t* pool_dy = nullptr,
                          const uint8_t* pool_idx = nullptr, const float* mc = nullptr, const float* coef = nullptr);

// ---------------------------------------------------------------- transformer.hip (row / elementwise)
void launch_rmsnorm_fwd(const uint16_t* x, const uint16_t* r, const void* w, bool w_bf16, uint16_t* s, uint16_t* y,
                        float* rstd, int R, int D, float eps, hipStream_t st);
int rmsnorm_bwd_parts(int R);
void launch_rmsnorm_bwd(const uint16_t* dy, const uint16_t* s, const void* w, bool w_bf16, const float* rstd,
                        const uint16_t* ds_in, uint16_t* dx, float* wpart, float* dw, int R, int D, hipStream_t st);
void launch_layernorm_fwd(const uint16_t* x, const uint16_t* o, const void* gamma, const void* beta, bool w_bf16,
                          uint16_t* s, uint16_t* y, float* mean, float* rstd, int R, int D, float eps, float p,
                          uint64_t seed, hipStream_t st);
int layernorm_bwd_parts(int R);
void launch_layernorm_bwd(const uint16_t* dy, const uint16_t* s, const void* gamma, bool w_bf16, const float* mean,
                          const float* rstd, uint16_t* dx, uint16_t* dout, float* part, float* dgamma, float* dbeta,
                          int R, int D, float p, uint64_t seed, hipStream_t st);
void launch_swiglu_fwd(const uint16_t* gu, uint16_t* h, int64_t R, int F, hipStream_t st);
void launch_swiglu_bwd(const uint16_t* dh, const uint16_t* gu, uint16_t* dgu, int64_t R, int F, hipStream_t st);
void launch_rope_split_fwd(const uint16_t* qkv, const float* cs, uint16_t* q, uint16_t* k, uint16_t* v, int B, int S,
                           int H, int KV, int hd, hipStream_t st);
void launch_rope_split_bwd(const uint16_t* dq, const uint16_t* dk, const uint16_t* dv, const float* cs,
                           uint16_t* dqkv, int B, int S, int H, int KV, int hd, hipStream_t st);

struct BnBwdArgs {
  const uint16_t* dy;
  const uint16_t* y;          // nullable when mask_coef is given (relu, no residual)
  const float* mask_coef;     // nullable: forward [scale | shift], relu mask recomputed from x
  const uint16_t* x;
  const float* gamma;
  const float* mean;
  const float* invstd;
  float* dgamma;  // nullable
  float* dbeta;   // nullable
  uint16_t* dx;
  uint16_t* dres;  // nullable: gradient of the fused residual input (= dz)
  const uint8_t* mbits;  // nullable: ReLU mask bits of the forward output (1 bit / element)
  float* ws;       // [2, G, C] partials + [3, C] coefficients
  int64_t R;
  int C;
  int G;
  int act;
};
void launch_bn_bwd(const BnBwdArgs& a, hipStream_t s);
int bn_red_blocks(int64_t R, int C);

// ---------------------------------------------------------------- dense.hip (MFMA)
// C[M,N] (+)= act(alpha * A[M,K] . B[N,K]^T + bias[N]); A, B bf16 K-contiguous; C bf16 or fp32.
// act: 0 none, 1 relu, 2 leaky relu(0.01), 3 reference clipped sigmoid (0.001 + 0.998*sigmoid)
void launch_gemm_nt_bf16(const uint16_t* a, int64_t lda, const uint16_t* b, int64_t ldb, void* c, int c_f32,
                         int64_t ldc, int M, int N, int K, float alpha, int accumulate, const float* bias, int act,
                         hipStream_t s);
void launch_act_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dz, int64_t n, int act, hipStream_t s);
// DLRM dot interaction: out [B, D + n(n-1)/2] = [x | triu(z z^T)], z = [x; e[b]] (n = T+1 <= 32, D % 32 == 0)
void launch_dlrm_interact_fwd(const uint16_t* x, const uint16_t* e, uint16_t* out, int B, int T, int D,
                              hipStream_t s);
void launch_dlrm_interact_bwd(const uint16_t* x, const uint16_t* e, const uint16_t* dout, uint16_t* dx, uint16_t* de,
                              int B, int T, int D, hipStream_t s);

// ---------------------------------------------------------------- convgemm.hip (MFMA implicit-GEMM convs)
// NHWC conv geometry of the A operand: input map H x W x C, output map OH x OW, square kernel
// ks with stride / pad.  Reduction index k = (kh * ks + kw) * C + c (channels_last weight order).
struct ConvGeo {
  int H, W, OH, OW, C, ks, stride, pad;
  int ksw;             // taps along the width (0: = ks, square kernel)
  int RH, RW, ra, rb;  // RH > 0: output pixel (i, oh, ow) lands at row (i, 2 oh + ra, 2 ow + rb) of an
                       // RH x RW map (one phase of a stride-2 data gradient); 0: rows in order
};
// n / d for 0 <= n < 2^31 as (umulhi(n, mul) + n) >> shift (d fixed per launch): the wide
// weight-gradient kernel decodes pixel indices with it instead of two integer divisions per DMA
// instruction per stage.
struct FastDiv {
  uint32_t mul, shift;
};
inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t sh = 0;
  while (sh < 32 && (uint64_t(1) << sh) < d) ++sh;
  const uint64_t one = 1;
  return FastDiv{static_cast<uint32_t>(((one << 32) * ((one << sh) - d)) / d + 1), sh};
}
struct ConvGemmArgs {
  const uint16_t* a;    // [images, H, W, C] bf16
  const uint16_t* b;    // [N, K] bf16, K = ks * ks * C
  uint16_t* c;          // [M, N] bf16, M = images * OH * OW
  int M, N, K;
  ConvGeo g;
  const float* pro;     // [scale | shift] (2C): A := relu(A * scale + shift) while staging; nullable
  int epi;              // 0 store, 1 + BN partial sums, 2 + residual, 3 ReLU mask + BN-backward sums,
                        // 4 + residual of the (OH+1)/2 x (OW+1)/2 map at even (h, w),
                        // 5 + residual masked by bits (aux * relu'(forward output)),
                        // 6/7/8 = 5/2/4 + the previous block's bn3 backward reduce (aux2, bits2,
                        // mean, invstd): output masked by bits2, sums into part; 9 = 6 + the
                        // previous block's downsample-BN sum (aux3, mean2, invstd2)
  const uint16_t* aux;  // epi 2/4/5: residual rows; epi 3: BN input z [M, N]
  const uint8_t* bits;  // epi 5/6: ReLU mask bits of aux's elements
  const uint16_t* aux2; // epi 6-8: previous block's bn3 input z3 [M, N]
  const uint8_t* bits2; // epi 6-8: ReLU mask bits of the previous block's output (= this input)
  const float* kshift;  // epi 1: shift of the partial sums [N] (nullable = 0)
  const float* mc;      // epi 3: [scale | shift] (2N) of that BN (ReLU mask)
  const float* mean;    // epi 3/6-8: [N]
  const float* invstd;  // epi 3/6-8: [N]
  float* part;          // epi 1/3/6-8: [2][conv_fwd_plan(M, N, K, pro).gm][N] block partial sums
                        // (epi 9: [3][gm][N], the third = the downsample BN's sum(g * xhat))
  const uint16_t* aux3; // epi 9: the previous block's downsample-BN input zd [M, N]
  const float* mean2;   // epi 9: [N] that BN's batch mean / inverse std
  const float* invstd2;
  // BN-backward prologue (1x1, epi 3 only; excludes pro): A := bf16(ca * a + cb * a2 + cc), the
  // previous BN's data gradient from its output gradient a and input a2 (coefficients bwd =
  // [ca | cb | cc], 3C); the A tile is also stored to aout [M, C] (by the channel-tile-0 blocks)
  const uint16_t* a2;   // [M, C] BN input; nullable
  const float* bwd;     // [3C]
  uint16_t* aout;       // [M, C]
  // block-output prologue (1x1 forward, epi 0/1; pro and a2 set, bwd null): A := relu(a * sc + sh
  // + r) with pro = [sc | sh] of bn3 and r = a2 (identity) or a2 * sc2 + sh2 (pro2 = the
  // downsample BN's [sc2 | sh2]); the block output goes to aout, its ReLU bits to abits [M C / 8]
  const float* pro2;    // [2C]; nullable
  uint8_t* abits;
  FastDiv fd_ohw, fd_ow;  // set by launch_conv_fwd (OH * OW, OW)
  int pgm;                // rows per partial slab (0: the launch's gm); several GEMMs share one part
  uint64_t* tbuf = nullptr;  // conv_big only, diagnostics: 8 wall-clock stamps per block (nullable)
};
struct ConvFwdPlan {
  int bm, bn, gm;       // tile pixels / channels, pixel-tile groups (partial-sum rows)
};
ConvFwdPlan conv_fwd_plan(int M, int N, int K, bool pro, int epi = 0);
// conv_big.hip: 256 x 256 tiles, one 512-thread block per CU, for deep-K 1x1 GEMMs (every epilogue);
// conv_fwd_plan_geo / launch_conv_fwd route there when conv_big_ok holds (gm = conv_big_gm(M))
bool conv_big_ok(int M, int N, int K, bool pro, const ConvGeo& g, int src2, int epi);
// the channel tile conv_big runs for this GEMM: 256, 128 (two blocks per CU), 0 = not eligible
int conv_big_tn(int M, int N, int K, bool pro, const ConvGeo& g, int src2, int epi);
int conv_big_gm(int M);
void launch_conv_big(const ConvGemmArgs& a, hipStream_t s);
// the four stride-2 data-gradient phase GEMMs (epi 3, no prologue, LDS-DMA staging, 128-pixel tiles)
// in one launch; phase i's partials go to rows [sum gm(<i), ..) of a part with pgm = sum of gm
void launch_conv_dgrad_phases(const ConvGemmArgs* ph, hipStream_t s);
int conv_dgrad_phase_gm(int M);
// the plan launch_conv_fwd uses for this geometry (the 3x3 patch-staged tiles where they apply)
// src2: the launch's two-source prologue (0 none, 1 block output, 2 BN backward)
ConvFwdPlan conv_fwd_plan_geo(int M, int N, int K, bool pro, const ConvGeo& g, int src2 = 0, int epi = 0);
void launch_conv_fwd(const ConvGemmArgs& a, hipStream_t s);
// Backward layouts of many conv weights in one launch: jobs = device array of
// {src, dst, kind (0 1x1 transpose, 1 3x3 flip-transpose, 2 3x3 stride-2 phases), A, B} (32 B each)
void launch_weight_prep(const void* jobs, int njobs, int max_blocks, hipStream_t s);

// Fused backward of a bottleneck's last 1x1 conv (conv3: CI -> CO channels) with bn3's backward
// in its prologue (conv_bwd_fused.hip): per 128-pixel tile, dz3 = bf16(ca g + cb z3 + cc) is built
// in LDS one 64-channel stage at a time and feeds BOTH GEMMs -- the data gradient
// gy = dz3 W3 (bn2's ReLU mask + backward sums in the epilogue, the conv_gemm epi-3 contract) and
// the weight gradient dW3 += dz3^T relu(bn2(z2)) (per-block fp32 slabs, fixed-order reduce) --
// so dz3 never reaches HBM and z2 is read once for both.
struct Conv11BwdArgs {
  const uint16_t* g;      // [M, CO] gradient at bn3's output (already ReLU-masked)
  const uint16_t* z3;     // [M, CO] bn3 input
  const float* cbwd;      // [3 CO] ca | cb | cc (bn3 backward coefficients)
  const uint16_t* wt;     // [CI, CO] conv3 weight transposed
  const uint16_t* z2;     // [M, CI] bn2 input (conv3's input before bn2 + ReLU)
  const float* cf2;       // [2 CI] bn2 scale | shift; nullptr: PLAIN (downsample: z2 used as is,
                          // gy unmasked, no part) -- the 64 -> 256 kernel only
  const float* mean2;     // [CI]
  const float* invstd2;   // [CI]
  uint16_t* gy;           // [M, CI] masked data gradient (bn2's output gradient)
  float* part;            // [2][gm][CI] bn2 backward partial sums
  float* ws;              // conv11_bwd_ws(M, CI, CO) floats: dW slabs (+ reduce scratch)
  uint16_t* dw;           // [CO, CI] bf16 conv3 weight gradient
  int M;
};
bool conv11_bwd_fused_ok(int CI, int CO);
bool conv11_bwd_plain_ok(int CI, int CO);
bool conv11_bwd_built(int CI, int CO);  // launchable (conv11_bwd_fused_ok: also chosen by default)
int conv11_bwd_blocks(int M, int CI, int CO);
int64_t conv11_bwd_ws(int M, int CI, int CO);
void launch_conv11_bwd_fused(const Conv11BwdArgs& a, int CI, int CO, hipStream_t s);

struct ConvWgradArgs {
  const uint16_t* dz;   // [M, N] output gradient rows
  const uint16_t* x;    // [images, H, W, C] input map
  int M, N, K;          // K = ks * ks * C
  ConvGeo g;
  const float* pro;     // [scale | shift] (2C) applied to x while staging; nullable
  float* ws;            // conv_wgrad_ws(M, N, K, C) floats
  uint16_t* dw;         // [N, K] bf16
  float* db;            // nullable: [N] fp32 column sums of dz (a Linear's bias gradient; wide plan only)
  float* dbws;          // [conv_wgrad_splits(...)][N] fp32 scratch when db is set
  FastDiv fd_ohw, fd_ow;  // set by launch_conv_wgrad (OH * OW, OW)
};
int conv_wgrad_splits(int M, int N, int K, int C, bool pro);
// workspace of launch_conv_wgrad for this geometry (the 3x3 patch kernel's plan where it applies)
int64_t conv_wgrad_ws_geo(int M, int N, int K, const ConvGeo& g, bool pro);
bool conv_wgrad_is_wide(int M, int N, int K, int C, bool pro);
int64_t conv_wgrad_ws(int M, int N, int K, int C, bool pro);
// Fused short-sequence attention (attention.hip): qkv [B, S, 3, H, 64] bf16 (Linear layout),
// out [B, S, H * 64], lse [B, H, S] fp32; S % 32 == 0, S <= 128; dropout p on the probabilities
void launch_attn_fwd(const uint16_t* qkv, uint16_t* out, float* lse, int B, int S, int H, float scale, float p,
                     uint64_t seed, hipStream_t s);
void launch_attn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse, uint16_t* dqkv,
                     int B, int S, int H, float scale, float p, uint64_t seed, hipStream_t s);
void launch_attn_dropout_mask(uint8_t* mask, int64_t n, float p, uint64_t seed, hipStream_t s);
// Causal GQA flash attention (flash_attn.hip): q [B, H, S, 128], k / v [B, KV, S, 128] bf16,
// out [B, S, H * 128], lse / dsum [B, H, S] fp32; S % 128 == 0
// Fused softmax cross-entropy over bf16 logits [R, V] (xent.hip): forward lse / per-row loss,
// backward dx = (softmax - onehot) * go / count (go, count: device scalars); ignored rows -> 0
void launch_xent_fwd(const uint16_t* x, const int64_t* lab, int64_t R, int V, int64_t ignore, float* lse, float* loss,
                     hipStream_t s);
void launch_xent_bwd(const uint16_t* x, const int64_t* lab, const float* lse, int64_t R, int V, int64_t ignore,
                     const float* go, const float* count, uint16_t* dx, hipStream_t s);
void launch_fa_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* out, float* lse, int B, int S,
                   int H, int KV, float scale, hipStream_t s);
void launch_fa_bwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, const uint16_t* out, const uint16_t* dout,
                   const float* lse, float* dsum, uint16_t* dq, uint16_t* dk, uint16_t* dv, int B, int S, int H,
                   int KV, float scale, hipStream_t s);
void launch_conv_wgrad(const ConvWgradArgs& a, hipStream_t s);
// BN helpers for the fused bottleneck (bn_act.hip): y = act(x*scale + shift [+ res [* rscale + rshift]])
// mbits (nullable): also write the ReLU mask of y, 1 bit per element
void launch_bn_apply_coef(const uint16_t* x, const uint16_t* res, const float* coef, const float* rcoef, uint16_t* y,
                          uint8_t* mbits, int64_t R, int C, int act, hipStream_t s);
// BN backward from producer partial sums pd/px [G][C] (g = already-masked output gradient)
void launch_bn_bwd_partials(const float* pd, const float* px, int G, const uint16_t* g, const uint16_t* x,
                            const float* gamma, const float* mean, const float* invstd, float* dgamma, float* dbeta,
                            float* coef, uint16_t* dx, int64_t R, int C, hipStream_t s);

}  // namespace psamd
