// Torch bindings for the ps_amd HIP kernels (module ps_amd._C).
//
// Every op validates device / dtype / contiguity / sizes on the host BEFORE launching, so a
// shape mismatch is a Python exception, never an out-of-bounds access on the GPU.  Launches
// go to the caller's current HIP stream (c10::hip::getCurrentHIPStream), so the ops compose
// with torch streams, events and HIP-graph capture.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "psamd_launch.h"

#include <atomic>
#include <map>
#include <mutex>
#include <string>

namespace {

// Dispatch log of the convolution routes (``route_log``): which kernel family / tile / prologue /
// epilogue each conv call ran on -- tests assert that a whole-network run exercised the
// production routes.  One relaxed load per call while disabled.
std::atomic<bool> g_route_on{false};
std::mutex g_route_mu;
std::map<std::string, int64_t>& routes() {
  static std::map<std::string, int64_t> r;
  return r;
}
void route(const std::string& name) {
  if (!g_route_on.load(std::memory_order_relaxed)) return;
  std::lock_guard<std::mutex> g(g_route_mu);
  routes()[name] += 1;
}
// -> the counts so far; then enables / disables logging and optionally clears the counts
std::map<std::string, int64_t> route_log(bool enable, bool reset) {
  std::lock_guard<std::mutex> g(g_route_mu);
  auto out = routes();
  if (reset) routes().clear();
  g_route_on.store(enable, std::memory_order_relaxed);
  return out;
}

using torch::Tensor;

hipStream_t cur_stream(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

int dcode(const Tensor& t, const char* name) {
  if (t.scalar_type() == torch::kFloat32) return 0;
  if (t.scalar_type() == torch::kBFloat16) return 1;
  TORCH_CHECK(false, name, ": dtype must be float32 or bfloat16, got ", t.scalar_type());
  return -1;
}

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void check_f32(const Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32");
}

void check_i64(const Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kInt64, name, " must be int64");
}

template <typename T>
T* opt_ptr(const c10::optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? static_cast<T*>(t->data_ptr()) : nullptr;
}

// ------------------------------------------------------------------------------ optimizers
void fused_opt(int64_t kind, Tensor w, c10::optional<Tensor> st0, c10::optional<Tensor> st1, Tensor g,
               c10::optional<Tensor> wout, double lr, double beta1, double beta2, double eps, double wd,
               double momentum, double dampening, bool nesterov, bool adamw, double bc1, double bc2, double l1,
               double l2, double fbeta, int64_t ftrl_mode, double gscale, c10::optional<Tensor> gscale_t) {
  check_f32(w, "w");
  check_gpu(g, "g");
  const int64_t n = w.numel();
  TORCH_CHECK(g.numel() == n, "grad numel ", g.numel(), " != weight numel ", n);
  if (st0.has_value() && st0->defined()) { check_f32(*st0, "st0"); TORCH_CHECK(st0->numel() == n, "st0 size"); }
  if (st1.has_value() && st1->defined()) { check_f32(*st1, "st1"); TORCH_CHECK(st1->numel() == n, "st1 size"); }
  if ((kind == 1 || kind == 3)) {
    TORCH_CHECK(st0.has_value() && st0->defined() && st1.has_value() && st1->defined(), "adam/ftrl need 2 states");
  }
  if (kind == 2) TORCH_CHECK(st0.has_value() && st0->defined(), "adagrad needs a state");
  if (kind == 0 && momentum != 0.0) TORCH_CHECK(st0.has_value() && st0->defined(), "momentum sgd needs a buffer");
  int wout_bf16 = 0;
  if (wout.has_value() && wout->defined()) {
    check_gpu(*wout, "wout");
    TORCH_CHECK(wout->numel() == n, "wout size");
    wout_bf16 = dcode(*wout, "wout");
  }
  if (gscale_t.has_value() && gscale_t->defined()) check_f32(*gscale_t, "gscale_t");
  const c10::DeviceGuard guard(w.device());
  psamd::FusedOptArgs a;
  a.kind = static_cast<int>(kind);
  a.w = w.data_ptr<float>();
  a.st0 = opt_ptr<float>(st0);
  a.st1 = opt_ptr<float>(st1);
  a.g = g.data_ptr();
  a.g_bf16 = dcode(g, "g");
  a.wout = opt_ptr<void>(wout);
  a.wout_bf16 = wout_bf16;
  a.n = n;
  a.lr = lr; a.beta1 = beta1; a.beta2 = beta2; a.eps = eps; a.wd = wd; a.momentum = momentum;
  a.dampening = dampening; a.nesterov = nesterov; a.adamw = adamw; a.bc1 = bc1; a.bc2 = bc2;
  a.l1 = l1; a.l2 = l2; a.fbeta = fbeta; a.ftrl_mode = static_cast<int>(ftrl_mode);
  a.gscale = gscale;
  a.gscale_ptr = opt_ptr<const float>(gscale_t);
  psamd::launch_fused_opt(a, cur_stream(w));
}

void sparse_opt(int64_t kind, Tensor table, c10::optional<Tensor> st0, c10::optional<Tensor> st1, Tensor rows,
                Tensor grad, bool rowwise, bool skip_zero, double lr, double beta1, double beta2, double eps,
                double wd, double momentum, double dampening, bool nesterov, bool adamw, double bc1, double bc2,
                double l1, double l2, double fbeta, int64_t ftrl_mode, double gscale, c10::optional<Tensor> perm,
                c10::optional<Tensor> ncount) {
  check_f32(table, "table");
  TORCH_CHECK(table.dim() == 2, "table must be [rows, dim]");
  check_i64(rows, "rows");
  check_gpu(grad, "grad");
  const int64_t dim = table.size(1);
  TORCH_CHECK(grad.numel() == rows.numel() * dim, "grad must be [nrows, dim]");
  if (perm.has_value() && perm->defined()) {
    check_i64(*perm, "perm");
    TORCH_CHECK(perm->numel() == rows.numel(), "perm must have one entry per row entry");
  }
  if (st0.has_value() && st0->defined()) {
    check_f32(*st0, "st0");
    const int64_t want = (kind == 2 && rowwise) ? table.size(0) : table.numel();
    TORCH_CHECK(st0->numel() == want, "st0 size (rowwise adagrad state is [rows])");
  }
  if (st1.has_value() && st1->defined()) { check_f32(*st1, "st1"); TORCH_CHECK(st1->numel() == table.numel(), "st1"); }
  if (kind == 1 || kind == 3) TORCH_CHECK(st0.has_value() && st1.has_value(), "adam/ftrl need 2 states");
  if (kind == 2) TORCH_CHECK(st0.has_value(), "adagrad needs a state");
  const c10::DeviceGuard guard(table.device());
  psamd::SparseOptArgs a;
  a.kind = static_cast<int>(kind);
  a.table = table.data_ptr<float>();
  a.st0 = opt_ptr<float>(st0);
  a.st1 = opt_ptr<float>(st1);
  a.rows = rows.data_ptr<int64_t>();
  a.perm = opt_ptr<const int64_t>(perm);
  a.grad = grad.data_ptr();
  a.g_bf16 = dcode(grad, "grad");
  a.nrows = rows.numel();
  a.dim = static_cast<int>(dim);
  a.rowwise = rowwise;
  a.skip_zero = skip_zero;
  a.lr = lr; a.beta1 = beta1; a.beta2 = beta2; a.eps = eps; a.wd = wd; a.momentum = momentum;
  a.dampening = dampening; a.nesterov = nesterov; a.adamw = adamw;
  a.bc1 = bc1; a.bc2 = bc2; a.l1 = l1; a.l2 = l2; a.fbeta = fbeta; a.ftrl_mode = static_cast<int>(ftrl_mode);
  a.gscale = gscale;
  if (ncount.has_value() && ncount->defined()) {  // device count of the live rows (a touched list)
    check_gpu(*ncount, "ncount");
    TORCH_CHECK(ncount->scalar_type() == torch::kInt32 && ncount->numel() == 1, "ncount: int32 [1]");
    a.ncount = ncount->data_ptr<int32_t>();
  }
  psamd::launch_sparse_opt(a, cur_stream(table));
}

// ------------------------------------------------------------------------------ reductions
void sumsq(Tensor x, Tensor out, bool accumulate) {
  check_gpu(x, "x");
  check_f32(out, "out");
  TORCH_CHECK(out.numel() >= 1, "out must hold one float");
  const c10::DeviceGuard guard(x.device());
  const int nb = psamd::sumsq_blocks(x.numel());
  auto partial = torch::empty({nb}, out.options());
  auto s = cur_stream(x);
  psamd::launch_sumsq_partial(x.data_ptr(), dcode(x, "x"), x.numel(), partial.data_ptr<float>(), nb, s);
  psamd::launch_sumsq_finish(partial.data_ptr<float>(), nb, out.data_ptr<float>(), accumulate, s);
}

void clip_factor(Tensor sq, double max_norm, Tensor factor) {
  check_f32(sq, "sumsq");
  check_f32(factor, "factor");
  const c10::DeviceGuard guard(sq.device());
  psamd::launch_clip_factor(sq.data_ptr<float>(), static_cast<float>(max_norm), factor.data_ptr<float>(),
                            cur_stream(sq));
}

void cast_(Tensor x, Tensor y, double scale) {
  check_gpu(x, "x");
  check_gpu(y, "y");
  TORCH_CHECK(x.numel() == y.numel(), "cast size mismatch");
  const c10::DeviceGuard guard(x.device());
  psamd::launch_cast(x.data_ptr(), dcode(x, "x"), y.data_ptr(), dcode(y, "y"), x.numel(), static_cast<float>(scale),
                     cur_stream(x));
}

void axpy_(double a, Tensor x, Tensor y) {
  check_gpu(x, "x");
  check_gpu(y, "y");
  TORCH_CHECK(x.numel() == y.numel(), "axpy size mismatch");
  const c10::DeviceGuard guard(x.device());
  psamd::launch_axpy(static_cast<float>(a), x.data_ptr(), dcode(x, "x"), y.data_ptr(), dcode(y, "y"), x.numel(),
                     cur_stream(x));
}

void reduce_n(Tensor x, Tensor y, double scale) {
  check_gpu(x, "x");
  check_gpu(y, "y");
  TORCH_CHECK(x.dim() == 2, "x must be [k, n]");
  TORCH_CHECK(x.size(1) == y.numel(), "reduce_n size mismatch");
  const c10::DeviceGuard guard(x.device());
  psamd::launch_reduce_n(x.data_ptr(), dcode(x, "x"), static_cast<int>(x.size(0)), x.size(1), y.data_ptr(),
                         dcode(y, "y"), static_cast<float>(scale), cur_stream(x));
}

void lerp(Tensor w0, Tensor w, double sc, Tensor out) {
  check_f32(w0, "w0");
  check_f32(w, "w");
  check_gpu(out, "out");
  TORCH_CHECK(w0.numel() == w.numel() && w.numel() == out.numel(), "lerp size mismatch");
  const c10::DeviceGuard guard(w.device());
  psamd::launch_lerp(w0.data_ptr<float>(), w.data_ptr<float>(), static_cast<float>(sc), out.data_ptr(),
                     dcode(out, "out"), w.numel(), cur_stream(w));
}

// ------------------------------------------------------------------------------ compression
void onebit_pack(Tensor g, Tensor err, Tensor words, Tensor scales, c10::optional<Tensor> mom, double beta1) {
  check_gpu(g, "g");
  check_gpu(err, "err");  // error feedback in fp32 or bf16
  check_gpu(words, "words");
  check_f32(scales, "scales");
  TORCH_CHECK(words.scalar_type() == torch::kInt64, "words must be int64 (bit-packed)");
  const int64_t n = g.numel();
  TORCH_CHECK(err.numel() == n, "err size");
  TORCH_CHECK(words.numel() >= (n + 63) / 64, "words too small");
  TORCH_CHECK(scales.numel() >= (n + psamd::kOnebitChunk - 1) / psamd::kOnebitChunk, "scales too small");
  const c10::DeviceGuard guard(g.device());
  TORCH_CHECK(err.is_contiguous(), "err must be contiguous");
  void* mp = nullptr;
  if (mom.has_value() && mom->defined()) {  // 1-bit Adam: the worker momentum, err's dtype
    check_gpu(*mom, "mom");
    TORCH_CHECK(mom->numel() == n && mom->is_contiguous() && mom->scalar_type() == err.scalar_type(),
                "mom: contiguous, err's size and dtype");
    mp = mom->data_ptr();
  }
  psamd::launch_onebit_pack(g.data_ptr(), dcode(g, "g"), err.data_ptr(), dcode(err, "err"), n,
                            reinterpret_cast<uint64_t*>(words.data_ptr<int64_t>()), scales.data_ptr<float>(),
                            cur_stream(g), mp, static_cast<float>(beta1));
}

void onebit_momentum(Tensor g, Tensor mom, double beta1) {
  check_gpu(g, "g");
  check_gpu(mom, "mom");
  TORCH_CHECK(g.is_contiguous() && mom.is_contiguous() && g.numel() == mom.numel(), "g, mom: contiguous, same size");
  const c10::DeviceGuard guard(g.device());
  psamd::launch_onebit_momentum(g.data_ptr(), dcode(g, "g"), mom.data_ptr(), dcode(mom, "mom"), g.numel(),
                                static_cast<float>(beta1), cur_stream(g));
}

void onebit_unpack_reduce(Tensor words, Tensor scales, Tensor out, double mult, bool accumulate) {
  check_gpu(words, "words");
  check_f32(scales, "scales");
  check_gpu(out, "out");
  TORCH_CHECK(words.dim() == 2 && scales.dim() == 2 && words.size(0) == scales.size(0), "words/scales [W, *]");
  const int64_t n = out.numel();
  TORCH_CHECK(words.size(1) >= (n + 63) / 64, "words too small");
  TORCH_CHECK(scales.size(1) >= (n + psamd::kOnebitChunk - 1) / psamd::kOnebitChunk, "scales too small");
  const c10::DeviceGuard guard(out.device());
  psamd::launch_onebit_unpack_reduce(reinterpret_cast<const uint64_t*>(words.data_ptr<int64_t>()),
                                     scales.data_ptr<float>(), static_cast<int>(words.size(0)), n, words.size(1),
                                     scales.size(1), out.data_ptr(), dcode(out, "out"), static_cast<float>(mult),
                                     accumulate, cur_stream(out));
}

// ------------------------------------------------------------------------------ sparse
void gather_rows(Tensor table, Tensor rows, Tensor out, int64_t out_off, int64_t act) {
  check_gpu(table, "table");
  check_i64(rows, "rows");
  check_gpu(out, "out");
  TORCH_CHECK(table.dim() == 2 && out.dim() == 2, "table/out must be 2-D");
  const int64_t dim = table.size(1);
  TORCH_CHECK(out.size(0) == rows.numel(), "out rows != len(rows)");
  TORCH_CHECK(out_off >= 0 && out_off + dim <= out.size(1), "out column slice out of range");
  const c10::DeviceGuard guard(table.device());
  psamd::launch_gather_rows(table.data_ptr(), dcode(table, "table"), rows.data_ptr<int64_t>(), rows.numel(),
                            static_cast<int>(dim), out.data_ptr(), dcode(out, "out"), out.size(1), out_off,
                            static_cast<int>(act), cur_stream(table));
}

void segment_reduce_rows(Tensor src, Tensor perm, Tensor seg_off, Tensor out, bool mean) {
  check_gpu(src, "src");
  check_i64(perm, "perm");
  check_i64(seg_off, "seg_off");
  check_gpu(out, "out");
  TORCH_CHECK(src.dim() == 2 && out.dim() == 2 && src.size(1) == out.size(1), "src/out [*, dim]");
  TORCH_CHECK(seg_off.numel() == out.size(0) + 1, "seg_off must have nseg+1 entries");
  TORCH_CHECK(perm.numel() == src.size(0), "perm must index every src row");
  const c10::DeviceGuard guard(src.device());
  psamd::launch_segment_reduce_rows(src.data_ptr(), dcode(src, "src"), perm.data_ptr<int64_t>(),
                                    seg_off.data_ptr<int64_t>(), out.size(0), static_cast<int>(src.size(1)),
                                    out.data_ptr(), dcode(out, "out"), mean, cur_stream(src));
}

void scatter_add_rows(Tensor src, Tensor rows, Tensor table) {
  check_gpu(src, "src");
  check_i64(rows, "rows");
  check_f32(table, "table");
  TORCH_CHECK(table.dim() == 2 && src.dim() == 2 && src.size(1) == table.size(1), "shape");
  TORCH_CHECK(src.size(0) == rows.numel(), "src rows != len(rows)");
  const c10::DeviceGuard guard(src.device());
  psamd::launch_scatter_add_rows(src.data_ptr(), dcode(src, "src"), rows.data_ptr<int64_t>(), rows.numel(),
                                 static_cast<int>(src.size(1)), table.data_ptr<float>(), cur_stream(src));
}

void embedding_bag_fwd(Tensor table, Tensor ids, Tensor out, int64_t out_off, int64_t act) {
  check_f32(table, "table");
  check_i64(ids, "ids");
  check_gpu(out, "out");
  TORCH_CHECK(ids.dim() == 2 && out.dim() == 2 && table.dim() == 2, "ids [B,F], out [B,*], table [R,D]");
  const int64_t fields = ids.size(1), dim = table.size(1);
  TORCH_CHECK(out.size(0) == ids.size(0), "batch mismatch");
  TORCH_CHECK(out_off >= 0 && out_off + fields * dim <= out.size(1), "out column slice out of range");
  const c10::DeviceGuard guard(table.device());
  psamd::launch_embedding_bag_fwd(table.data_ptr<float>(), ids.data_ptr<int64_t>(), ids.size(0),
                                  static_cast<int>(fields), static_cast<int>(dim), out.data_ptr(), dcode(out, "out"),
                                  out.size(1), out_off, static_cast<int>(act), cur_stream(table));
}

void sparse_lr_fwd(Tensor w, Tensor ids, c10::optional<Tensor> bias, Tensor out) {
  check_f32(w, "w");
  check_i64(ids, "ids");
  check_f32(out, "out");
  TORCH_CHECK(ids.dim() == 2 && out.numel() == ids.size(0), "ids [B,F], out [B]");
  if (bias.has_value() && bias->defined()) check_f32(*bias, "bias");
  const c10::DeviceGuard guard(w.device());
  psamd::launch_sparse_lr_fwd(w.data_ptr<float>(), ids.data_ptr<int64_t>(), ids.size(0),
                              static_cast<int>(ids.size(1)), w.numel(), opt_ptr<const float>(bias),
                              out.data_ptr<float>(), cur_stream(w));
}

void lazy_init_rows(Tensor table, Tensor rows, Tensor flags, int64_t seed, int64_t row_base, double lo, double hi,
                    c10::optional<Tensor> keys) {
  check_f32(table, "table");
  check_i64(rows, "rows");
  check_gpu(flags, "flags");
  TORCH_CHECK(flags.scalar_type() == torch::kUInt8 && flags.numel() == table.size(0), "flags uint8 [rows]");
  if (keys.has_value() && keys->defined()) {
    check_i64(*keys, "keys");
    TORCH_CHECK(keys->numel() == rows.numel(), "keys must have one entry per row");
  }
  const c10::DeviceGuard guard(table.device());
  psamd::launch_lazy_init_rows(table.data_ptr<float>(), rows.data_ptr<int64_t>(), opt_ptr<const int64_t>(keys),
                               rows.numel(), static_cast<int>(table.size(1)), flags.data_ptr<uint8_t>(),
                               static_cast<uint64_t>(seed), row_base, static_cast<float>(lo), static_cast<float>(hi),
                               cur_stream(table));
}

// (ukeys [n], seg [n + 1]) from sorted keys and their unique indices (see sparse.hip)
void unique_runs(Tensor srt, Tensor uidx, int64_t mask, Tensor ukeys, Tensor seg) {
  check_i64(srt, "srt");
  check_i64(uidx, "uidx");
  check_i64(ukeys, "ukeys");
  check_i64(seg, "seg");
  const int64_t n = srt.numel();
  TORCH_CHECK(uidx.numel() == n && ukeys.numel() >= n && seg.numel() >= n + 1, "unique_runs sizes");
  const c10::DeviceGuard guard(srt.device());
  psamd::launch_unique_runs(srt.data_ptr<int64_t>(), uidx.data_ptr<int64_t>(), n, mask, ukeys.data_ptr<int64_t>(),
                            seg.data_ptr<int64_t>(), cur_stream(srt));
}

// out[i] = slot of ids[i] in the device hash map ``hkeys`` (int64 [capacity], power of two,
// -1 = empty); insert claims a slot for a new id.  status (int32 [1]) is set on a miss/overflow.
void hash_slots(Tensor hkeys, Tensor ids, Tensor out, bool insert, Tensor status) {
  check_i64(hkeys, "hkeys");
  check_i64(ids, "ids");
  check_i64(out, "out");
  check_gpu(status, "status");
  TORCH_CHECK(status.scalar_type() == torch::kInt32 && status.numel() >= 1, "status int32 [1]");
  const int64_t cap = hkeys.numel();
  TORCH_CHECK(cap > 0 && (cap & (cap - 1)) == 0, "hash capacity must be a power of two");
  TORCH_CHECK(out.numel() == ids.numel(), "out must match ids");
  const c10::DeviceGuard guard(ids.device());
  psamd::launch_hash_slots(hkeys.data_ptr<int64_t>(), cap, ids.data_ptr<int64_t>(), ids.numel(),
                           out.data_ptr<int64_t>(), insert, status.data_ptr<int32_t>(), cur_stream(ids));
}

// ------------------------------------------------------------------------------ fused FC layer
// dy, y [M, N]; x [M, K]; w [N, K]; all fp32 or all bf16, contiguous; outputs optional
void fc_bwd(Tensor dy, Tensor y, Tensor x, Tensor w, c10::optional<Tensor> dw, c10::optional<Tensor> db,
            c10::optional<Tensor> dx, int64_t act) {
  for (auto* t : {&dy, &y, &x, &w}) check_gpu(*t, "fc_bwd operand");
  const int code = dcode(dy, "dy");
  TORCH_CHECK(dcode(y, "y") == code && dcode(x, "x") == code && dcode(w, "w") == code, "fc_bwd: one dtype");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && w.dim() == 2 && y.sizes() == dy.sizes(), "fc_bwd: 2-D operands");
  const int64_t M = dy.size(0), N = dy.size(1), K = x.size(1);
  TORCH_CHECK(x.size(0) == M && w.size(0) == N && w.size(1) == K, "fc_bwd: shape mismatch");
  void* pdw = nullptr;
  void* pdx = nullptr;
  float* pdb = nullptr;
  if (dw.has_value() && dw->defined()) {
    check_gpu(*dw, "dw");
    TORCH_CHECK(dcode(*dw, "dw") == code && dw->numel() == N * K, "dw [N, K]");
    pdw = dw->data_ptr();
  }
  if (db.has_value() && db->defined()) {
    check_f32(*db, "db");
    TORCH_CHECK(db->numel() == N && pdw != nullptr, "db [N] (computed with dW)");
    pdb = db->data_ptr<float>();
  }
  if (dx.has_value() && dx->defined()) {
    check_gpu(*dx, "dx");
    TORCH_CHECK(dcode(*dx, "dx") == code && dx->numel() == M * K, "dx [M, K]");
    pdx = dx->data_ptr();
  }
  const c10::DeviceGuard guard(dy.device());
  const int64_t nws = pdw != nullptr ? psamd::fc_bwd_ws_floats(static_cast<int>(M), static_cast<int>(N),
                                                               static_cast<int>(K))
                                     : 0;
  Tensor ws;  // split-reduction dW slabs (stream-ordered caching allocator: freed after the launch)
  if (nws > 0) ws = torch::empty({nws}, dy.options().dtype(torch::kFloat32));
  psamd::launch_fc_bwd(dy.data_ptr(), y.data_ptr(), x.data_ptr(), w.data_ptr(), pdw, pdb, pdx, code,
                       static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), static_cast<int>(act),
                       nws > 0 ? ws.data_ptr<float>() : nullptr, cur_stream(dy));
}

void fc_fwd_f32(Tensor x, Tensor w, c10::optional<Tensor> b, Tensor y, int64_t act) {
  check_f32(x, "x");
  check_f32(w, "w");
  check_f32(y, "y");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "x [M, K], w [N, K]");
  TORCH_CHECK(y.size(0) == x.size(0) && y.size(1) == w.size(0), "y [M, N]");
  if (b.has_value() && b->defined()) {
    check_f32(*b, "b");
    TORCH_CHECK(b->numel() == w.size(0), "b [N]");
  }
  const c10::DeviceGuard guard(x.device());
  psamd::launch_fc_fwd_f32(x.data_ptr<float>(), w.data_ptr<float>(), opt_ptr<const float>(b), y.data_ptr<float>(),
                           static_cast<int>(x.size(0)), static_cast<int>(w.size(0)), static_cast<int>(x.size(1)),
                           static_cast<int>(act), cur_stream(x));
}

// ------------------------------------------------------------------------------ reference ops
void softmax_temp_bwd(Tensor p, Tensor dy, Tensor dx, double scale) {
  check_f32(p, "p");
  check_f32(dy, "dy");
  check_f32(dx, "dx");
  TORCH_CHECK(p.dim() == 2 && p.sizes() == dy.sizes() && p.sizes() == dx.sizes(), "p, dy, dx [rows, cols]");
  const c10::DeviceGuard guard(p.device());
  psamd::launch_softmax_temp_bwd(p.data_ptr<float>(), dy.data_ptr<float>(), dx.data_ptr<float>(), p.size(0),
                                 static_cast<int>(p.size(1)), static_cast<float>(scale), cur_stream(p));
}

void softmax_temp_fwd(Tensor x, Tensor y, double temp, double clamp_lo, double clamp_hi) {
  check_f32(x, "x");
  check_f32(y, "y");
  TORCH_CHECK(x.dim() == 2 && x.sizes() == y.sizes(), "x,y [rows, cols]");
  const c10::DeviceGuard guard(x.device());
  psamd::launch_softmax_temp_fwd(x.data_ptr<float>(), y.data_ptr<float>(), x.size(0), static_cast<int>(x.size(1)),
                                 static_cast<float>(1.0 / temp), static_cast<float>(clamp_lo),
                                 static_cast<float>(clamp_hi), cur_stream(x));
}

void softmax_xent(Tensor p, Tensor labels, Tensor loss, c10::optional<Tensor> grad) {
  check_f32(p, "p");
  check_i64(labels, "labels");
  check_f32(loss, "loss");
  TORCH_CHECK(p.dim() == 2 && labels.numel() == p.size(0), "p [B,C], labels [B]");
  if (grad.has_value() && grad->defined()) { check_f32(*grad, "grad"); TORCH_CHECK(grad->sizes() == p.sizes(), "grad"); }
  const c10::DeviceGuard guard(p.device());
  psamd::launch_softmax_xent(p.data_ptr<float>(), labels.data_ptr<int64_t>(), p.size(0), static_cast<int>(p.size(1)),
                             loss.data_ptr<float>(), opt_ptr<float>(grad), cur_stream(p));
}

void bce(Tensor p, Tensor y, Tensor loss, c10::optional<Tensor> grad) {
  check_f32(p, "p");
  check_f32(y, "y");
  check_f32(loss, "loss");
  TORCH_CHECK(p.numel() == y.numel(), "p/y size");
  if (grad.has_value() && grad->defined()) { check_f32(*grad, "grad"); TORCH_CHECK(grad->numel() == p.numel(), "grad"); }
  const c10::DeviceGuard guard(p.device());
  psamd::launch_bce(p.data_ptr<float>(), y.data_ptr<float>(), p.numel(), loss.data_ptr<float>(), opt_ptr<float>(grad),
                    cur_stream(p));
}

void maxpool2d_fwd(Tensor x, int64_t k, int64_t stride, int64_t pad, Tensor y, Tensor argmax) {
  check_gpu(x, "x");
  check_gpu(y, "y");
  check_gpu(argmax, "argmax");
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4, "NCHW");
  TORCH_CHECK(argmax.scalar_type() == torch::kInt32 && argmax.sizes() == y.sizes(), "argmax int32 like y");
  TORCH_CHECK(x.scalar_type() == y.scalar_type(), "x/y dtype");
  const int64_t h = x.size(2), w = x.size(3), oh = y.size(2), ow = y.size(3);
  TORCH_CHECK(oh == (h + 2 * pad - k) / stride + 1 && ow == (w + 2 * pad - k) / stride + 1, "pool output shape");
  const c10::DeviceGuard guard(x.device());
  psamd::launch_maxpool2d_fwd(x.data_ptr(), dcode(x, "x"), x.size(0) * x.size(1), static_cast<int>(h),
                              static_cast<int>(w), static_cast<int>(k), static_cast<int>(stride),
                              static_cast<int>(pad), y.data_ptr(), argmax.data_ptr<int32_t>(), static_cast<int>(oh),
                              static_cast<int>(ow), cur_stream(x));
}

void maxpool2d_bwd(Tensor dy, Tensor argmax, int64_t k, int64_t stride, int64_t pad, Tensor dx) {
  check_gpu(dy, "dy");
  check_gpu(dx, "dx");
  TORCH_CHECK(argmax.scalar_type() == torch::kInt32 && argmax.sizes() == dy.sizes(), "argmax");
  TORCH_CHECK(dy.scalar_type() == dx.scalar_type(), "dtype");
  TORCH_CHECK(dx.dim() == 4 && dy.dim() == 4 && dx.size(0) == dy.size(0) && dx.size(1) == dy.size(1), "NCHW");
  const c10::DeviceGuard guard(dy.device());
  psamd::launch_maxpool2d_bwd(dy.data_ptr(), dcode(dy, "dy"), argmax.data_ptr<int32_t>(), dx.size(0) * dx.size(1),
                              static_cast<int>(dx.size(2)), static_cast<int>(dx.size(3)), static_cast<int>(dy.size(2)),
                              static_cast<int>(dy.size(3)), static_cast<int>(k), static_cast<int>(stride),
                              static_cast<int>(pad), dx.data_ptr(), cur_stream(dy));
}

void im2col(Tensor x, int64_t k, int64_t stride, int64_t pad, Tensor col) {
  check_f32(x, "x");
  check_f32(col, "col");
  TORCH_CHECK(x.dim() == 4, "x NCHW");
  const int64_t n = x.size(0), c = x.size(1), h = x.size(2), w = x.size(3);
  const int64_t oh = (h + 2 * pad - k) / stride + 1, ow = (w + 2 * pad - k) / stride + 1;
  TORCH_CHECK(col.numel() == n * oh * ow * c * k * k, "col must be [n*oh*ow, c*k*k]");
  const c10::DeviceGuard guard(x.device());
  psamd::launch_im2col(x.data_ptr<float>(), n, static_cast<int>(c), static_cast<int>(h), static_cast<int>(w),
                       static_cast<int>(k), static_cast<int>(stride), static_cast<int>(pad), static_cast<int>(oh),
                       static_cast<int>(ow), col.data_ptr<float>(), cur_stream(x));
}

void col2im(Tensor col, int64_t k, int64_t stride, int64_t pad, Tensor x) {
  check_f32(x, "x");
  check_f32(col, "col");
  TORCH_CHECK(x.dim() == 4, "x NCHW");
  const int64_t n = x.size(0), c = x.size(1), h = x.size(2), w = x.size(3);
  const int64_t oh = (h + 2 * pad - k) / stride + 1, ow = (w + 2 * pad - k) / stride + 1;
  TORCH_CHECK(col.numel() == n * oh * ow * c * k * k, "col must be [n*oh*ow, c*k*k]");
  const c10::DeviceGuard guard(x.device());
  psamd::launch_col2im(col.data_ptr<float>(), n, static_cast<int>(c), static_cast<int>(h), static_cast<int>(w),
                       static_cast<int>(k), static_cast<int>(stride), static_cast<int>(pad), static_cast<int>(oh),
                       static_cast<int>(ow), x.data_ptr<float>(), cur_stream(x));
}

void dropout(Tensor x, Tensor y, double p, int64_t seed, int64_t offset) {
  check_gpu(x, "x");
  check_gpu(y, "y");
  TORCH_CHECK(x.numel() == y.numel() && x.scalar_type() == y.scalar_type(), "dropout shape/dtype");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "p in [0, 1)");
  const c10::DeviceGuard guard(x.device());
  psamd::launch_dropout_fwd(x.data_ptr(), dcode(x, "x"), y.data_ptr(), x.numel(), static_cast<float>(p),
                            static_cast<uint64_t>(seed), static_cast<uint64_t>(offset), cur_stream(x));
}

void uniform_init(Tensor w, int64_t seed, int64_t offset, double lo, double hi) {
  check_f32(w, "w");
  const c10::DeviceGuard guard(w.device());
  psamd::launch_uniform_init(w.data_ptr<float>(), w.numel(), static_cast<uint64_t>(seed),
                             static_cast<uint64_t>(offset), static_cast<float>(lo), static_cast<float>(hi),
                             cur_stream(w));
}

// ------------------------------------------------------------------------------ batchnorm
static std::vector<Tensor> bn_fwd_impl(Tensor x, c10::optional<Tensor> res, c10::optional<Tensor> gamma,
                                       c10::optional<Tensor> beta, c10::optional<Tensor> rmean,
                                       c10::optional<Tensor> rvar, bool training, double momentum, double eps,
                                       int64_t act, bool apply) {
  check_gpu(x, "x");
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16, "x must be bf16 (NHWC-contiguous [R, C] view)");
  TORCH_CHECK(x.dim() == 2, "x must be viewed as [R, C]");
  const int64_t R = x.size(0), C = x.size(1);
  TORCH_CHECK(C % 8 == 0, "C must be a multiple of 8");
  if (res.has_value() && res->defined()) {
    check_gpu(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes() && res->scalar_type() == x.scalar_type(), "res like x");
  }
  for (auto* t : {&gamma, &beta, &rmean, &rvar})
    if (t->has_value() && (*t)->defined()) {
      check_f32(**t, "bn param");
      TORCH_CHECK((*t)->numel() == C, "bn param size");
    }
  if (!training) TORCH_CHECK(rmean.has_value() && rvar.has_value(), "eval mode needs running stats");
  const c10::DeviceGuard guard(x.device());
  auto y = apply ? torch::empty_like(x) : Tensor();
  auto fopt = x.options().dtype(torch::kFloat32);
  auto mean = torch::empty({C}, fopt), invstd = torch::empty({C}, fopt);
  auto coef = torch::empty({2 * C}, fopt);
  const int G = psamd::bn_red_blocks(R, static_cast<int>(C));
  auto ws = torch::empty({training ? 2 * G * C : 1}, fopt);
  psamd::BnFwdArgs a;
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.res = (res.has_value() && res->defined()) ? reinterpret_cast<const uint16_t*>(res->data_ptr()) : nullptr;
  a.y = apply ? reinterpret_cast<uint16_t*>(y.data_ptr()) : nullptr;
  a.gamma = opt_ptr<const float>(gamma);
  a.beta = opt_ptr<const float>(beta);
  a.rmean = opt_ptr<float>(rmean);
  a.rvar = opt_ptr<float>(rvar);
  a.mean = mean.data_ptr<float>();
  a.invstd = invstd.data_ptr<float>();
  a.scale = coef.data_ptr<float>();
  a.shift = coef.data_ptr<float>() + C;
  a.ws = ws.data_ptr<float>();
  a.R = R;
  a.C = static_cast<int>(C);
  a.G = G;
  a.act = static_cast<int>(act);
  a.training = training;
  a.eps = static_cast<float>(eps);
  a.momentum = static_cast<float>(momentum);
  psamd::launch_bn_fwd(a, cur_stream(x));
  return {y, mean, invstd, coef};
}

std::vector<Tensor> bn_act_fwd(Tensor x, c10::optional<Tensor> res, c10::optional<Tensor> gamma,
                               c10::optional<Tensor> beta, c10::optional<Tensor> rmean, c10::optional<Tensor> rvar,
                               bool training, double momentum, double eps, int64_t act) {
  return bn_fwd_impl(x, res, gamma, beta, rmean, rvar, training, momentum, eps, act, true);
}

// batch statistics + running-stat update + [scale | shift] only; the apply is fused into a consumer
std::vector<Tensor> bn_stats(Tensor x, c10::optional<Tensor> gamma, c10::optional<Tensor> beta,
                             c10::optional<Tensor> rmean, c10::optional<Tensor> rvar, bool training, double momentum,
                             double eps) {
  auto r = bn_fwd_impl(x, c10::nullopt, gamma, beta, rmean, rvar, training, momentum, eps, 0, false);
  return {r[1], r[2], r[3]};
}

// ------------------------------------------------------------------------------ transformer row kernels
static void check_rows(const Tensor& t, const char* n) {
  check_gpu(t, n);
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16 && t.is_contiguous(), n, ": bf16 contiguous");
}
static void check_dim(int64_t D) { TORCH_CHECK(D % 8 == 0 && D <= 4096, "row length must be a multiple of 8, <= 4096"); }
static const uint16_t* u16(const Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
static uint16_t* u16m(Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

// x [R, D] (+ r) -> [s (or empty), y, rstd]
std::vector<Tensor> rmsnorm_fwd(Tensor x, c10::optional<Tensor> r, Tensor w, double eps) {
  check_rows(x, "x");
  const int64_t D = x.size(-1), R = x.numel() / D;
  check_dim(D);
  check_gpu(w, "w");
  TORCH_CHECK(w.numel() == D && w.is_contiguous() && (w.scalar_type() == torch::kBFloat16 || w.scalar_type() == torch::kFloat32), "w [D]");
  const bool res = r.has_value() && r->defined();
  if (res) {
    check_rows(*r, "r");
    TORCH_CHECK(r->sizes() == x.sizes(), "r like x");
  }
  const c10::DeviceGuard guard(x.device());
  auto y = torch::empty_like(x);
  auto s = res ? torch::empty_like(x) : Tensor();
  auto rstd = torch::empty({R}, x.options().dtype(torch::kFloat32));
  psamd::launch_rmsnorm_fwd(u16(x), res ? u16(*r) : nullptr, w.data_ptr(), w.scalar_type() == torch::kBFloat16,
                            res ? u16m(s) : nullptr, u16m(y), rstd.data_ptr<float>(), R, D, static_cast<float>(eps),
                            cur_stream(x));
  return {s, y, rstd};
}

// -> [dx, dw (fp32)]; ds_in: extra gradient of s (residual stream) added into dx
std::vector<Tensor> rmsnorm_bwd(Tensor dy, Tensor s, Tensor w, Tensor rstd, c10::optional<Tensor> ds_in) {
  check_rows(dy, "dy");
  check_rows(s, "s");
  TORCH_CHECK(dy.sizes() == s.sizes(), "dy like s");
  const int64_t D = s.size(-1), R = s.numel() / D;
  check_dim(D);
  check_f32(rstd, "rstd");
  const bool add = ds_in.has_value() && ds_in->defined();
  if (add) {
    check_rows(*ds_in, "ds_in");
    TORCH_CHECK(ds_in->sizes() == s.sizes(), "ds_in like s");
  }
  const c10::DeviceGuard guard(s.device());
  auto dx = torch::empty_like(s);
  auto fopt = s.options().dtype(torch::kFloat32);
  auto wpart = torch::empty({psamd::rmsnorm_bwd_parts(static_cast<int>(R)), D}, fopt);
  auto dw = torch::empty({D}, fopt);
  psamd::launch_rmsnorm_bwd(u16(dy), u16(s), w.data_ptr(), w.scalar_type() == torch::kBFloat16, rstd.data_ptr<float>(),
                            add ? u16(*ds_in) : nullptr, u16m(dx), wpart.data_ptr<float>(), dw.data_ptr<float>(), R, D,
                            cur_stream(s));
  return {dx, dw};
}

// s = x + dropout_p(o); y = LN(s) -> [s, y, mean, rstd]
std::vector<Tensor> layernorm_fwd(Tensor x, Tensor o, Tensor gamma, Tensor beta, double eps, double p, int64_t seed) {
  check_rows(x, "x");
  check_rows(o, "o");
  TORCH_CHECK(o.sizes() == x.sizes(), "o like x");
  const int64_t D = x.size(-1), R = x.numel() / D;
  check_dim(D);
  check_gpu(gamma, "gamma");
  check_gpu(beta, "beta");
  const bool wb = gamma.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(gamma.numel() == D && beta.numel() == D && beta.scalar_type() == gamma.scalar_type() &&
                  (wb || gamma.scalar_type() == torch::kFloat32), "gamma/beta [D], fp32 or bf16");
  const c10::DeviceGuard guard(x.device());
  auto s = torch::empty_like(x), y = torch::empty_like(x);
  auto fopt = x.options().dtype(torch::kFloat32);
  auto mean = torch::empty({R}, fopt), rstd = torch::empty({R}, fopt);
  psamd::launch_layernorm_fwd(u16(x), u16(o), gamma.data_ptr(), beta.data_ptr(), wb, u16m(s), u16m(y),
                              mean.data_ptr<float>(), rstd.data_ptr<float>(), R, D, static_cast<float>(eps),
                              static_cast<float>(p), static_cast<uint64_t>(seed), cur_stream(x));
  return {s, y, mean, rstd};
}

// -> [dx (residual input), do (dropout input), dgamma, dbeta]
std::vector<Tensor> layernorm_bwd(Tensor dy, Tensor s, Tensor gamma, Tensor mean, Tensor rstd, double p, int64_t seed) {
  check_rows(dy, "dy");
  check_rows(s, "s");
  TORCH_CHECK(dy.sizes() == s.sizes(), "dy like s");
  const int64_t D = s.size(-1), R = s.numel() / D;
  check_dim(D);
  const c10::DeviceGuard guard(s.device());
  auto dx = torch::empty_like(s), dout = torch::empty_like(s);
  auto fopt = s.options().dtype(torch::kFloat32);
  const int parts = psamd::layernorm_bwd_parts(static_cast<int>(R));
  auto part = torch::empty({2, parts, D}, fopt);
  auto dg = torch::empty({D}, fopt), db = torch::empty({D}, fopt);
  psamd::launch_layernorm_bwd(u16(dy), u16(s), gamma.data_ptr(), gamma.scalar_type() == torch::kBFloat16,
                              mean.data_ptr<float>(), rstd.data_ptr<float>(),
                              u16m(dx), u16m(dout), part.data_ptr<float>(), dg.data_ptr<float>(), db.data_ptr<float>(),
                              R, D, static_cast<float>(p), static_cast<uint64_t>(seed), cur_stream(s));
  return {dx, dout, dg, db};
}

// Fused short-sequence attention (attention.hip): qkv [B, S, 3 * H * 64] -> [out [B, S, H * 64], lse [B, H, S]]
static void check_attn(const Tensor& qkv, int64_t heads) {
  check_rows(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 3 && heads > 0 && qkv.size(2) == 3 * heads * 64, "qkv [B, S, 3 * heads * 64]");
  const int64_t S = qkv.size(1);
  TORCH_CHECK(S > 0 && S % 32 == 0 && S <= 128, "sequence length a multiple of 32, <= 128");
  TORCH_CHECK(qkv.size(0) * heads < (int64_t(1) << 31), "batch * heads");
}

std::vector<Tensor> attn_fwd(Tensor qkv, int64_t heads, double p, int64_t seed) {
  check_attn(qkv, heads);
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout p in [0, 1)");
  const int64_t B = qkv.size(0), S = qkv.size(1);
  const c10::DeviceGuard guard(qkv.device());
  auto out = torch::empty({B, S, heads * 64}, qkv.options());
  auto lse = torch::empty({B, heads, S}, qkv.options().dtype(torch::kFloat32));
  psamd::launch_attn_fwd(u16(qkv), u16m(out), lse.data_ptr<float>(), static_cast<int>(B), static_cast<int>(S),
                         static_cast<int>(heads), 0.125f, static_cast<float>(p), static_cast<uint64_t>(seed),
                         cur_stream(qkv));
  return {out, lse};
}

Tensor attn_bwd(Tensor qkv, Tensor out, Tensor dout, Tensor lse, int64_t heads, double p, int64_t seed) {
  check_attn(qkv, heads);
  const int64_t B = qkv.size(0), S = qkv.size(1);
  check_rows(out, "out");
  check_rows(dout, "dout");
  TORCH_CHECK(out.sizes() == torch::IntArrayRef({B, S, heads * 64}) && dout.sizes() == out.sizes(),
              "out / dout [B, S, heads * 64]");
  check_gpu(lse, "lse");
  TORCH_CHECK(lse.scalar_type() == torch::kFloat32 && lse.is_contiguous() && lse.numel() == B * heads * S,
              "lse fp32 [B, heads, S]");
  const c10::DeviceGuard guard(qkv.device());
  auto dqkv = torch::empty_like(qkv);
  psamd::launch_attn_bwd(u16(qkv), u16(out), u16(dout), lse.data_ptr<float>(), u16m(dqkv), static_cast<int>(B),
                         static_cast<int>(S), static_cast<int>(heads), 0.125f, static_cast<float>(p),
                         static_cast<uint64_t>(seed), cur_stream(qkv));
  return dqkv;
}

// keep mask [B * H, S, S] (uint8) of the attention dropout for (p, seed) -- tests
Tensor attn_dropout_mask(Tensor like, int64_t bh, int64_t S, double p, int64_t seed) {
  check_gpu(like, "like");
  const c10::DeviceGuard guard(like.device());
  auto m = torch::empty({bh, S, S}, like.options().dtype(torch::kUInt8));
  psamd::launch_attn_dropout_mask(m.data_ptr<uint8_t>(), m.numel(), static_cast<float>(p),
                                  static_cast<uint64_t>(seed), cur_stream(like));
  return m;
}

// Causal GQA flash attention: q [B, H, S, 128], k / v [B, KV, S, 128] -> [out [B, S, H * 128], lse [B, H, S]]
static void check_fa(const Tensor& q, const Tensor& k, const Tensor& v) {
  for (const Tensor* t : {&q, &k, &v}) {
    check_gpu(*t, "q/k/v");
    TORCH_CHECK(t->scalar_type() == torch::kBFloat16 && t->is_contiguous() && t->dim() == 4 && t->size(3) == 128,
                "q / k / v: contiguous bf16 [B, heads, S, 128]");
  }
  TORCH_CHECK(k.sizes() == v.sizes() && q.size(0) == k.size(0) && q.size(2) == k.size(2), "k like v, q matches");
  TORCH_CHECK(q.size(1) % k.size(1) == 0, "q heads a multiple of kv heads");
  TORCH_CHECK(q.size(2) % 128 == 0 && q.size(2) > 0, "sequence length a multiple of 128");
}

// fused cross-entropy over bf16 logits [R, V] with int64 labels (ignore_index rows contribute 0)
std::vector<Tensor> xent_fwd(Tensor x, Tensor lab, int64_t ignore) {
  check_gpu(x, "x");
  check_gpu(lab, "labels");
  TORCH_CHECK(x.dim() == 2 && x.scalar_type() == torch::kBFloat16 && x.is_contiguous(), "x: contiguous bf16 [R, V]");
  TORCH_CHECK(lab.scalar_type() == torch::kInt64 && lab.numel() == x.size(0) && lab.is_contiguous(), "labels [R] int64");
  TORCH_CHECK(x.size(1) < (int64_t(1) << 31), "vocab");
  const c10::DeviceGuard guard(x.device());
  auto fopt = x.options().dtype(torch::kFloat32);
  auto lse = torch::empty({x.size(0)}, fopt), loss = torch::empty({x.size(0)}, fopt);
  psamd::launch_xent_fwd(u16(x), lab.data_ptr<int64_t>(), x.size(0), static_cast<int>(x.size(1)), ignore,
                         lse.data_ptr<float>(), loss.data_ptr<float>(), cur_stream(x));
  return {lse, loss};
}

Tensor xent_bwd(Tensor x, Tensor lab, Tensor lse, Tensor go, Tensor count, int64_t ignore) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.scalar_type() == torch::kBFloat16 && x.is_contiguous(), "x: contiguous bf16 [R, V]");
  TORCH_CHECK(lab.scalar_type() == torch::kInt64 && lab.numel() == x.size(0), "labels [R] int64");
  check_f32(lse, "lse");
  check_f32(go, "go");
  check_f32(count, "count");
  TORCH_CHECK(lse.numel() == x.size(0) && go.numel() == 1 && count.numel() == 1, "lse [R], go / count scalars");
  const c10::DeviceGuard guard(x.device());
  auto dx = torch::empty_like(x);
  psamd::launch_xent_bwd(u16(x), lab.data_ptr<int64_t>(), lse.data_ptr<float>(), x.size(0), static_cast<int>(x.size(1)),
                         ignore, go.data_ptr<float>(), count.data_ptr<float>(), u16m(dx), cur_stream(x));
  return dx;
}

std::vector<Tensor> fa_fwd(Tensor q, Tensor k, Tensor v) {
  check_fa(q, k, v);
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), KV = k.size(1);
  const c10::DeviceGuard guard(q.device());
  auto out = torch::empty({B, S, H * 128}, q.options());
  auto lse = torch::empty({B, H, S}, q.options().dtype(torch::kFloat32));
  psamd::launch_fa_fwd(u16(q), u16(k), u16(v), u16m(out), lse.data_ptr<float>(), static_cast<int>(B),
                       static_cast<int>(S), static_cast<int>(H), static_cast<int>(KV), 1.f / std::sqrt(128.f),
                       cur_stream(q));
  return {out, lse};
}

std::vector<Tensor> fa_bwd(Tensor q, Tensor k, Tensor v, Tensor out, Tensor dout, Tensor lse) {
  check_fa(q, k, v);
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), KV = k.size(1);
  check_rows(out, "out");
  check_rows(dout, "dout");
  TORCH_CHECK(out.numel() == B * S * H * 128 && dout.numel() == out.numel(), "out / dout [B, S, H * 128]");
  check_gpu(lse, "lse");
  TORCH_CHECK(lse.scalar_type() == torch::kFloat32 && lse.numel() == B * H * S, "lse fp32 [B, H, S]");
  const c10::DeviceGuard guard(q.device());
  auto fopt = q.options().dtype(torch::kFloat32);
  auto dsum = torch::empty({B, H, S}, fopt);
  auto dq = torch::empty_like(q), dk = torch::empty_like(k), dv = torch::empty_like(v);
  psamd::launch_fa_bwd(u16(q), u16(k), u16(v), u16(out), u16(dout), lse.data_ptr<float>(), dsum.data_ptr<float>(),
                       u16m(dq), u16m(dk), u16m(dv),
                       static_cast<int>(B), static_cast<int>(S), static_cast<int>(H), static_cast<int>(KV),
                       1.f / std::sqrt(128.f), cur_stream(q));
  return {dq, dk, dv};
}

Tensor swiglu_fwd(Tensor gu) {
  check_rows(gu, "gu");
  const int64_t F2 = gu.size(-1), R = gu.numel() / F2;
  TORCH_CHECK(F2 % 16 == 0, "2F % 16");
  const c10::DeviceGuard guard(gu.device());
  auto shape = gu.sizes().vec();
  shape.back() = F2 / 2;
  auto h = torch::empty(shape, gu.options());
  psamd::launch_swiglu_fwd(u16(gu), u16m(h), R, static_cast<int>(F2 / 2), cur_stream(gu));
  return h;
}

Tensor swiglu_bwd(Tensor dh, Tensor gu) {
  check_rows(dh, "dh");
  check_rows(gu, "gu");
  const int64_t F2 = gu.size(-1), R = gu.numel() / F2;
  TORCH_CHECK(dh.numel() == R * (F2 / 2), "dh [.., F]");
  const c10::DeviceGuard guard(gu.device());
  auto dgu = torch::empty_like(gu);
  psamd::launch_swiglu_bwd(u16(dh), u16(gu), u16m(dgu), R, static_cast<int>(F2 / 2), cur_stream(gu));
  return dgu;
}

// qkv [B, S, H + 2KV, hd] -> [q [B,H,S,hd], k [B,KV,S,hd], v [B,KV,S,hd]]; cs [S, hd/2, 2] fp32
std::vector<Tensor> rope_split_fwd(Tensor qkv, Tensor cs, int64_t H, int64_t KV) {
  check_rows(qkv, "qkv");
  check_f32(cs, "cs");
  TORCH_CHECK(qkv.dim() == 4 && qkv.size(2) == H + 2 * KV, "qkv [B, S, H+2KV, hd]");
  const int64_t B = qkv.size(0), S = qkv.size(1), hd = qkv.size(3);
  TORCH_CHECK(hd % 16 == 0 && cs.numel() == S * hd, "hd % 16, cs [S, hd/2, 2]");
  const c10::DeviceGuard guard(qkv.device());
  auto q = torch::empty({B, H, S, hd}, qkv.options());
  auto k = torch::empty({B, KV, S, hd}, qkv.options());
  auto v = torch::empty({B, KV, S, hd}, qkv.options());
  psamd::launch_rope_split_fwd(u16(qkv), cs.data_ptr<float>(), u16m(q), u16m(k), u16m(v), B, S, H, KV, hd,
                               cur_stream(qkv));
  return {q, k, v};
}

Tensor rope_split_bwd(Tensor dq, Tensor dk, Tensor dv, Tensor cs) {
  check_rows(dq, "dq");
  check_rows(dk, "dk");
  check_rows(dv, "dv");
  const int64_t B = dq.size(0), H = dq.size(1), S = dq.size(2), hd = dq.size(3), KV = dk.size(1);
  TORCH_CHECK(dk.sizes() == dv.sizes() && dk.size(0) == B && dk.size(2) == S && dk.size(3) == hd, "dk/dv [B,KV,S,hd]");
  const c10::DeviceGuard guard(dq.device());
  auto dqkv = torch::empty({B, S, H + 2 * KV, hd}, dq.options());
  psamd::launch_rope_split_bwd(u16(dq), u16(dk), u16(dv), cs.data_ptr<float>(), u16m(dqkv), B, S, H, KV, hd,
                               cur_stream(dq));
  return dqkv;
}

// ------------------------------------------------------------------------------ DLRM interaction
static void check_interact(const Tensor& x, const Tensor& e) {
  check_gpu(x, "x");
  check_gpu(e, "e");
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 && e.scalar_type() == torch::kBFloat16, "bf16 x/e");
  TORCH_CHECK(x.dim() == 2 && e.dim() == 3 && e.size(0) == x.size(0) && e.size(2) == x.size(1), "x [B,D], e [B,T,D]");
  TORCH_CHECK(x.is_contiguous() && e.is_contiguous(), "contiguous x/e");
  TORCH_CHECK(e.size(1) + 1 <= 32 && x.size(1) % 32 == 0 && x.size(1) <= 224, "n = T+1 <= 32, D % 32 == 0, D <= 224");
}

Tensor dlrm_interact_fwd(Tensor x, Tensor e) {
  check_interact(x, e);
  const int64_t B = x.size(0), D = x.size(1), T = e.size(1), n = T + 1;
  const c10::DeviceGuard guard(x.device());
  auto out = torch::empty({B, D + n * (n - 1) / 2}, x.options());
  psamd::launch_dlrm_interact_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                  reinterpret_cast<const uint16_t*>(e.data_ptr()),
                                  reinterpret_cast<uint16_t*>(out.data_ptr()), B, T, D, cur_stream(x));
  return out;
}

std::vector<Tensor> dlrm_interact_bwd(Tensor x, Tensor e, Tensor dout) {
  check_interact(x, e);
  const int64_t B = x.size(0), D = x.size(1), T = e.size(1), n = T + 1;
  check_gpu(dout, "dout");
  TORCH_CHECK(dout.scalar_type() == torch::kBFloat16 && dout.is_contiguous() && dout.dim() == 2 &&
                  dout.size(0) == B && dout.size(1) == D + n * (n - 1) / 2, "dout [B, D + n(n-1)/2] bf16");
  const c10::DeviceGuard guard(x.device());
  auto dx = torch::empty_like(x);
  auto de = torch::empty_like(e);
  psamd::launch_dlrm_interact_bwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                  reinterpret_cast<const uint16_t*>(e.data_ptr()),
                                  reinterpret_cast<const uint16_t*>(dout.data_ptr()),
                                  reinterpret_cast<uint16_t*>(dx.data_ptr()), reinterpret_cast<uint16_t*>(de.data_ptr()),
                                  B, T, D, cur_stream(x));
  return {dx, de};
}

// ------------------------------------------------------------------------------ ResNet stem conv
static void check_stem(const Tensor& x) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 4 && (x.size(3) == 3 || x.size(3) == 4) && x.scalar_type() == torch::kBFloat16 &&
                  x.is_contiguous(), "x: [N, H, W, 3 or 4] bf16 contiguous");
}

// returns [z, part]; with kshift (running mean, [64] fp32) the BN partial sums of z are
// produced in the conv epilogue: part [2, blocks, 64] (else an empty tensor)
std::vector<Tensor> stem_conv_fwd(Tensor x, Tensor wp, c10::optional<Tensor> kshift) {
  check_stem(x);
  check_gpu(wp, "wp");
  TORCH_CHECK(wp.scalar_type() == torch::kBFloat16 && wp.numel() == 64 * 224 && wp.is_contiguous(), "wp [64,224]");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(OW <= 128, "stem kernel supports OW <= 128");
  const bool stats = kshift.has_value() && kshift->defined();
  if (stats) {
    check_f32(*kshift, "kshift");
    TORCH_CHECK(kshift->numel() == 64, "kshift [64]");
  }
  const c10::DeviceGuard guard(x.device());
  auto z = torch::empty({N, OH, OW, 64}, x.options());
  const int nblk = psamd::stem_fwd_blocks(static_cast<int>(N));
  auto part = stats ? torch::empty({2, nblk, 64}, x.options().dtype(torch::kFloat32)) : Tensor();
  psamd::launch_stem_conv_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()), static_cast<int>(x.size(3)),
                              reinterpret_cast<const uint16_t*>(wp.data_ptr()), reinterpret_cast<uint16_t*>(z.data_ptr()),
                              N, H, W, OH, OW, stats ? kshift->data_ptr<float>() : nullptr,
                              stats ? part.data_ptr<float>() : nullptr, cur_stream(x));
  return {z, part};
}

// BN statistics from producer partial sums: part [2, G, C] about kshift over R rows.
// [2, G, C] partials -> a [2, S, C] first-level fold when G is tall (S = partials_fold_rows(G)),
// else the input itself
// part [2, G, C] with contiguous slabs (part.stride(0) >= G * C: e.g. slabs 0 and 2 of a [3, G, C]
// epilogue-9 part, no stacking copy); the second slab starts part.stride(0) floats after the first
static bool slabs_ok(const Tensor& part) {
  return part.dim() == 3 && part.size(0) == 2 && part.stride(2) == 1 && part.stride(1) == part.size(2) &&
         part.stride(0) >= part.size(1) * part.size(2);
}

static void check_part_slabs(const Tensor& part) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == torch::kFloat32, "part must be a float32 GPU tensor");
  TORCH_CHECK(slabs_ok(part), "part [2, G, C] (contiguous slabs)");
}

static Tensor fold_partials(const Tensor& part, hipStream_t s) {
  const int G = static_cast<int>(part.size(1)), C = static_cast<int>(part.size(2));
  const int S = psamd::partials_fold_rows(G);
  if (S == 0) return part;
  auto f = torch::empty({2, S, C}, part.options());
  psamd::launch_partials_fold(part.data_ptr<float>(), part.data_ptr<float>() + part.stride(0), G, C,
                              f.data_ptr<float>(), f.data_ptr<float>() + static_cast<int64_t>(S) * C, s);
  return f;
}

// Returns [mean, invstd, coef = scale | shift]; updates running stats when given.
std::vector<Tensor> bn_finalize_sums(Tensor part, Tensor kshift, int64_t R, c10::optional<Tensor> gamma,
                                     c10::optional<Tensor> beta, c10::optional<Tensor> rmean,
                                     c10::optional<Tensor> rvar, double momentum, double eps) {
  check_f32(part, "part");
  check_f32(kshift, "kshift");
  TORCH_CHECK(part.dim() == 3 && part.size(0) == 2 && part.is_contiguous(), "part [2, G, C]");
  const int64_t C = part.size(2);
  TORCH_CHECK(C % 8 == 0 && kshift.numel() == C, "C % 8, kshift [C]");
  const c10::DeviceGuard guard(part.device());
  auto fopt = part.options();
  auto mean = torch::empty({C}, fopt), invstd = torch::empty({C}, fopt), coef = torch::empty({2 * C}, fopt);
  const Tensor fp = fold_partials(part, cur_stream(part));
  const int64_t Gf = fp.size(1);
  psamd::launch_bn_finalize_sums(fp.data_ptr<float>(), fp.data_ptr<float>() + Gf * C, kshift.data_ptr<float>(),
                                 static_cast<int>(Gf), static_cast<int>(C), R, static_cast<float>(eps),
                                 static_cast<float>(momentum), opt_ptr<const float>(gamma), opt_ptr<const float>(beta),
                                 opt_ptr<float>(rmean), opt_ptr<float>(rvar), mean.data_ptr<float>(),
                                 invstd.data_ptr<float>(), coef.data_ptr<float>(), coef.data_ptr<float>() + C,
                                 cur_stream(part));
  return {mean, invstd, coef};
}

Tensor stem_conv_wrw(Tensor x, Tensor dz) {
  check_stem(x);
  check_gpu(dz, "dz");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(dz.dim() == 4 && dz.size(0) == N && dz.size(1) == OH && dz.size(2) == OW && dz.size(3) == 64 &&
                  dz.scalar_type() == torch::kBFloat16 && dz.is_contiguous(), "dz: [N, OH, OW, 64] bf16 contiguous");
  TORCH_CHECK(OW <= 128, "stem kernel supports OW <= 128");
  const c10::DeviceGuard guard(x.device());
  auto fopt = x.options().dtype(torch::kFloat32);
  const int nblk = psamd::stem_wrw_blocks(N, OH);
  auto ws = torch::empty({(nblk + 32) * 64 * 224}, fopt);
  auto dwp = torch::empty({64, 224}, fopt);
  psamd::launch_stem_conv_wrw(reinterpret_cast<const uint16_t*>(x.data_ptr()), static_cast<int>(x.size(3)),
                              reinterpret_cast<const uint16_t*>(dz.data_ptr()), ws.data_ptr<float>(),
                              dwp.data_ptr<float>(), N, H, W, OH, OW, cur_stream(x));
  return dwp;
}

// Stem backward with the BN-backward apply inside the weight gradient: the statistics pass of
// pool_bn_bwd (dgamma, dbeta, coefficients), then stem_conv_wrw computing each dz row from the
// pooled gradient + argmax + z -- the full-resolution dz never reaches HBM.  -> [dwp, dg, db]
std::vector<Tensor> stem_bwd_fused(Tensor x, Tensor dy, Tensor idx, Tensor z, Tensor mask_coef, Tensor gamma,
                                   Tensor mean, Tensor invstd) {
  check_stem(x);
  check_gpu(dy, "dy");
  check_gpu(z, "z");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(z.dim() == 4 && z.size(0) == N && z.size(1) == OH && z.size(2) == OW && z.size(3) == 64 &&
                  z.scalar_type() == torch::kBFloat16 && z.is_contiguous(), "z: [N, OH, OW, 64] bf16 contiguous");
  TORCH_CHECK(OW <= 128 && OH % 2 == 0 && OW % 2 == 0, "stem: OW <= 128, even OH / OW");
  TORCH_CHECK(dy.dim() == 4 && dy.size(0) == N && dy.size(1) == OH / 2 && dy.size(2) == OW / 2 && dy.size(3) == 64 &&
                  dy.scalar_type() == torch::kBFloat16 && dy.is_contiguous(), "dy: [N, OH/2, OW/2, 64] bf16");
  TORCH_CHECK(idx.sizes() == dy.sizes() && idx.scalar_type() == torch::kUInt8 && idx.is_contiguous(), "idx like dy");
  for (const Tensor* t : {&mask_coef, &gamma, &mean, &invstd}) check_f32(*t, "bn vector");
  TORCH_CHECK(mask_coef.numel() == 128 && gamma.numel() == 64 && mean.numel() == 64 && invstd.numel() == 64, "bn sizes");
  const c10::DeviceGuard guard(x.device());
  auto fopt = x.options().dtype(torch::kFloat32);
  const int C = 64;
  const int G = psamd::pool_bn_bwd_blocks(N, static_cast<int>(OH), static_cast<int>(OW), C);
  auto pws = torch::empty({2 * G * C + 3 * C}, fopt);
  auto dg = torch::empty({C}, fopt), db = torch::empty({C}, fopt);
  const auto st = cur_stream(x);
  psamd::launch_pool_bn_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()), idx.data_ptr<uint8_t>(),
                            reinterpret_cast<const uint16_t*>(z.data_ptr()), mask_coef.data_ptr<float>(),
                            mean.data_ptr<float>(), invstd.data_ptr<float>(), gamma.data_ptr<float>(),
                            pws.data_ptr<float>(), G, dg.data_ptr<float>(), db.data_ptr<float>(), nullptr,
                            static_cast<int>(N), static_cast<int>(OH), static_cast<int>(OW), C,
                            static_cast<int>(OH / 2), static_cast<int>(OW / 2), st);
  const int nblk = psamd::stem_wrw_blocks(N, OH);
  auto ws = torch::empty({(nblk + 32) * 64 * 224}, fopt);
  auto dwp = torch::empty({64, 224}, fopt);
  psamd::launch_stem_conv_wrw(reinterpret_cast<const uint16_t*>(x.data_ptr()), static_cast<int>(x.size(3)),
                              reinterpret_cast<const uint16_t*>(z.data_ptr()), ws.data_ptr<float>(),
                              dwp.data_ptr<float>(), N, H, W, OH, OW, st,
                              reinterpret_cast<const uint16_t*>(dy.data_ptr()), idx.data_ptr<uint8_t>(),
                              mask_coef.data_ptr<float>(), pws.data_ptr<float>() + 2 * G * C);
  return {dwp, dg, db};
}

// ------------------------------------------------------------------------------ NHWC max pool
// x: [N, H, W, C] bf16 contiguous; coef: optional [scale | shift] (fused BN-apply + ReLU prologue)
std::vector<Tensor> maxpool_nhwc_fwd(Tensor x, c10::optional<Tensor> coef, int64_t k, int64_t s, int64_t p) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.scalar_type() == torch::kBFloat16 && x.is_contiguous(), "x: [N,H,W,C] bf16");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0 && k >= 1 && k <= 15 && s >= 1 && p >= 0 && p < k, "unsupported pool geometry");
  const bool bn = coef.has_value() && coef->defined();
  if (bn) {
    check_f32(*coef, "coef");
    TORCH_CHECK(coef->numel() == 2 * C, "coef = [scale | shift]");
  }
  const int64_t OH = (H + 2 * p - k) / s + 1, OW = (W + 2 * p - k) / s + 1;
  TORCH_CHECK(OH > 0 && OW > 0, "empty output");
  const c10::DeviceGuard guard(x.device());
  auto y = torch::empty({N, OH, OW, C}, x.options());
  auto idx = torch::empty({N, OH, OW, C}, x.options().dtype(torch::kUInt8));
  psamd::launch_maxpool_nhwc_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()), bn ? coef->data_ptr<float>() : nullptr,
                                 reinterpret_cast<uint16_t*>(y.data_ptr()), idx.data_ptr<uint8_t>(), N, H, W, C, OH,
                                 OW, k, s, p, cur_stream(x));
  return {y, idx};
}

Tensor maxpool_nhwc_bwd(Tensor dy, Tensor idx, int64_t H, int64_t W, int64_t k, int64_t s, int64_t p) {
  check_gpu(dy, "dy");
  TORCH_CHECK(dy.dim() == 4 && dy.scalar_type() == torch::kBFloat16 && dy.is_contiguous(), "dy: [N,OH,OW,C] bf16");
  TORCH_CHECK(idx.sizes() == dy.sizes() && idx.scalar_type() == torch::kUInt8 && idx.is_contiguous(), "idx like dy");
  const int64_t N = dy.size(0), OH = dy.size(1), OW = dy.size(2), C = dy.size(3);
  TORCH_CHECK(C % 8 == 0 && OH == (H + 2 * p - k) / s + 1 && OW == (W + 2 * p - k) / s + 1, "pool geometry");
  const c10::DeviceGuard guard(dy.device());
  auto dx = torch::empty({N, H, W, C}, dy.options());
  psamd::launch_maxpool_nhwc_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()), idx.data_ptr<uint8_t>(),
                                 reinterpret_cast<uint16_t*>(dx.data_ptr()), N, H, W, C, OH, OW, k, s, p,
                                 cur_stream(dy));
  return dx;
}

// ------------------------------------------------------------------ one-node row exchange
static psamd::RowPeers row_peers(const std::vector<int64_t>& skeys, const std::vector<int64_t>& meta,
                                 const std::vector<int64_t>& rows, const std::vector<int64_t>& grads) {
  psamd::RowPeers P{};
  const size_t W = std::max({skeys.size(), meta.size(), rows.size(), grads.size()});
  TORCH_CHECK(W >= 1 && W <= static_cast<size_t>(psamd::kPlaneMaxSrc), "row plane: 1..", psamd::kPlaneMaxSrc, " ranks");
  for (size_t w = 0; w < W; ++w) {
    if (w < skeys.size()) P.skeys[w] = reinterpret_cast<const int64_t*>(skeys[w]);
    if (w < meta.size()) P.meta[w] = reinterpret_cast<const int64_t*>(meta[w]);
    if (w < rows.size()) P.rows[w] = reinterpret_cast<float*>(rows[w]);
    if (w < grads.size()) P.grads[w] = reinterpret_cast<const float*>(grads[w]);
  }
  P.W = static_cast<int>(W);
  return P;
}

static void check_i64_gpu(const Tensor& t, int64_t n, const char* what) {
  check_gpu(t, what);
  TORCH_CHECK(t.scalar_type() == torch::kInt64 && t.is_contiguous() && t.numel() == n, what, ": int64 [", n, "]");
}

// owner: rkeys[w * cap + j] = worker w's j-th key for this owner (-1 past its count); pmeta = the
// W (offset, count) pairs
void row_plane_recv(std::vector<int64_t> skeys, std::vector<int64_t> meta, int64_t me, int64_t cap, Tensor rkeys,
                    Tensor pmeta) {
  const auto P = row_peers(skeys, meta, {}, {});
  TORCH_CHECK(skeys.size() == meta.size() && me >= 0 && me < P.W && cap > 0, "row plane recv args");
  check_i64_gpu(rkeys, P.W * cap, "rkeys");
  check_i64_gpu(pmeta, 2 * P.W, "pmeta");
  const c10::DeviceGuard guard(rkeys.device());
  psamd::launch_row_plane_recv(P, static_cast<int>(me), cap, rkeys.data_ptr<int64_t>(), pmeta.data_ptr<int64_t>(),
                               cur_stream(rkeys));
}

// owner: rows of rslots -> every worker's arena rows at its offsets
void row_plane_send(Tensor table, Tensor rslots, Tensor pmeta, std::vector<int64_t> rows, int64_t cap) {
  const auto P = row_peers({}, {}, rows, {});
  check_f32(table, "table");
  TORCH_CHECK(table.dim() == 2 && table.is_contiguous(), "table [rows, dim]");
  check_i64_gpu(rslots, P.W * cap, "rslots");
  check_i64_gpu(pmeta, 2 * P.W, "pmeta");
  const int dim = static_cast<int>(table.size(1));
  const int lpe = dim % 4 == 0 ? dim / 4 : dim;
  TORCH_CHECK(cap % 256 == 0, "row plane capacity must be a multiple of 256");
  TORCH_CHECK(dim % 4 != 0 || (reinterpret_cast<uintptr_t>(table.data_ptr()) & 15) == 0, "table 16-B aligned");
  (void)lpe;
  const c10::DeviceGuard guard(table.device());
  psamd::launch_row_plane_send(table.data_ptr<float>(), rslots.data_ptr<int64_t>(), pmeta.data_ptr<int64_t>(), P, cap,
                               dim, cur_stream(table));
}

// owner: the W workers' pushed rows -> acc, in rank order (tflag / tag / touched / tcount: the
// round's touched-slot list)
void row_plane_accum(std::vector<int64_t> grads, Tensor rslots, Tensor pmeta, Tensor acc, Tensor tflag, int64_t tag,
                     Tensor touched, Tensor tcount, int64_t cap) {
  const auto P = row_peers({}, {}, {}, grads);
  check_f32(acc, "acc");
  TORCH_CHECK(acc.dim() == 2 && acc.is_contiguous(), "acc [rows, dim]");
  check_i64_gpu(rslots, P.W * cap, "rslots");
  check_i64_gpu(pmeta, 2 * P.W, "pmeta");
  check_i64_gpu(touched, acc.size(0), "touched");  // at most one entry per slot
  check_gpu(tflag, "tflag");
  check_gpu(tcount, "tcount");
  TORCH_CHECK(tflag.scalar_type() == torch::kInt32 && tflag.numel() == acc.size(0), "tflag: int32 [rows]");
  TORCH_CHECK(tcount.scalar_type() == torch::kInt32 && tcount.numel() == 1, "tcount: int32 [1]");
  const c10::DeviceGuard guard(acc.device());
  psamd::launch_row_plane_accum(P, rslots.data_ptr<int64_t>(), pmeta.data_ptr<int64_t>(), acc.data_ptr<float>(),
                                tflag.data_ptr<int32_t>(), static_cast<int32_t>(tag), touched.data_ptr<int64_t>(),
                                tcount.data_ptr<int32_t>(), cap, static_cast<int>(acc.size(1)), cur_stream(acc));
}

// stem: dz, dgamma, dbeta of z -> BN -> ReLU -> maxpool 3x3/2/1 from the pooled gradient (pool.hip)
std::vector<Tensor> pool_bn_bwd(Tensor dy, Tensor idx, Tensor z, Tensor mask_coef, Tensor gamma, Tensor mean,
                                Tensor invstd) {
  check_gpu(dy, "dy");
  check_gpu(z, "z");
  TORCH_CHECK(dy.dim() == 4 && dy.scalar_type() == torch::kBFloat16 && dy.is_contiguous(), "dy: [N,OH,OW,C] bf16");
  TORCH_CHECK(z.dim() == 4 && z.scalar_type() == torch::kBFloat16 && z.is_contiguous(), "z: [N,H,W,C] bf16");
  TORCH_CHECK(idx.sizes() == dy.sizes() && idx.scalar_type() == torch::kUInt8 && idx.is_contiguous(), "idx like dy");
  const int64_t N = z.size(0), H = z.size(1), W = z.size(2), C = z.size(3);
  TORCH_CHECK(dy.size(0) == N && dy.size(3) == C && H % 2 == 0 && W % 2 == 0 && dy.size(1) == H / 2 &&
                  dy.size(2) == W / 2, "pool 3x3/2/1 over even H, W");
  TORCH_CHECK(C % 8 == 0 && 256 % (C / 8) == 0, "C / 8 must divide 256");
  TORCH_CHECK(N * (H / 2) * (W / 2) * (C / 8) < (int64_t(1) << 31), "32-bit quad index");
  for (const Tensor* t : {&mask_coef, &gamma, &mean, &invstd}) check_f32(*t, "bn vector");
  TORCH_CHECK(mask_coef.numel() == 2 * C && gamma.numel() == C && mean.numel() == C && invstd.numel() == C, "bn sizes");
  const c10::DeviceGuard guard(z.device());
  auto fopt = z.options().dtype(torch::kFloat32);
  const int G = psamd::pool_bn_bwd_blocks(N, static_cast<int>(H), static_cast<int>(W), static_cast<int>(C));
  auto ws = torch::empty({2 * G * C + 3 * C}, fopt);
  auto dz = torch::empty_like(z);
  auto dg = torch::empty({C}, fopt), db = torch::empty({C}, fopt);
  psamd::launch_pool_bn_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()), idx.data_ptr<uint8_t>(),
                            reinterpret_cast<const uint16_t*>(z.data_ptr()), mask_coef.data_ptr<float>(),
                            mean.data_ptr<float>(), invstd.data_ptr<float>(), gamma.data_ptr<float>(),
                            ws.data_ptr<float>(), G, dg.data_ptr<float>(), db.data_ptr<float>(),
                            reinterpret_cast<uint16_t*>(dz.data_ptr()), static_cast<int>(N), static_cast<int>(H),
                            static_cast<int>(W), static_cast<int>(C), static_cast<int>(H / 2), static_cast<int>(W / 2),
                            cur_stream(z));
  return {dz, dg, db};
}

std::vector<Tensor> bn_act_bwd(Tensor dy, c10::optional<Tensor> y, Tensor x, c10::optional<Tensor> gamma, Tensor mean,
                               Tensor invstd, int64_t act, bool want_dres, bool affine,
                               c10::optional<Tensor> mask_coef, c10::optional<Tensor> mbits) {
  check_gpu(dy, "dy");
  check_gpu(x, "x");
  const bool has_y = y.has_value() && y->defined();
  const bool has_mc = mask_coef.has_value() && mask_coef->defined();
  TORCH_CHECK(x.dim() == 2 && dy.sizes() == x.sizes(), "dy/x [R, C]");
  TORCH_CHECK(dy.scalar_type() == torch::kBFloat16 && x.scalar_type() == torch::kBFloat16, "bf16 tensors");
  if (has_y) {
    check_gpu(*y, "y");
    TORCH_CHECK(y->sizes() == x.sizes() && y->scalar_type() == torch::kBFloat16, "y like x");
  }
  if (has_mc) {
    check_f32(*mask_coef, "mask_coef");
    TORCH_CHECK(mask_coef->numel() == 2 * x.size(1), "mask_coef = [scale | shift]");
    TORCH_CHECK(!want_dres, "recomputed relu mask is only valid without a residual");
  }
  const bool has_mb = mbits.has_value() && mbits->defined();
  if (has_mb) {
    check_gpu(*mbits, "mbits");
    TORCH_CHECK(mbits->scalar_type() == torch::kUInt8 && mbits->numel() * 8 == x.numel(), "mbits: uint8 [R*C/8]");
  }
  TORCH_CHECK(act == 0 || has_y || has_mc || has_mb, "relu backward needs y, mask_coef or mbits");
  const int64_t R = x.size(0), C = x.size(1);
  TORCH_CHECK(C % 8 == 0, "C % 8");
  check_f32(mean, "mean");
  check_f32(invstd, "invstd");
  TORCH_CHECK(mean.numel() == C && invstd.numel() == C, "stats size");
  if (gamma.has_value() && gamma->defined()) check_f32(*gamma, "gamma");
  const c10::DeviceGuard guard(x.device());
  auto fopt = x.options().dtype(torch::kFloat32);
  auto dx = torch::empty_like(x);
  Tensor dres = want_dres ? torch::empty_like(x) : Tensor();
  Tensor dgamma = affine ? torch::empty({C}, fopt) : Tensor();
  Tensor dbeta = affine ? torch::empty({C}, fopt) : Tensor();
  const int G = psamd::bn_red_blocks(R, static_cast<int>(C));
  auto ws = torch::empty({2 * G * C + 3 * C}, fopt);
  psamd::BnBwdArgs a;
  a.dy = reinterpret_cast<const uint16_t*>(dy.data_ptr());
  a.y = has_y ? reinterpret_cast<const uint16_t*>(y->data_ptr()) : nullptr;
  a.mask_coef = has_mc ? mask_coef->data_ptr<float>() : nullptr;
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.gamma = opt_ptr<const float>(gamma);
  a.mean = mean.data_ptr<float>();
  a.invstd = invstd.data_ptr<float>();
  a.dgamma = affine ? dgamma.data_ptr<float>() : nullptr;
  a.dbeta = affine ? dbeta.data_ptr<float>() : nullptr;
  a.dx = reinterpret_cast<uint16_t*>(dx.data_ptr());
  a.dres = want_dres ? reinterpret_cast<uint16_t*>(dres.data_ptr()) : nullptr;
  a.mbits = has_mb ? mbits->data_ptr<uint8_t>() : nullptr;
  a.ws = ws.data_ptr<float>();
  a.R = R;
  a.C = static_cast<int>(C);
  a.G = G;
  a.act = static_cast<int>(act);
  psamd::launch_bn_bwd(a, cur_stream(x));
  return {dx, dres, dgamma, dbeta};
}

// ------------------------------------------------------------------------------ MFMA linear
void gemm_nt(Tensor a, Tensor b, Tensor c, c10::optional<Tensor> bias, int64_t act, double alpha, bool accumulate) {
  check_gpu(a, "a");
  check_gpu(b, "b");
  check_gpu(c, "c");
  TORCH_CHECK(a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16, "a, b must be bf16");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "2-D operands");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "inner dims differ: ", K, " vs ", b.size(1));
  TORCH_CHECK(c.size(0) == M && c.size(1) == N, "c must be [M, N]");
  if (bias.has_value() && bias->defined()) {
    check_f32(*bias, "bias");
    TORCH_CHECK(bias->numel() == N, "bias must be [N]");
  }
  const c10::DeviceGuard guard(a.device());
  psamd::launch_gemm_nt_bf16(reinterpret_cast<const uint16_t*>(a.data_ptr()), K,
                             reinterpret_cast<const uint16_t*>(b.data_ptr()), K, c.data_ptr(), dcode(c, "c") == 0, N,
                             static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), static_cast<float>(alpha),
                             accumulate, opt_ptr<const float>(bias), static_cast<int>(act), cur_stream(a));
}

Tensor act_bwd(Tensor dy, Tensor y, int64_t act) {
  check_gpu(dy, "dy");
  check_gpu(y, "y");
  TORCH_CHECK(dy.scalar_type() == torch::kBFloat16 && y.scalar_type() == torch::kBFloat16, "bf16");
  TORCH_CHECK(dy.numel() == y.numel(), "dy/y size");
  const c10::DeviceGuard guard(dy.device());
  auto dz = torch::empty_like(dy);
  psamd::launch_act_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(y.data_ptr()),
                        reinterpret_cast<uint16_t*>(dz.data_ptr()), dy.numel(), static_cast<int>(act), cur_stream(dy));
  return dz;
}

// ------------------------------------------------------------------------------ implicit-GEMM convs (convgemm.hip)
static const float* f32_opt(const c10::optional<Tensor>& t, int64_t n, const char* name) {
  if (!(t.has_value() && t->defined())) return nullptr;
  check_f32(*t, name);
  TORCH_CHECK(t->numel() == n, name, ": expected ", n, " elements, got ", t->numel());
  return t->data_ptr<float>();
}

// geo = [H, W, OH, OW, ks, stride, pad] of a [images*H*W, C] NHWC row tensor -> (geometry, images)
static std::pair<psamd::ConvGeo, int64_t> conv_geo(const Tensor& a, const std::vector<int64_t>& geo) {
  TORCH_CHECK(geo.size() == 7, "geo = [H, W, OH, OW, ks, stride, pad]");
  const int64_t H = geo[0], W = geo[1], OH = geo[2], OW = geo[3], ks = geo[4], st = geo[5], pd = geo[6];
  TORCH_CHECK(H > 0 && W > 0 && ks >= 1 && ks <= 7 && st >= 1 && st <= 4 && pd >= 0 && pd < ks, "conv geometry");
  TORCH_CHECK(OH == (H + 2 * pd - ks) / st + 1 && OW == (W + 2 * pd - ks) / st + 1, "output map size");
  const int64_t C = a.size(1);
  TORCH_CHECK(C % 64 == 0, "input channels must be a multiple of 64");
  TORCH_CHECK(a.size(0) % (H * W) == 0, "rows of the input must be images * H * W");
  psamd::ConvGeo g{static_cast<int>(H), static_cast<int>(W), static_cast<int>(OH), static_cast<int>(OW),
                   static_cast<int>(C), static_cast<int>(ks), static_cast<int>(st), static_cast<int>(pd)};
  return {g, a.size(0) / (H * W)};
}

// The tile plan conv_gemm picks: [bm, bn, gm] (src2: 0 one row source, 1 the block-output
// prologue, 2 the BN-backward prologue) -- tests and the fused ResNet path use it to see which
// kernel family a shape runs on (bm = bn = 256: conv_big.hip)
std::vector<int64_t> conv_gemm_plan(int64_t M, int64_t N, int64_t C, std::vector<int64_t> geo, bool pro, int64_t epi,
                                    int64_t src2) {
  TORCH_CHECK(geo.size() == 7, "geo = [H, W, OH, OW, ks, stride, pad]");
  const psamd::ConvGeo g{static_cast<int>(geo[0]), static_cast<int>(geo[1]), static_cast<int>(geo[2]),
                         static_cast<int>(geo[3]), static_cast<int>(C), static_cast<int>(geo[4]),
                         static_cast<int>(geo[5]), static_cast<int>(geo[6])};
  const int K = static_cast<int>(geo[4] * geo[4] * C);
  const auto pl = psamd::conv_fwd_plan_geo(static_cast<int>(M), static_cast<int>(N), K, pro, g, static_cast<int>(src2),
                                           static_cast<int>(epi));
  return {pl.bm, pl.bn, pl.gm};
}

// c [M, N] = epilogue(sum_k f(a[src(m, k)]) b[n, k]) -> [c, BN partials [2, G, N] (epi 1/3)]
std::vector<Tensor> conv_gemm(Tensor a, Tensor b, std::vector<int64_t> geo, c10::optional<Tensor> pro, int64_t epi,
                              c10::optional<Tensor> aux, c10::optional<Tensor> kshift, c10::optional<Tensor> mc,
                              c10::optional<Tensor> mean, c10::optional<Tensor> invstd, c10::optional<Tensor> bits,
                              c10::optional<Tensor> aux2, c10::optional<Tensor> bits2, c10::optional<Tensor> a2,
                              c10::optional<Tensor> bwd, c10::optional<Tensor> aux3, c10::optional<Tensor> mean2,
                              c10::optional<Tensor> invstd2, c10::optional<Tensor> pro2, c10::optional<Tensor> aout,
                              c10::optional<Tensor> abits, c10::optional<Tensor> tbuf) {
  check_rows(a, "a");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2, "a [rows, C], b [N, K]");
  const auto gi = conv_geo(a, geo);
  const psamd::ConvGeo g = gi.first;
  const int64_t N = b.size(0), K = b.size(1);
  TORCH_CHECK(K == static_cast<int64_t>(g.ks) * g.ks * g.C, "b must be [N, ks*ks*C]");
  TORCH_CHECK(N % 64 == 0 && N <= 8192, "N must be a multiple of 64, <= 8192");
  TORCH_CHECK(epi >= 0 && epi <= 9, "epi in 0..9");
  const int base = epi == 6 || epi == 9 ? 5 : epi == 7 ? 2 : epi == 8 ? 4 : static_cast<int>(epi);
  const bool fold = epi >= 6;
  const int64_t M = gi.second * g.OH * g.OW;
  TORCH_CHECK(M > 0 && M < (int64_t(1) << 31), "pixel count");
  const uint16_t* auxp = nullptr;
  if (epi >= 2) {
    TORCH_CHECK(aux.has_value() && aux->defined(), "epi ", epi, " needs aux");
    check_rows(*aux, "aux");
    const int64_t want = base == 4 ? gi.second * ((g.OH + 1) / 2) * ((g.OW + 1) / 2) * N : M * N;
    TORCH_CHECK(aux->numel() == want, "aux has ", aux->numel(), " elements, expected ", want);
    auxp = u16(*aux);
  }
  if (epi == 3) TORCH_CHECK(mc.has_value() && mean.has_value() && invstd.has_value(), "epi 3 needs mc, mean, invstd");
  const uint8_t* bitsp = nullptr;
  if (base == 5) {
    TORCH_CHECK(bits.has_value() && bits->defined(), "epi 5/6 needs bits");
    check_gpu(*bits, "bits");
    TORCH_CHECK(bits->scalar_type() == torch::kUInt8 && bits->numel() * 8 == M * N, "bits: uint8 [M * N / 8]");
    bitsp = bits->data_ptr<uint8_t>();
  }
  TORCH_CHECK(!(pro.has_value() && pro->defined()) || epi <= 1, "the BN prologue combines with epilogue 0 or 1 only");
  const bool has_bwd = bwd.has_value() && bwd->defined();
  if (has_bwd) {  // BN-backward prologue: A := ca * a + cb * a2 + cc, stored to a third output
    TORCH_CHECK(!(pro.has_value() && pro->defined()), "the BN-backward prologue excludes pro");
    TORCH_CHECK(epi == 3 || ((epi == 2 || epi >= 4) &&
                             psamd::conv_big_ok(static_cast<int>(gi.second * g.OH * g.OW), static_cast<int>(N),
                                                static_cast<int>(K), true, g, 2, static_cast<int>(epi))),
                "the BN-backward prologue combines with epi 3, or with 2 / 4-9 on the 256 x 256 tiles");
    TORCH_CHECK(g.ks == 1 && g.stride == 1 && g.pad == 0, "the BN-backward prologue is for 1x1 stride-1 convs");
    TORCH_CHECK(a2.has_value() && a2->defined(), "the BN-backward prologue needs a2");
    check_rows(*a2, "a2");
    TORCH_CHECK(a2->sizes() == a.sizes(), "a2 must match a");
    check_f32(*bwd, "bwd");
    TORCH_CHECK(bwd->numel() == 3 * g.C, "bwd must be [3C]");
  }
  // block-output prologue: A := relu(bn3(a) + r), r = a2 or the downsample BN of a2 (pro2); the
  // block output and its ReLU bits land in the caller's aout / abits
  const bool has_a2 = a2.has_value() && a2->defined();
  const bool resp = has_a2 && !has_bwd;
  if (resp) {
    TORCH_CHECK(pro.has_value() && pro->defined(), "a2 without bwd is the block-output prologue: needs pro");
    TORCH_CHECK(g.ks == 1 && g.stride == 1 && g.pad == 0, "the block-output prologue is for 1x1 stride-1 convs");
    check_rows(*a2, "a2");
    TORCH_CHECK(a2->sizes() == a.sizes(), "a2 must match a");
    TORCH_CHECK(aout.has_value() && aout->defined() && abits.has_value() && abits->defined(),
                "the block-output prologue needs aout and abits");
    check_rows(*aout, "aout");
    TORCH_CHECK(aout->sizes() == a.sizes(), "aout must match a");
    check_gpu(*abits, "abits");
    TORCH_CHECK(abits->scalar_type() == torch::kUInt8 && abits->is_contiguous() && abits->numel() * 8 == a.numel(),
                "abits: uint8 [rows * C / 8]");
  } else {
    TORCH_CHECK(!(pro2.has_value() && pro2->defined()) && !(aout.has_value() && aout->defined()),
                "pro2 / aout belong to the block-output prologue (pro + a2)");
  }
  const uint16_t* aux2p = nullptr;
  const uint8_t* bits2p = nullptr;
  if (fold) {
    TORCH_CHECK(aux2.has_value() && aux2->defined() && bits2.has_value() && bits2->defined() && mean.has_value() &&
                    invstd.has_value(),
                "epi ", epi, " needs aux2, bits2, mean, invstd");
    check_rows(*aux2, "aux2");
    TORCH_CHECK(aux2->numel() == M * N, "aux2 must be [M, N]");
    check_gpu(*bits2, "bits2");
    TORCH_CHECK(bits2->scalar_type() == torch::kUInt8 && bits2->numel() * 8 == M * N, "bits2: uint8 [M * N / 8]");
    aux2p = u16(*aux2);
    bits2p = bits2->data_ptr<uint8_t>();
  }
  const uint16_t* aux3p = nullptr;
  if (epi == 9) {
    TORCH_CHECK(aux3.has_value() && aux3->defined() && mean2.has_value() && invstd2.has_value(),
                "epi 9 needs aux3, mean2, invstd2");
    check_rows(*aux3, "aux3");
    TORCH_CHECK(aux3->numel() == M * N, "aux3 must be [M, N]");
    aux3p = u16(*aux3);
  }
  const c10::DeviceGuard guard(a.device());
  auto c = torch::empty({M, N}, a.options());
  auto fopt = a.options().dtype(torch::kFloat32);
  const bool has_pro = pro.has_value() && pro->defined();
  const int G = psamd::conv_fwd_plan_geo(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K),
                                        has_pro || has_bwd, g, resp ? 1 : has_bwd ? 2 : 0, static_cast<int>(epi)).gm;
  b = b.contiguous();  // b may be a strided view (e.g. a transposed weight)
  check_rows(b, "b");
  const bool sums = epi == 1 || epi == 3 || fold;
  TORCH_CHECK(epi != 9 || psamd::conv_fwd_plan_geo(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K),
                                                   has_pro || has_bwd, g, 0, static_cast<int>(epi)).bm >= 128,
              "epi 9 runs on the 128- or 256-pixel tiles");
  Tensor part = sums ? torch::empty({epi == 9 ? 3 : 2, G, N}, fopt) : Tensor();
  psamd::ConvGemmArgs p{};
  p.a = u16(a);
  p.b = u16(b);
  p.c = u16m(c);
  p.M = static_cast<int>(M);
  p.N = static_cast<int>(N);
  p.K = static_cast<int>(K);
  p.g = g;
  p.pro = f32_opt(pro, 2 * g.C, "pro");
  p.epi = static_cast<int>(epi);
  p.aux = auxp;
  p.bits = bitsp;
  p.aux2 = aux2p;
  p.bits2 = bits2p;
  p.kshift = f32_opt(kshift, N, "kshift");
  p.mc = f32_opt(mc, 2 * N, "mc");
  p.mean = f32_opt(mean, N, "mean");
  p.invstd = f32_opt(invstd, N, "invstd");
  p.part = sums ? part.data_ptr<float>() : nullptr;
  p.aux3 = aux3p;
  p.mean2 = epi == 9 ? f32_opt(mean2, N, "mean2") : nullptr;
  p.invstd2 = epi == 9 ? f32_opt(invstd2, N, "invstd2") : nullptr;
  Tensor bwd_out;
  if (has_bwd) {
    bwd_out = torch::empty_like(a);
    p.a2 = u16(*a2);
    p.bwd = bwd->data_ptr<float>();
    p.aout = u16m(bwd_out);
  }
  if (resp) {
    p.a2 = u16(*a2);
    p.pro2 = f32_opt(pro2, 2 * g.C, "pro2");
    p.aout = u16m(*aout);
    p.abits = abits->data_ptr<uint8_t>();
  }
  if (tbuf.has_value() && tbuf->defined()) {  // phase stamps of the 256 x 256-tile kernel (probes)
    check_gpu(*tbuf, "tbuf");
    TORCH_CHECK(tbuf->scalar_type() == torch::kInt64 && tbuf->is_contiguous(), "tbuf: int64");
    const auto pl = psamd::conv_fwd_plan_geo(p.M, p.N, p.K, has_pro || has_bwd, g, resp ? 1 : has_bwd ? 2 : 0, p.epi);
    TORCH_CHECK(pl.bm == 256 && tbuf->numel() >= int64_t(8) * pl.gm * (N / pl.bn), "tbuf: [8 x blocks] on the big tiles");
    p.tbuf = reinterpret_cast<uint64_t*>(tbuf->data_ptr<int64_t>());
  }
  if (g_route_on.load(std::memory_order_relaxed)) {
    const auto pl = psamd::conv_fwd_plan_geo(p.M, p.N, p.K, has_pro || has_bwd, g, resp ? 1 : has_bwd ? 2 : 0, p.epi);
    route((pl.bm == 256 && pl.bn == 256 ? std::string("conv_big") : "conv_fwd_" + std::to_string(pl.bm) + "x" +
                                                                          std::to_string(pl.bn)) +
          "/k" + std::to_string(g.ks) + (g.stride == 2 ? "s2" : "") + (has_pro ? "/pro" : "") + (has_bwd ? "/bnbwd" : "") +
          (resp ? "/blockout" : "") + "/epi" + std::to_string(epi));
  }
  psamd::launch_conv_fwd(p, cur_stream(a));
  if (has_bwd) return {c, part, bwd_out};
  return {c, part};
}

// Data gradient of a 3x3 / stride-2 / pad-1 convolution as four stride-1 phase GEMMs over dz:
// input pixel (2i + a, 2j + b) gathers dz rows i (+1) with the taps kh = 1 (a = 0) or kh = 2, 0
// (a = 1) -- likewise for the width -- so phase (a, b) is a 1x1 / 1x2 / 2x1 / 2x2 "convolution"
// over the dz map whose epilogue writes every other row of dx.  Every dx pixel is written by
// exactly one phase (H, W even): no zero fill, no scatter-add.  epi 3 (z1, mc, mean, invstd):
// ReLU mask of the BN that produced the conv input + its backward sums; partials of the four
// phases are concatenated along the partial-row axis.
//   dz [n*OH*OW, C2], wph: 4 weights [C1, nh*nw*C2] in phase order (0,0) (0,1) (1,0) (1,1)
std::vector<Tensor> conv_dgrad_s2(Tensor dz, std::vector<Tensor> wph, int64_t H, int64_t W, int64_t epi,
                                  c10::optional<Tensor> z, c10::optional<Tensor> mc, c10::optional<Tensor> mean,
                                  c10::optional<Tensor> invstd) {
  check_rows(dz, "dz");
  TORCH_CHECK(H % 2 == 0 && W % 2 == 0 && H > 0 && W > 0, "stride-2 phases need an even input map");
  TORCH_CHECK(wph.size() == 4, "four phase weights");
  TORCH_CHECK(epi == 0 || epi == 3, "epi 0 or 3");
  const int64_t OH = H / 2, OW = W / 2, C2 = dz.size(1);
  TORCH_CHECK(C2 % 64 == 0 && dz.size(0) % (OH * OW) == 0, "dz must be [images*OH*OW, C2], C2 % 64 == 0");
  const int64_t imgs = dz.size(0) / (OH * OW), M = imgs * OH * OW, C1 = wph[0].size(0);
  TORCH_CHECK(C1 % 64 == 0 && C1 <= 8192 && imgs * H * W < (int64_t(1) << 31), "C1 / size");
  const uint16_t* zp = nullptr;
  if (epi == 3) {
    TORCH_CHECK(z.has_value() && z->defined() && mc.has_value() && mean.has_value() && invstd.has_value(),
                "epi 3 needs z, mc, mean, invstd");
    check_rows(*z, "z");
    TORCH_CHECK(z->numel() == imgs * H * W * C1, "z must be [images*H*W, C1]");
    zp = u16(*z);
  }
  const c10::DeviceGuard guard(dz.device());
  auto dx = torch::empty({imgs * H * W, C1}, dz.options());
  // the four phases in one grid (csrc convgemm.hip conv_dgrad_phases_kernel)
  {
    std::vector<Tensor> ws;  // (temporary contiguous weights are freed stream-ordered)
    ws.reserve(4);
    psamd::ConvGemmArgs ps[4] = {};
    const int gm = psamd::conv_dgrad_phase_gm(static_cast<int>(M));
    Tensor part = epi == 3 ? torch::empty({2, 4 * gm, C1}, dz.options().dtype(torch::kFloat32)) : Tensor();
    for (int ph = 0; ph < 4; ++ph) {
      const int a = ph >> 1, b = ph & 1, nh = a ? 2 : 1, nw = b ? 2 : 1;
      ws.push_back(wph[ph].contiguous());
      const Tensor& w = ws.back();
      check_rows(w, "phase weight");
      TORCH_CHECK(w.dim() == 2 && w.size(0) == C1 && w.size(1) == nh * nw * C2, "phase weight [C1, nh*nw*C2]");
      psamd::ConvGemmArgs& p = ps[ph];
      p.a = u16(dz);
      p.b = u16(w);
      p.c = u16m(dx);
      p.M = static_cast<int>(M);
      p.N = static_cast<int>(C1);
      p.K = static_cast<int>(nh * nw * C2);
      p.g = psamd::ConvGeo{static_cast<int>(OH), static_cast<int>(OW), static_cast<int>(OH), static_cast<int>(OW),
                           static_cast<int>(C2), nh, 1, 0, nw, static_cast<int>(H), static_cast<int>(W), a, b};
      p.epi = static_cast<int>(epi);
      if (epi == 3) {
        p.aux = zp;
        p.mc = f32_opt(mc, 2 * C1, "mc");
        p.mean = f32_opt(mean, C1, "mean");
        p.invstd = f32_opt(invstd, C1, "invstd");
        p.part = part.data_ptr<float>() + static_cast<int64_t>(ph) * gm * C1;  // rows [ph gm, (ph + 1) gm)
        p.pgm = 4 * gm;
      }
    }
    route("conv_dgrad_phases/epi" + std::to_string(epi));
    psamd::launch_conv_dgrad_phases(ps, cur_stream(dz));
    return {dx, part};
  }
}

// dW [N, ks*ks*C] (bf16) = sum_m dz[m, :]^T f(x[src(m, k)])
Tensor conv_wgrad(Tensor dz, Tensor x, std::vector<int64_t> geo, c10::optional<Tensor> pro) {
  check_rows(dz, "dz");
  check_rows(x, "x");
  TORCH_CHECK(dz.dim() == 2 && x.dim() == 2, "dz [M, N], x [rows, C]");
  const auto gi = conv_geo(x, geo);
  const psamd::ConvGeo g = gi.first;
  const int64_t M = dz.size(0), N = dz.size(1), K = static_cast<int64_t>(g.ks) * g.ks * g.C;
  TORCH_CHECK(M == gi.second * g.OH * g.OW, "dz rows must be images * OH * OW");
  TORCH_CHECK(N % 64 == 0 && N <= 8192, "N must be a multiple of 64, <= 8192");
  const c10::DeviceGuard guard(dz.device());
  const float* prop = f32_opt(pro, 2 * g.C, "pro");
  auto ws = torch::empty({psamd::conv_wgrad_ws_geo(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), g,
                                                   prop != nullptr)},
                         dz.options().dtype(torch::kFloat32));
  auto dw = torch::empty({N, K}, dz.options());
  psamd::ConvWgradArgs p{};
  p.dz = u16(dz);
  p.x = u16(x);
  p.M = static_cast<int>(M);
  p.N = static_cast<int>(N);
  p.K = static_cast<int>(K);
  p.g = g;
  p.pro = prop;
  p.ws = ws.data_ptr<float>();
  p.dw = u16m(dw);
  if (g_route_on.load(std::memory_order_relaxed))
    route("conv_wgrad/k" + std::to_string(g.ks) + (g.stride == 2 ? "s2" : "") + (prop != nullptr ? "/pro" : ""));
  psamd::launch_conv_wgrad(p, cur_stream(dz));
  return dw;
}

// conv3's backward in one pass (csrc/kernels/conv_bwd_fused.hip): bn3's backward prologue
// dz3 = bf16(ca g + cb z3 + cc) never leaves LDS; -> [gy [M, CI] (masked by bn2's ReLU), part
// [2, G, CI] (bn2 backward sums, the conv_gemm epi-3 layout), dW3 [CO, CI] bf16]
std::vector<Tensor> conv11_bwd_fused(Tensor g, Tensor z3, Tensor cbwd, Tensor wt, Tensor z2, c10::optional<Tensor> cf2,
                                     c10::optional<Tensor> mean2, c10::optional<Tensor> invstd2) {
  check_rows(g, "g");
  check_rows(z3, "z3");
  check_rows(z2, "z2");
  check_rows(wt, "wt");
  TORCH_CHECK(g.dim() == 2 && z3.sizes() == g.sizes() && z2.dim() == 2 && z2.size(0) == g.size(0),
              "g, z3 [M, CO]; z2 [M, CI]");
  const int64_t M = g.size(0), CO = g.size(1), CI = z2.size(1);
  // no bn2 parameters: the PLAIN (downsample) pass -- z2 is the weight gradient's operand as is and
  // the data gradient leaves unmasked, with no partial sums
  const bool plain = !cf2.has_value();
  TORCH_CHECK(plain == !mean2.has_value() && plain == !invstd2.has_value(), "cf2, mean2, invstd2: all or none");
  TORCH_CHECK(plain ? psamd::conv11_bwd_plain_ok(static_cast<int>(CI), static_cast<int>(CO))
                    : psamd::conv11_bwd_built(static_cast<int>(CI), static_cast<int>(CO)),
              "conv11_bwd_fused: unsupported channels CI=", CI, " CO=", CO, plain ? " (plain)" : "");
  TORCH_CHECK(M > 0 && M < (int64_t(1) << 31) / CO, "pixel count");
  TORCH_CHECK(wt.dim() == 2 && wt.size(0) == CI && wt.size(1) == CO, "wt must be [CI, CO]");
  check_f32(cbwd, "cbwd");
  TORCH_CHECK(cbwd.numel() == 3 * CO, "cbwd [3 CO]");
  if (!plain) {
    check_f32(*cf2, "cf2");
    check_f32(*mean2, "mean2");
    check_f32(*invstd2, "invstd2");
    TORCH_CHECK(cf2->numel() == 2 * CI && mean2->numel() == CI && invstd2->numel() == CI,
                "cf2 [2 CI], mean2 / invstd2 [CI]");
  }
  const c10::DeviceGuard guard(g.device());
  const int m = static_cast<int>(M), ci = static_cast<int>(CI), co = static_cast<int>(CO);
  const int G = psamd::conv11_bwd_blocks(m, ci, co);
  auto gy = torch::empty({M, CI}, g.options());
  auto part = torch::empty({plain ? 0 : 2, G, CI}, g.options().dtype(torch::kFloat32));
  auto ws = torch::empty({psamd::conv11_bwd_ws(m, ci, co)}, g.options().dtype(torch::kFloat32));
  auto dw = torch::empty({CO, CI}, g.options());
  psamd::Conv11BwdArgs a{};
  a.g = u16(g);
  a.z3 = u16(z3);
  a.cbwd = cbwd.data_ptr<float>();
  a.wt = u16(wt);
  a.z2 = u16(z2);
  a.cf2 = plain ? nullptr : cf2->data_ptr<float>();
  a.mean2 = plain ? nullptr : mean2->data_ptr<float>();
  a.invstd2 = plain ? nullptr : invstd2->data_ptr<float>();
  a.gy = u16m(gy);
  a.part = plain ? nullptr : part.data_ptr<float>();
  a.ws = ws.data_ptr<float>();
  a.dw = u16m(dw);
  a.M = m;
  route(std::string("conv11_bwd_fused/") + (plain ? "plain" : "bn2") + "/" + std::to_string(ci) + "x" +
        std::to_string(co));
  psamd::launch_conv11_bwd_fused(a, ci, co, cur_stream(g));
  return {gy, part, dw};
}

bool conv11_bwd_fused_supported(int64_t ci, int64_t co, bool plain) {
  return plain ? psamd::conv11_bwd_plain_ok(static_cast<int>(ci), static_cast<int>(co))
               : psamd::conv11_bwd_fused_ok(static_cast<int>(ci), static_cast<int>(co));
}

// Linear weight + bias gradient in one pass over dz: [dW [N, K] bf16, db [N] fp32] with
// dW = dz^T x (x [M, K] rows), db = column sums of dz (fused into the wide split-K kernel; a
// torch reduction where the plan is not wide)
std::vector<Tensor> linear_wgrad_db(Tensor dz, Tensor x) {
  check_rows(dz, "dz");
  check_rows(x, "x");
  TORCH_CHECK(dz.dim() == 2 && x.dim() == 2 && dz.size(0) == x.size(0), "dz [M, N], x [M, K]");
  const int64_t M = dz.size(0), N = dz.size(1), K = x.size(1);
  TORCH_CHECK(N % 64 == 0 && N <= 8192 && K % 64 == 0 && M < (int64_t(1) << 31), "N, K multiples of 64");
  const int m = static_cast<int>(M), n = static_cast<int>(N), k = static_cast<int>(K);
  const c10::DeviceGuard guard(dz.device());
  const bool wide = psamd::conv_wgrad_is_wide(m, n, k, k, false);
  const int64_t wsz = psamd::conv_wgrad_ws(m, n, k, k, false);
  const int64_t dbsz = wide ? static_cast<int64_t>(psamd::conv_wgrad_splits(m, n, k, k, false)) * N : 0;
  auto ws = torch::empty({wsz + dbsz}, dz.options().dtype(torch::kFloat32));
  auto dw = torch::empty({N, K}, dz.options());
  auto db = wide ? torch::empty({N}, dz.options().dtype(torch::kFloat32)) : dz.sum(0, false, torch::kFloat32);
  psamd::ConvWgradArgs p{};
  p.dz = u16(dz);
  p.x = u16(x);
  p.M = m;
  p.N = n;
  p.K = k;
  p.g = psamd::ConvGeo{m, 1, m, 1, k, 1, 1, 0};
  p.pro = nullptr;
  p.ws = ws.data_ptr<float>();
  p.dw = u16m(dw);
  p.db = wide ? db.data_ptr<float>() : nullptr;
  p.dbws = wide ? ws.data_ptr<float>() + wsz : nullptr;
  psamd::launch_conv_wgrad(p, cur_stream(dz));
  return {dw, db};
}

// y = act(x * scale + shift [+ res [* rscale + rshift]]) from precomputed coefficients [scale | shift]
// -> [y, ReLU mask bits (uint8 [R*C/8], with want_mask) or empty]
std::vector<Tensor> bn_apply_coef(Tensor x, Tensor coef, c10::optional<Tensor> res, c10::optional<Tensor> rcoef,
                                  int64_t act, bool want_mask) {
  check_rows(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 8 == 0, "x [R, C], C % 8");
  const int64_t R = x.size(0), C = x.size(1);
  check_f32(coef, "coef");
  TORCH_CHECK(coef.numel() == 2 * C, "coef = [scale | shift]");
  const bool hr = res.has_value() && res->defined();
  if (hr) {
    check_rows(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes(), "res like x");
  }
  const float* rc = f32_opt(rcoef, 2 * C, "rcoef");
  TORCH_CHECK(!rc || hr, "rcoef needs res");
  const c10::DeviceGuard guard(x.device());
  auto y = torch::empty_like(x);
  Tensor mb = want_mask ? torch::empty({R * C / 8}, x.options().dtype(torch::kUInt8)) : Tensor();
  psamd::launch_bn_apply_coef(u16(x), hr ? u16(*res) : nullptr, coef.data_ptr<float>(), rc, u16m(y),
                              want_mask ? mb.data_ptr<uint8_t>() : nullptr, R, static_cast<int>(C),
                              static_cast<int>(act), cur_stream(x));
  return {y, mb};
}

// Backward weight layouts (convgemm.hip weight_prep): jobs = int64 [J, 4] on the device, rows
// {src ptr, dst ptr, kind | A << 32, B} (the WPrepJob layout) -- built once per weight set and reused
// max_blocks: the largest (taps x 64-tiles) count over the jobs (one block per transposed tile)
void weight_prep(Tensor jobs, int64_t max_blocks) {
  check_gpu(jobs, "jobs");
  TORCH_CHECK(jobs.scalar_type() == torch::kInt64 && jobs.dim() == 2 && jobs.size(1) == 4 && jobs.is_contiguous(),
              "jobs: int64 [J, 4]");
  static_assert(sizeof(void*) == 8, "64-bit pointers");
  const c10::DeviceGuard guard(jobs.device());
  TORCH_CHECK(max_blocks > 0 && max_blocks < (1 << 20), "max_blocks");
  psamd::launch_weight_prep(jobs.data_ptr(), static_cast<int>(jobs.size(0)), static_cast<int>(max_blocks),
                            cur_stream(jobs));
}

// BN backward coefficients only (dx = ca * g + cb * x + cc for a GEMM prologue to apply) from
// producer partial sums part [2, G, C] over R rows -> [dgamma, dbeta, coef = ca | cb | cc]
std::vector<Tensor> bn_bwd_coef(Tensor part, c10::optional<Tensor> gamma, Tensor mean, Tensor invstd, int64_t R) {
  check_part_slabs(part);
  const int64_t C = part.size(2);
  TORCH_CHECK(C % 8 == 0, "C % 8");
  const c10::DeviceGuard guard(part.device());
  auto fopt = part.options();
  auto dg = torch::empty({C}, fopt), db = torch::empty({C}, fopt), coef = torch::empty({3 * C}, fopt);
  const Tensor fp = fold_partials(part, cur_stream(part));
  const int64_t Gf = fp.size(1);
  psamd::launch_bn_bwd_partials(fp.data_ptr<float>(), fp.data_ptr<float>() + fp.stride(0), static_cast<int>(Gf), nullptr,
                                nullptr, f32_opt(gamma, C, "gamma"), f32_opt(mean, C, "mean"), f32_opt(invstd, C, "invstd"),
                                dg.data_ptr<float>(), db.data_ptr<float>(), coef.data_ptr<float>(), nullptr, R,
                                static_cast<int>(C), cur_stream(part));
  return {dg, db, coef};
}

// BN backward from producer partial sums part [2, G, C] (conv_gemm epi 3); g = masked gradient
std::vector<Tensor> bn_bwd_partials(Tensor g, Tensor x, Tensor part, c10::optional<Tensor> gamma, Tensor mean,
                                    Tensor invstd) {
  check_rows(g, "g");
  check_rows(x, "x");
  TORCH_CHECK(x.dim() == 2 && g.sizes() == x.sizes() && x.size(1) % 8 == 0, "g/x [R, C], C % 8");
  const int64_t R = x.size(0), C = x.size(1);
  check_part_slabs(part);
  TORCH_CHECK(part.size(2) == C, "part [2, G, C]");
  const c10::DeviceGuard guard(x.device());
  auto fopt = x.options().dtype(torch::kFloat32);
  auto dx = torch::empty_like(x);
  auto dg = torch::empty({C}, fopt), db = torch::empty({C}, fopt), coef = torch::empty({3 * C}, fopt);
  const Tensor fp = fold_partials(part, cur_stream(x));
  const int64_t Gf = fp.size(1);
  psamd::launch_bn_bwd_partials(fp.data_ptr<float>(), fp.data_ptr<float>() + fp.stride(0), static_cast<int>(Gf), u16(g), u16(x),
                                f32_opt(gamma, C, "gamma"), f32_opt(mean, C, "mean"), f32_opt(invstd, C, "invstd"),
                                dg.data_ptr<float>(), db.data_ptr<float>(), coef.data_ptr<float>(), u16m(dx), R,
                                static_cast<int>(C), cur_stream(x));
  return {dx, dg, db};
}

}  // namespace

void register_async_ps(pybind11::module& m);  // csrc/async_ps_gpu.cpp
void register_plane(pybind11::module& m);      // csrc/plane.cpp
void register_async_rows(pybind11::module& m); // csrc/async_rows_gpu.cpp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "ps_amd HIP kernels for MI355X (gfx950)";
  register_async_ps(m);
  register_plane(m);
  register_async_rows(m);
  m.def("conv_gemm", &conv_gemm, py::arg("a"), py::arg("b"), py::arg("geo"), py::arg("pro") = py::none(),
        py::arg("epi") = 0, py::arg("aux") = py::none(), py::arg("kshift") = py::none(), py::arg("mc") = py::none(),
        py::arg("mean") = py::none(), py::arg("invstd") = py::none(), py::arg("bits") = py::none(),
        py::arg("aux2") = py::none(), py::arg("bits2") = py::none(), py::arg("a2") = py::none(),
        py::arg("bwd") = py::none(), py::arg("aux3") = py::none(), py::arg("mean2") = py::none(),
        py::arg("invstd2") = py::none(), py::arg("pro2") = py::none(), py::arg("aout") = py::none(),
        py::arg("abits") = py::none(), py::arg("tbuf") = py::none());
  m.def("route_log", &route_log, py::arg("enable") = true, py::arg("reset") = true);
  m.def("linear_wgrad_db", &linear_wgrad_db);
  m.def("bn_bwd_coef", &bn_bwd_coef);
  m.def("weight_prep", &weight_prep, py::arg("jobs"), py::arg("max_blocks") = 1024);
  m.def("conv_dgrad_s2", &conv_dgrad_s2, py::arg("dz"), py::arg("wph"), py::arg("H"), py::arg("W"),
        py::arg("epi") = 0, py::arg("z") = py::none(), py::arg("mc") = py::none(), py::arg("mean") = py::none(),
        py::arg("invstd") = py::none());
  m.def("conv_wgrad", &conv_wgrad, py::arg("dz"), py::arg("x"), py::arg("geo"), py::arg("pro") = py::none());
  m.def("conv_gemm_plan", &conv_gemm_plan, py::arg("M"), py::arg("N"), py::arg("C"), py::arg("geo"),
        py::arg("pro") = false, py::arg("epi") = 0, py::arg("src2") = 0);
  m.def("conv11_bwd_fused", &conv11_bwd_fused, py::arg("g"), py::arg("z3"), py::arg("cbwd"), py::arg("wt"), py::arg("z2"),
        py::arg("cf2") = py::none(), py::arg("mean2") = py::none(), py::arg("invstd2") = py::none());
  m.def("conv11_bwd_fused_supported", &conv11_bwd_fused_supported, py::arg("ci"), py::arg("co"),
        py::arg("plain") = false);
  m.def("bn_apply_coef", &bn_apply_coef, py::arg("x"), py::arg("coef"), py::arg("res") = py::none(),
        py::arg("rcoef") = py::none(), py::arg("act") = 1, py::arg("want_mask") = false);
  m.def("bn_bwd_partials", &bn_bwd_partials);
  m.def("fused_opt", &fused_opt);
  m.def("sparse_opt", &sparse_opt, py::arg("kind"), py::arg("table"), py::arg("st0"), py::arg("st1"),
        py::arg("rows"), py::arg("grad"), py::arg("rowwise"), py::arg("skip_zero"), py::arg("lr"), py::arg("beta1"),
        py::arg("beta2"), py::arg("eps"), py::arg("wd"), py::arg("momentum"), py::arg("dampening"),
        py::arg("nesterov"), py::arg("adamw"), py::arg("bc1"), py::arg("bc2"), py::arg("l1"), py::arg("l2"),
        py::arg("fbeta"), py::arg("ftrl_mode"), py::arg("gscale"), py::arg("perm") = py::none(), py::arg("ncount") = py::none());
  m.def("sumsq", &sumsq);
  m.def("clip_factor", &clip_factor);
  m.def("cast_", &cast_);
  m.def("axpy_", &axpy_);
  m.def("reduce_n", &reduce_n);
  m.def("lerp", &lerp);
  m.def("onebit_pack", &onebit_pack, py::arg("g"), py::arg("err"), py::arg("words"), py::arg("scales"),
        py::arg("mom") = py::none(), py::arg("beta1") = 0.0);
  m.def("onebit_momentum", &onebit_momentum);
  m.def("onebit_unpack_reduce", &onebit_unpack_reduce);
  m.def("gather_rows", &gather_rows);
  m.def("segment_reduce_rows", &segment_reduce_rows);
  m.def("scatter_add_rows", &scatter_add_rows);
  m.def("embedding_bag_fwd", &embedding_bag_fwd);
  m.def("sparse_lr_fwd", &sparse_lr_fwd);
  m.def("lazy_init_rows", &lazy_init_rows, py::arg("table"), py::arg("rows"), py::arg("flags"), py::arg("seed"),
        py::arg("row_base"), py::arg("lo"), py::arg("hi"), py::arg("keys") = py::none());
  m.def("hash_slots", &hash_slots);
  m.def("unique_runs", &unique_runs);
  m.def("softmax_temp_fwd", &softmax_temp_fwd);
  m.def("softmax_temp_bwd", &softmax_temp_bwd);
  m.def("softmax_xent", &softmax_xent);
  m.def("bce", &bce);
  m.def("maxpool2d_fwd", &maxpool2d_fwd);
  m.def("maxpool2d_bwd", &maxpool2d_bwd);
  m.def("im2col", &im2col);
  m.def("col2im", &col2im);
  m.def("dropout", &dropout);
  m.def("uniform_init", &uniform_init);
  m.def("gemm_nt", &gemm_nt);
  m.def("fc_bwd", &fc_bwd, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("w"), py::arg("dw") = py::none(),
        py::arg("db") = py::none(), py::arg("dx") = py::none(), py::arg("act") = 0);
  m.def("fc_fwd_f32", &fc_fwd_f32);
  m.def("act_bwd", &act_bwd);
  m.def("bn_act_fwd", &bn_act_fwd);
  m.def("bn_stats", &bn_stats);
  m.def("maxpool_nhwc_fwd", &maxpool_nhwc_fwd);
  m.def("stem_conv_fwd", &stem_conv_fwd, py::arg("x"), py::arg("wp"), py::arg("kshift") = py::none());
  m.def("bn_finalize_sums", &bn_finalize_sums);
  m.def("stem_conv_wrw", &stem_conv_wrw);
  m.def("stem_bwd_fused", &stem_bwd_fused);
  m.def("dlrm_interact_fwd", &dlrm_interact_fwd);
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("layernorm_bwd", &layernorm_bwd);
  m.def("attn_fwd", &attn_fwd);
  m.def("xent_fwd", &xent_fwd, py::arg("x"), py::arg("labels"), py::arg("ignore_index"));
  m.def("xent_bwd", &xent_bwd, py::arg("x"), py::arg("labels"), py::arg("lse"), py::arg("go"), py::arg("count"),
        py::arg("ignore_index"));
  m.def("fa_fwd", &fa_fwd);
  m.def("fa_bwd", &fa_bwd);
  m.def("attn_bwd", &attn_bwd);
  m.def("attn_dropout_mask", &attn_dropout_mask);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("rope_split_fwd", &rope_split_fwd);
  m.def("rope_split_bwd", &rope_split_bwd);
  m.def("dlrm_interact_bwd", &dlrm_interact_bwd);
  m.def("maxpool_nhwc_bwd", &maxpool_nhwc_bwd);
  m.def("pool_bn_bwd", &pool_bn_bwd);
  m.def("row_plane_recv", &row_plane_recv);
  m.def("row_plane_send", &row_plane_send);
  m.def("row_plane_accum", &row_plane_accum);
  m.def("bn_act_bwd", &bn_act_bwd, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("gamma"), py::arg("mean"),
        py::arg("invstd"), py::arg("act"), py::arg("want_dres"), py::arg("affine"),
        py::arg("mask_coef") = py::none(), py::arg("mbits") = py::none());
  m.attr("ONEBIT_CHUNK") = psamd::kOnebitChunk;
  m.attr("ARCH") = "gfx950";
}
