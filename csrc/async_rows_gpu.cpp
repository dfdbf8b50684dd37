// GPU owner service of the asynchronous sparse-row tables (ps_amd/parallel/async_rows.py).
//
// Reference: an async PServer applies every row push the moment it arrives
// (net/PServer.java:164-184) and serves row pulls from its store (net/PServer.java:101-117,
// 143-162, lazily creating rows).  Here each owner runs ONE native thread that polls the table's
// shared-memory control words (the RowPoller layout of csrc/runtime/bindings_native.cpp: req /
// resp / nreq / pseq / pack per (owner, worker)) and does the owner's row work itself, on its
// own HIP stream, straight out of its device mailboxes:
//   pull  keys rq[w][0 : n] (n = the word after the mailbox's cap entries, written by the worker's
//         copy kernel) -> slots (device hash map, CAS insert; or key - row_base) -> deterministic
//         lazy init keyed by the global key -> rows gathered into the response mailbox rs[w];
//   push  keys + summed gradient rows of mailbox slot m -> slots -> the HIP row optimizer
//         (gradient / W, bias correction per applied push) -> pack[me][w]++.
// No Python, no GIL: the training thread of the same process never contends with it, and the
// workers' keys, rows and gradients never leave device memory (the worker side moves them with
// the segment kernels of csrc/kernels/sparse.hip).  The one host read per request is the count
// word, by this thread (its own stream, synchronised before it answers).
#include <torch/extension.h>

#include <ATen/hip/HIPContext.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>

#include "async_ctl.h"
#include "psamd_launch.h"

namespace {

using torch::Tensor;

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

class GpuRowService {
 public:
  GpuRowService(uintptr_t ctl, int64_t me, int64_t cap, int64_t dim)
      : b_(reinterpret_cast<int64_t*>(ctl)), me_(static_cast<int>(me)), cap_(cap), dim_(static_cast<int>(dim)) {
    W_ = b_[1];
    TORCH_CHECK(W_ >= 1 && me >= 0 && me < W_, "row service rank");
    // pinned landing words for the request count and the status word: a D2H copy into pageable
    // memory is staged and synchronous (~2x the cost of the whole small request)
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&pinned_), 2 * sizeof(int64_t), hipHostMallocDefault), "pinned words");
  }
  ~GpuRowService() {
    stop();
    if (pinned_ != nullptr) (void)hipHostFree(pinned_);
  }

  // this owner's mailboxes: rq [W, cap + 1] int64, rs [W, cap, dim] f32, pk [W, MB, cap + 1]
  // int64, pg [W, MB, cap, dim] f32 (the word after cap entries = the count)
  void set_mailboxes(Tensor rq, Tensor rs, Tensor pk, Tensor pg) {
    for (const Tensor* t : {&rq, &rs, &pk, &pg}) TORCH_CHECK(t->is_cuda() && t->is_contiguous(), "device mailboxes");
    TORCH_CHECK(rq.scalar_type() == torch::kInt64 && rq.numel() == W_ * (cap_ + 1), "rq [W, cap + 1]");
    TORCH_CHECK(rs.scalar_type() == torch::kFloat32 && rs.numel() == W_ * cap_ * dim_, "rs [W, cap, dim]");
    TORCH_CHECK(pk.scalar_type() == torch::kInt64 && pk.numel() == W_ * psasync::kMbox * (cap_ + 1), "pk");
    TORCH_CHECK(pg.scalar_type() == torch::kFloat32 && pg.numel() == W_ * psasync::kMbox * cap_ * dim_, "pg");
    rq_ = rq;
    rs_ = rs;
    pk_ = pk;
    pg_ = pg;
    dev_ = rq.device().index();
    slots_ = torch::empty({cap_}, rq.options());
  }

  // the shard: fp32 table, init flags, hash keys (map mode; undefined = range partition with
  // row_base), overflow status, optimizer states
  void set_shard(Tensor table, Tensor flags, c10::optional<Tensor> hkeys, int64_t row_base, Tensor status,
                 c10::optional<Tensor> st0, c10::optional<Tensor> st1, int64_t seed, double lo, double hi) {
    TORCH_CHECK(!running(), "row service: set_shard while the service thread runs (stop() first)");
    TORCH_CHECK(table.is_cuda() && table.scalar_type() == torch::kFloat32 && table.dim() == 2 &&
                    table.size(1) == dim_ && table.is_contiguous(), "table [rows, dim] fp32");
    table_ = table;
    flags_ = flags;
    if (hkeys.has_value() && hkeys->defined()) hkeys_ = *hkeys;
    row_base_ = row_base;
    status_ = status;
    if (st0.has_value() && st0->defined()) st0_ = *st0;
    if (st1.has_value() && st1->defined()) st1_ = *st1;
    seed_ = static_cast<uint64_t>(seed);
    lo_ = static_cast<float>(lo);
    hi_ = static_cast<float>(hi);
  }

  // row updater: kernel kind, the 16 hyper-parameters (ps_amd/parallel/plane.py order), bias
  // mode (0 none, 1 1 - beta^t per applied push, 2 constant), row-wise accumulator, FTRL skip
  void set_updater(int64_t kind, std::vector<double> h, int64_t bias_mode, bool rowwise, bool skip_zero,
                   double gscale) {
    // The hyper-parameters are a snapshot: the thread copies a_ per push without a lock, so
    // they may only change while it is stopped (AsyncRowTable.set_updater stops and restarts
    // the service around a reconfiguration).
    TORCH_CHECK(!running(), "row service: set_updater while the service thread runs (stop() first)");
    TORCH_CHECK(h.size() == 16, "16 hyper-parameters");
    a_ = psamd::SparseOptArgs{};
    a_.kind = static_cast<int>(kind);
    a_.lr = h[0]; a_.beta1 = h[1]; a_.beta2 = h[2]; a_.eps = h[3]; a_.wd = h[4]; a_.momentum = h[5];
    a_.dampening = h[6]; a_.nesterov = h[7] != 0.0; a_.adamw = h[8] != 0.0; a_.bc1 = h[9]; a_.bc2 = h[10];
    a_.l1 = h[11]; a_.l2 = h[12]; a_.fbeta = h[13]; a_.ftrl_mode = static_cast<int>(h[14]);
    a_.gscale = static_cast<float>(h[15] * gscale);
    a_.rowwise = rowwise ? 1 : 0;
    a_.skip_zero = skip_zero ? 1 : 0;
    bias_mode_ = static_cast<int>(bias_mode);
    has_updater_.store(true, std::memory_order_release);  // after a_: the service thread reads it first
  }

  bool running() const { return th_.joinable(); }

  void start() {
    TORCH_CHECK(!running(), "row service already running");
    TORCH_CHECK(rq_.defined() && table_.defined(), "row service: mailboxes and shard first");
    stop_ = false;
    th_ = std::thread([this] { run(); });
  }
  void stop() {
    stop_ = true;
    if (th_.joinable()) th_.join();
  }
  std::string error() {
    std::lock_guard<std::mutex> g(mu_);
    return err_;
  }
  int64_t applied() const { return applied_.load(); }
  void set_applied(int64_t n) { applied_.store(n); }
  int64_t served() const { return served_.load(); }

 private:
  int64_t* w(int k, int64_t o, int64_t wk) const { return b_ + 4 + k * W_ * W_ + o * W_ + wk; }

  int64_t count_at(const int64_t* word, hipStream_t s) {
    psamd::launch_system_acquire(s);  // the mailbox was written by a peer's kernel
    hip_ok(hipMemcpyAsync(pinned_, word, sizeof(int64_t), hipMemcpyDeviceToHost, s), "count read");
    hip_ok(hipStreamSynchronize(s), "count read");
    const int64_t n = *reinterpret_cast<volatile int64_t*>(pinned_);
    TORCH_CHECK(n >= 0 && n <= cap_, "row service: bad request count ", n);
    return n;
  }

  // The owner's device hash map reports a full map (an insert that found no slot: its pull
  // would return zero rows, its push would be dropped) in the shard's status word; the Python
  // service checked it after every request (SparseShard.check), so this thread does too: the
  // 4-byte read rides the synchronisation every request already ends with.
  void check_status(hipStream_t s) {
    if (!hkeys_.defined() || !status_.defined()) return;
    int32_t* word = reinterpret_cast<int32_t*>(pinned_ + 1);
    hip_ok(hipMemcpyAsync(word, status_.data_ptr<int32_t>(), sizeof(int32_t), hipMemcpyDeviceToHost, s), "status read");
    hip_ok(hipStreamSynchronize(s), "status read");
    TORCH_CHECK(*reinterpret_cast<volatile int32_t*>(word) == 0, "sparse table shard full (device hash map of owner ",
                me_, ": ", hkeys_.numel(), " slots)");
  }

  void slots_of(const int64_t* keys, int64_t n, hipStream_t s) {
    int64_t* sl = slots_.data_ptr<int64_t>();
    if (hkeys_.defined())
      psamd::launch_hash_slots(hkeys_.data_ptr<int64_t>(), hkeys_.numel(), keys, n, sl, 1, status_.data_ptr<int32_t>(),
                               s);
    else
      psamd::launch_keys_to_rows(keys, n, row_base_, sl, s);
  }

  void serve_pull(int64_t k, hipStream_t s) {
    const int64_t* keys = rq_.data_ptr<int64_t>() + k * (cap_ + 1);
    const int64_t n = count_at(keys + cap_, s);
    if (n == 0) return;
    slots_of(keys, n, s);
    const int64_t* sl = slots_.data_ptr<int64_t>();
    if (lo_ != 0.f || hi_ != 0.f)
      psamd::launch_lazy_init_rows(table_.data_ptr<float>(), sl, keys, n, dim_, flags_.data_ptr<uint8_t>(), seed_, 0,
                                   lo_, hi_, s);
    psamd::launch_gather_rows(table_.data_ptr<float>(), 0, sl, n, dim_, rs_.data_ptr<float>() + k * cap_ * dim_, 0,
                              dim_, 0, 0, s);
    check_status(s);  // synchronises the stream
  }

  void serve_push(int64_t k, int m, hipStream_t s) {
    TORCH_CHECK(has_updater_.load(std::memory_order_acquire), "row table has no updater");
    const int64_t* keys = pk_.data_ptr<int64_t>() + (k * psasync::kMbox + m) * (cap_ + 1);
    const int64_t n = count_at(keys + cap_, s);
    const int64_t step = applied_.load() + 1;
    if (n > 0) {
      slots_of(keys, n, s);
      psamd::SparseOptArgs a = a_;
      if (bias_mode_ == 1) {
        a.bc1 = static_cast<float>(1.0 / (1.0 - std::pow(static_cast<double>(a.beta1), static_cast<double>(step))));
        a.bc2 = static_cast<float>(1.0 / (1.0 - std::pow(static_cast<double>(a.beta2), static_cast<double>(step))));
      } else if (bias_mode_ == 2) {
        a.bc1 = 1.f / (1.f - a.beta1);
        a.bc2 = 1.f / (1.f - a.beta2);
      }
      a.table = table_.data_ptr<float>();
      a.st0 = st0_.defined() ? st0_.data_ptr<float>() : nullptr;
      a.st1 = st1_.defined() ? st1_.data_ptr<float>() : nullptr;
      a.rows = slots_.data_ptr<int64_t>();
      a.perm = nullptr;
      a.grad = pg_.data_ptr<float>() + (k * psasync::kMbox + m) * cap_ * dim_;
      a.g_bf16 = 0;
      a.nrows = n;
      a.dim = dim_;
      psamd::launch_sparse_opt(a, s);
      check_status(s);  // synchronises the stream
    }
    applied_ += 1;
  }

  void run() {
    hipStream_t s = nullptr;
    try {
      hip_ok(hipSetDevice(dev_), "hipSetDevice");
      hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
      psasync::Backoff idle;
      while (!stop_.load(std::memory_order_acquire) && psasync::ld(b_ + 2) == 0) {
        bool did = false;
        for (int64_t k = 0; k < W_; ++k) {
          const int64_t rq = psasync::ld(w(0, me_, k)), rs = psasync::ld(w(1, me_, k));
          if (rq > rs) {
            serve_pull(k, s);
            psasync::st(w(1, me_, k), rq);
            served_ += 1;
            did = true;
          }
          const int64_t ps = psasync::ld(w(3, me_, k)), pa = psasync::ld(w(4, me_, k));
          if (ps > pa) {
            serve_push(k, static_cast<int>(pa % psasync::kMbox), s);
            psasync::st(w(4, me_, k), pa + 1);
            did = true;
          }
        }
        if (did) idle.n = 0;
        else idle();
      }
    } catch (const std::exception& e) {
      {
        std::lock_guard<std::mutex> g(mu_);
        err_ = e.what();
      }
      psasync::st(b_ + 2, 1);  // stop every service of the table: workers time out loudly
    }
    if (s != nullptr) {
      hipStreamSynchronize(s);
      hipStreamDestroy(s);
    }
  }

  int64_t* b_;
  int64_t W_ = 1;
  int me_;
  int64_t cap_;
  int dim_;
  int dev_ = 0;
  Tensor rq_, rs_, pk_, pg_, slots_;
  Tensor table_, flags_, hkeys_, status_, st0_, st1_;
  int64_t row_base_ = 0;
  uint64_t seed_ = 0;
  float lo_ = 0.f, hi_ = 0.f;
  int64_t* pinned_ = nullptr;  // [0] request count, [1] status word (pinned host)
  psamd::SparseOptArgs a_{};
  int bias_mode_ = 0;
  std::atomic<bool> has_updater_{false};
  std::atomic<bool> stop_{true};
  std::atomic<int64_t> applied_{0}, served_{0};
  std::thread th_;
  std::mutex mu_;
  std::string err_;
};

// After every kernel queued so far on a stream completes: add 1 to each shared-memory word (the
// worker's "request / push deposited" signals), from a completion thread, in enqueue order.
class WordNotifier {
 public:
  WordNotifier() : th_([this] { run(); }) {}
  ~WordNotifier() {
    {
      std::lock_guard<std::mutex> g(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }
  void after(int64_t stream, int64_t device, std::vector<int64_t> words) {
    hip_ok(hipSetDevice(static_cast<int>(device)), "hipSetDevice");
    hipEvent_t ev;
    hip_ok(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipEventRecord(ev, reinterpret_cast<hipStream_t>(stream)), "hipEventRecord");
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(Job{ev, static_cast<int>(device), std::move(words)});
      pending_ += 1;
    }
    cv_.notify_all();
  }
  void drain() {
    std::unique_lock<std::mutex> g(mu_);
    cv_.wait(g, [this] { return pending_ == 0; });
  }

 private:
  struct Job {
    hipEvent_t ev;
    int device;
    std::vector<int64_t> words;
  };
  void run() {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [this] { return quit_ || !q_.empty(); });
        if (q_.empty()) return;
        j = std::move(q_.front());
        q_.pop_front();
      }
      hipSetDevice(j.device);
      hipEventSynchronize(j.ev);
      hipEventDestroy(j.ev);
      for (auto a : j.words) psasync::add(reinterpret_cast<int64_t*>(a), 1);
      {
        std::lock_guard<std::mutex> g(mu_);
        pending_ -= 1;
      }
      cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
  int64_t pending_ = 0;
  bool quit_ = false;
  std::thread th_;
};

psamd::PeerSegs peer_segs(const std::vector<int64_t>& ptrs, const std::vector<int64_t>& cnts) {
  psamd::PeerSegs P{};
  TORCH_CHECK(!ptrs.empty() && ptrs.size() <= static_cast<size_t>(psamd::kPlaneMaxSrc), "1..", psamd::kPlaneMaxSrc,
              " peers");
  TORCH_CHECK(cnts.empty() || cnts.size() == ptrs.size(), "one count word per peer");
  for (size_t i = 0; i < ptrs.size(); ++i) {
    P.ptr[i] = reinterpret_cast<void*>(ptrs[i]);
    P.cnt[i] = cnts.empty() ? nullptr : reinterpret_cast<int64_t*>(cnts[i]);
  }
  P.W = static_cast<int>(ptrs.size());
  return P;
}

}  // namespace

void register_async_rows(pybind11::module& m) {
  namespace py = pybind11;
  auto r = m.def_submodule("rows", "GPU owner service + worker segment moves of the asynchronous row tables");
  py::class_<GpuRowService>(r, "Service")
      .def(py::init<uintptr_t, int64_t, int64_t, int64_t>())
      .def("set_mailboxes", &GpuRowService::set_mailboxes)
      .def("set_shard", &GpuRowService::set_shard)
      .def("set_updater", &GpuRowService::set_updater)
      .def("start", &GpuRowService::start)
      .def_property_readonly("running", &GpuRowService::running)
      .def("stop", &GpuRowService::stop, py::call_guard<py::gil_scoped_release>())
      .def("error", &GpuRowService::error)
      .def_property_readonly("applied", &GpuRowService::applied)
      .def("set_applied", &GpuRowService::set_applied)
      .def_property_readonly("served", &GpuRowService::served);
  py::class_<WordNotifier>(r, "Notifier")
      .def(py::init<>())
      .def("after", &WordNotifier::after)
      .def("drain", &WordNotifier::drain, py::call_guard<py::gil_scoped_release>());
  // owner-sorted local buffer -> the owners' mailboxes (+ their count words), or back
  r.def("to_peers", [](Tensor local, Tensor meta, std::vector<int64_t> ptrs, std::vector<int64_t> cnts, int64_t width,
                       int64_t cap) {
    TORCH_CHECK(local.is_cuda() && local.is_contiguous() && meta.is_cuda() && meta.scalar_type() == torch::kInt64,
                "device buffers");
    TORCH_CHECK(local.scalar_type() == torch::kInt64 || local.scalar_type() == torch::kFloat32, "int64 keys / f32 rows");
    const auto P = peer_segs(ptrs, cnts);
    TORCH_CHECK(meta.numel() == 2 * P.W, "meta [2W]");
    const c10::DeviceGuard guard(local.device());
    psamd::launch_segs_peers(true, local.data_ptr(), static_cast<int>(local.element_size()), meta.data_ptr<int64_t>(),
                             P, width, cap, c10::hip::getCurrentHIPStream(local.device().index()).stream());
  });
  r.def("from_peers", [](Tensor local, Tensor meta, std::vector<int64_t> ptrs, int64_t width, int64_t cap) {
    TORCH_CHECK(local.is_cuda() && local.is_contiguous() && local.scalar_type() == torch::kFloat32, "f32 rows");
    const auto P = peer_segs(ptrs, {});
    TORCH_CHECK(meta.numel() == 2 * P.W, "meta [2W]");
    const c10::DeviceGuard guard(local.device());
    psamd::launch_segs_peers(false, local.data_ptr(), 4, meta.data_ptr<int64_t>(), P, width, cap,
                             c10::hip::getCurrentHIPStream(local.device().index()).stream());
  });
}
