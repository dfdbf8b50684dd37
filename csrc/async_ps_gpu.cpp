// GPU side of the asynchronous parameter server (see csrc/include/async_ctl.h for the protocol).
//
//  GpuAsyncServer  owner progress thread: waits for deposited pushes in the shared control
//                  block, runs the fused HIP optimizer (csrc/kernels/optim.hip) of every
//                  updater segment of the fp32 master shard (per-key-prefix updaters, e.g.
//                  FTRL wide rows + Adam elsewhere) with the worker's mailbox as gradient,
//                  writing the new weights straight into a free published slot, synchronises
//                  its own stream, then publishes + acknowledges.  Its stream never touches the
//                  training streams.
//  GpuNotifier     worker completion thread: the training thread records an event after the
//                  peer copies of a push (or a pull) and hands the follow-up bookkeeping (bump
//                  seq / clock, unpin slots) to this thread, so neither the push nor the pull
//                  blocks the host that keeps launching the next step's kernels.
#include <torch/extension.h>

#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <thread>

#include "async_ctl.h"
#include "psamd_launch.h"

namespace {

using torch::Tensor;
psasync::AsyncCtl* ctl_at(uintptr_t addr) { return reinterpret_cast<psasync::AsyncCtl*>(addr); }

void hip_ok(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e));
}

class GpuAsyncServer {
 public:
  // mbox: W * kMbox mailboxes (worker w, slot m at w * kMbox + m); pub: kSlots published slots.
  // Updater segments (per-key-prefix updaters, ColocatedPS-style) are added before start().
  GpuAsyncServer(uintptr_t ctl, int64_t me, Tensor master, std::vector<Tensor> mbox, std::vector<Tensor> pub,
                 double gscale)
      : ctl_(ctl_at(ctl)), me_(static_cast<int>(me)), master_(master), mbox_(mbox), pub_(pub), gscale_(gscale) {
    TORCH_CHECK(master.is_cuda() && master.scalar_type() == torch::kFloat32 && master.is_contiguous(), "master");
    TORCH_CHECK(static_cast<int64_t>(pub.size()) == psasync::kSlots, "need ", psasync::kSlots, " published slots");
    TORCH_CHECK(static_cast<int64_t>(mbox.size()) == ctl_->world * psasync::kMbox, "W x kMbox mailboxes");
    const int64_t n = master.numel();
    for (auto& t : mbox) TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.numel() == n, "mailbox shape");
    for (auto& t : pub) TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.numel() == n, "slot shape");
    TORCH_CHECK(mbox[0].scalar_type() == pub[0].scalar_type(), "mailbox / slot dtype");
    dev_ = master.device().index();
    bf16_ = mbox[0].scalar_type() == torch::kBFloat16;
    esize_ = bf16_ ? 2 : 4;
    // test hook: a slow owner (the worker's host then runs far ahead of the server)
    if (const char* d = std::getenv("PS_AMD_ASYNC_SERVE_DELAY_US")) delay_us_ = std::atoi(d);
  }
  ~GpuAsyncServer() { stop(); }

  // [lo, hi) of the shard with its own kernel kind, state tensors (segment-sized) and
  // hyper-parameters (ps_amd/parallel/plane.py order); bias_mode 0 none, 1 1-beta^t, 2 constant
  void add_segment(int64_t kind, int64_t lo, int64_t hi, c10::optional<Tensor> st0, c10::optional<Tensor> st1,
                   std::vector<double> h, int64_t bias_mode) {
    TORCH_CHECK(h.size() == 16, "16 hyper-parameters");
    TORCH_CHECK(lo >= 0 && hi <= master_.numel() && lo < hi, "segment range");
    Seg sg;
    sg.lo = lo;
    sg.hi = hi;
    sg.bias_mode = static_cast<int>(bias_mode);
    if (st0.has_value() && st0->defined()) sg.st0 = *st0;
    if (st1.has_value() && st1->defined()) sg.st1 = *st1;
    for (auto* t : {&sg.st0, &sg.st1})
      if (t->defined())
        TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kFloat32 && t->numel() == hi - lo, "segment state");
    psamd::FusedOptArgs& a = sg.a;
    a.kind = static_cast<int>(kind);
    a.w = master_.data_ptr<float>() + lo;
    a.st0 = sg.st0.defined() ? sg.st0.data_ptr<float>() : nullptr;
    a.st1 = sg.st1.defined() ? sg.st1.data_ptr<float>() : nullptr;
    a.g_bf16 = bf16_;
    a.wout_bf16 = bf16_;
    a.n = hi - lo;
    a.lr = h[0]; a.beta1 = h[1]; a.beta2 = h[2]; a.eps = h[3]; a.wd = h[4]; a.momentum = h[5];
    a.dampening = h[6]; a.nesterov = h[7] != 0.0; a.adamw = h[8] != 0.0; a.bc1 = h[9]; a.bc2 = h[10];
    a.l1 = h[11]; a.l2 = h[12]; a.fbeta = h[13]; a.ftrl_mode = static_cast<int>(h[14]);
    a.gscale = static_cast<float>(h[15] * gscale_);
    a.gscale_ptr = nullptr;
    segs_.push_back(sg);
  }

  void start() {
    TORCH_CHECK(!segs_.empty(), "async server without updater segments");
    stop_ = false;
    th_ = std::thread([this] {
      hip_ok(hipSetDevice(dev_), "hipSetDevice");
      hipStream_t s;
      hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
      psasync::serve_loop(ctl_, me_, &stop_, [&](int w, int mslot, int slot, int64_t step) {
        if (delay_us_ > 0) std::this_thread::sleep_for(std::chrono::microseconds(delay_us_));
        const void* g = mbox_[static_cast<size_t>(w * psasync::kMbox + mslot)].data_ptr();
        char* out = static_cast<char*>(pub_[static_cast<size_t>(slot)].data_ptr());
        for (const Seg& sg : segs_) {
          psamd::FusedOptArgs a = sg.a;
          if (sg.bias_mode == 1) {
            a.bc1 = 1.f / (1.f - std::pow(static_cast<double>(a.beta1), static_cast<double>(step)));
            a.bc2 = 1.f / (1.f - std::pow(static_cast<double>(a.beta2), static_cast<double>(step)));
          } else if (sg.bias_mode == 2) {
            a.bc1 = 1.f / (1.f - a.beta1);
            a.bc2 = 1.f / (1.f - a.beta2);
          }
          a.wout = out + sg.lo * esize_;
          // the mailbox was written by a peer GPU's copy kernel: the multi-source form (one
          // source) starts with the system-scope acquire that keeps stale lines out
          psamd::MultiGrad m{};
          m.nsrc = 1;
          m.g[0] = g;
          m.off = sg.lo;
          psamd::launch_fused_opt_multi(a, m, s);
        }
        hip_ok(hipStreamSynchronize(s), "async server step");
        applied_ += 1;
      });
      hipStreamDestroy(s);
    });
  }
  void stop() {
    stop_ = true;
    if (th_.joinable()) th_.join();
  }
  int64_t applied() const { return applied_; }

 private:
  struct Seg {
    int64_t lo, hi;
    int bias_mode;
    Tensor st0, st1;
    psamd::FusedOptArgs a{};
  };
  psasync::AsyncCtl* ctl_;
  int me_;
  int dev_ = 0;
  Tensor master_;
  std::vector<Tensor> mbox_, pub_;
  double gscale_;
  bool bf16_ = true;
  int64_t esize_ = 2;
  std::vector<Seg> segs_;
  std::atomic<bool> stop_{true};
  std::thread th_;
  int64_t applied_ = 0;
  int delay_us_ = 0;
};

class GpuNotifier {
 public:
  explicit GpuNotifier(uintptr_t ctl) : ctl_(ctl_at(ctl)) {
    th_ = std::thread([this] { run(); });
  }
  ~GpuNotifier() {
    {
      std::lock_guard<std::mutex> g(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }
  // After all work queued so far on ``stream`` completes: seq[o][worker]++ for o in seq_owners,
  // clock[worker]++ if bump_clock, unpin (o, slot) pairs.
  void after(int64_t stream, int64_t device, std::vector<int64_t> seq_owners, int64_t worker, bool bump_clock,
             std::vector<std::pair<int64_t, int64_t>> unpins) {
    hip_ok(hipSetDevice(static_cast<int>(device)), "hipSetDevice");
    hipEvent_t ev;
    hip_ok(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipEventRecord(ev, reinterpret_cast<hipStream_t>(stream)), "hipEventRecord");
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(Job{ev, static_cast<int>(device), std::move(seq_owners), static_cast<int>(worker), bump_clock,
                       std::move(unpins)});
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
    std::vector<int64_t> seq_owners;
    int worker;
    bool clock;
    std::vector<std::pair<int64_t, int64_t>> unpins;
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
      hipEventSynchronize(j.ev);  // jobs complete in stream order: FIFO keeps seq/clock ordered
      hipEventDestroy(j.ev);
      for (auto o : j.seq_owners) psasync::add(&ctl_->seq[o][j.worker], 1);
      if (j.clock) psasync::add(&ctl_->clock[j.worker], 1);
      for (auto& u : j.unpins) psasync::unpin(ctl_, static_cast<int>(u.first), static_cast<int>(u.second));
      {
        std::lock_guard<std::mutex> g(mu_);
        pending_ -= 1;
      }
      cv_.notify_all();
    }
  }
  psasync::AsyncCtl* ctl_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
  int64_t pending_ = 0;
  bool quit_ = false;
  std::thread th_;
};

}  // namespace

void register_async_ps(pybind11::module& m) {
  pybind11::class_<GpuAsyncServer>(m, "GpuAsyncServer")
      .def(pybind11::init<uintptr_t, int64_t, Tensor, std::vector<Tensor>, std::vector<Tensor>, double>())
      .def("add_segment", &GpuAsyncServer::add_segment)
      .def("start", &GpuAsyncServer::start)
      .def("stop", &GpuAsyncServer::stop, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def_property_readonly("applied", &GpuAsyncServer::applied);
  pybind11::class_<GpuNotifier>(m, "GpuNotifier")
      .def(pybind11::init<uintptr_t>())
      .def("after", &GpuNotifier::after)
      .def("drain", &GpuNotifier::drain, pybind11::call_guard<pybind11::gil_scoped_release>());
}
