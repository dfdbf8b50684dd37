// GPU side of the asynchronous parameter server (see csrc/include/async_ctl.h for the protocol).
//
//  GpuAsyncServer  owner progress thread: waits for deposited pushes in the shared control
//                  block, runs the fused HIP optimizer (csrc/kernels/optim.hip) on the fp32
//                  master shard with the worker's mailbox as gradient, writing the new weights
//                  straight into a free published slot, synchronises its own stream, then
//                  publishes + acknowledges.  Its stream never touches the training streams.
//  GpuNotifier     worker completion thread: the training thread records an event after the
//                  peer copies of a push (or a pull) and hands the follow-up bookkeeping (bump
//                  seq / clock, unpin slots) to this thread, so neither the push nor the pull
//                  blocks the host that keeps launching the next step's kernels.
#include <torch/extension.h>

#include <chrono>
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
  // kind / hyper-parameters as ops/optim.py fused_opt; bias_mode 0 none, 1 1-beta^t, 2 constant
  GpuAsyncServer(uintptr_t ctl, int64_t me, int64_t kind, Tensor master, c10::optional<Tensor> st0,
                 c10::optional<Tensor> st1, std::vector<Tensor> mbox, std::vector<Tensor> pub, double lr,
                 double beta1, double beta2, double eps, double wd, double momentum, double dampening, bool nesterov,
                 bool adamw, int64_t bias_mode, double l1, double l2, double fbeta, int64_t ftrl_mode,
                 double gscale)
      : ctl_(ctl_at(ctl)), me_(static_cast<int>(me)), master_(master), mbox_(mbox), pub_(pub),
        beta1_(beta1), beta2_(beta2), bias_mode_(static_cast<int>(bias_mode)) {
    TORCH_CHECK(master.is_cuda() && master.scalar_type() == torch::kFloat32 && master.is_contiguous(), "master");
    TORCH_CHECK(static_cast<int64_t>(pub.size()) == psasync::kSlots, "need ", psasync::kSlots, " published slots");
    TORCH_CHECK(static_cast<int64_t>(mbox.size()) == ctl_->world, "one mailbox per worker");
    const int64_t n = master.numel();
    for (auto& t : mbox) TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.numel() == n, "mailbox shape");
    for (auto& t : pub) TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.numel() == n, "slot shape");
    dev_ = master.device().index();
    if (st0.has_value() && st0->defined()) st0_ = *st0;
    if (st1.has_value() && st1->defined()) st1_ = *st1;
    a_.kind = static_cast<int>(kind);
    a_.w = master.data_ptr<float>();
    a_.st0 = st0_.defined() ? st0_.data_ptr<float>() : nullptr;
    a_.st1 = st1_.defined() ? st1_.data_ptr<float>() : nullptr;
    a_.g_bf16 = mbox[0].scalar_type() == torch::kBFloat16;
    a_.wout_bf16 = pub[0].scalar_type() == torch::kBFloat16;
    a_.n = n;
    a_.lr = lr; a_.beta1 = beta1; a_.beta2 = beta2; a_.eps = eps; a_.wd = wd; a_.momentum = momentum;
    a_.dampening = dampening; a_.nesterov = nesterov; a_.adamw = adamw; a_.bc1 = 1.f; a_.bc2 = 1.f;
    a_.l1 = l1; a_.l2 = l2; a_.fbeta = fbeta; a_.ftrl_mode = static_cast<int>(ftrl_mode);
    a_.gscale = gscale; a_.gscale_ptr = nullptr;
    // test hook: a slow owner (the worker's host then runs far ahead of the server)
    if (const char* d = std::getenv("PS_AMD_ASYNC_SERVE_DELAY_US")) delay_us_ = std::atoi(d);
  }
  ~GpuAsyncServer() { stop(); }

  void start() {
    stop_ = false;
    th_ = std::thread([this] {
      hip_ok(hipSetDevice(dev_), "hipSetDevice");
      hipStream_t s;
      hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
      psasync::serve_loop(ctl_, me_, &stop_, [&](int w, int slot, int64_t step) {
        psamd::FusedOptArgs a = a_;
        if (bias_mode_ == 1) {
          a.bc1 = 1.f / (1.f - std::pow(beta1_, static_cast<double>(step)));
          a.bc2 = 1.f / (1.f - std::pow(beta2_, static_cast<double>(step)));
        } else if (bias_mode_ == 2) {
          a.bc1 = 1.f / (1.f - beta1_);
          a.bc2 = 1.f / (1.f - beta2_);
        }
        if (delay_us_ > 0) std::this_thread::sleep_for(std::chrono::microseconds(delay_us_));
        a.g = mbox_[static_cast<size_t>(w)].data_ptr();
        a.wout = pub_[static_cast<size_t>(slot)].data_ptr();
        psamd::launch_fused_opt(a, s);
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
  psasync::AsyncCtl* ctl_;
  int me_;
  int dev_ = 0;
  Tensor master_, st0_, st1_;
  std::vector<Tensor> mbox_, pub_;
  double beta1_, beta2_;
  int bias_mode_;
  psamd::FusedOptArgs a_{};
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
      .def(pybind11::init<uintptr_t, int64_t, int64_t, Tensor, c10::optional<Tensor>, c10::optional<Tensor>,
                          std::vector<Tensor>, std::vector<Tensor>, double, double, double, double, double, double,
                          double, bool, bool, int64_t, double, double, double, int64_t, double>())
      .def("start", &GpuAsyncServer::start)
      .def("stop", &GpuAsyncServer::stop, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def_property_readonly("applied", &GpuAsyncServer::applied);
  pybind11::class_<GpuNotifier>(m, "GpuNotifier")
      .def(pybind11::init<uintptr_t>())
      .def("after", &GpuNotifier::after)
      .def("drain", &GpuNotifier::drain, pybind11::call_guard<pybind11::gil_scoped_release>());
}
