// Native engine of the xGMI parameter-server plane (ps_amd/parallel/plane.py).
//
// Reference round (store/KVStore.java:240-268, net/PServer.java:164-214, 238-283): every worker
// pushes each key's gradient to the key's server, meets the others at a barrier, the server
// applies the updater, the workers pull the new weights.  On one MI355X node every rank is a
// worker AND the owner of a range chunk of every bucket (ps_amd/parallel/registry.py), and the
// round of bucket b is three one-sided steps over IPC-mapped device memory:
//
//   push   the worker lands b's gradient in its OWN bucket buffer (compute stream) and this
//          engine publishes ready[me][b] = round + 1 once the landing event completed;
//   serve  when every rank's ready[.][b] reached the round, ONE kernel on the owner reads its
//          chunk of b from all W peers' buffers at once (W xGMI links), sums in fp32 in rank
//          order and applies the fused optimizer (csrc/kernels/optim.hip fused_opt_multi),
//          writing the new weights into the owner's own replica; served[me][b] = round + 1;
//   pull   when every owner served b, ONE kernel copies the other owners' fresh chunks out of
//          their replicas into this one (csrc/kernels/plane.hip), blocks dealt over the owners.
//
// The control words live in POSIX shared memory (one node) and are only touched by host
// threads: no kernel ever spins on a flag, so a dead or slow peer can stall a round but never
// hang the GPU (every wait here has a deadline and an abort word every rank watches).  The
// training thread never blocks on a peer either: it hands (bucket, round, landing event) to
// this engine and later makes its compute stream wait on the round's last pull event.
//
// Options: 1-bit pushes (the owner decodes W packed pushes inside the same kernel), global-norm
// clipping (reduce all buckets -> publish partial sum of squares -> every rank sums the W
// partials in rank order -> factor -> serve), bounded staleness via gradient / weight rings of
// nslots slots (the Python side chooses the slots; ordering is causal, see plane.py).
//
// Without a GPU (CPU processes over gloo, used by the tests) the same state machine drives
// Python callbacks that do the serve / pull / reduce work on shared-memory tensors.
#include <torch/extension.h>

#include <chrono>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "async_ctl.h"
#include "psamd_launch.h"

namespace {

namespace py = pybind11;
using Clock = std::chrono::steady_clock;

constexpr int64_t kPlaneMagic = 0x504c414e45303031ll;  // "PLANE001"
constexpr int kHdr = 8;
constexpr int kHyper = 16;  // lr beta1 beta2 eps wd momentum dampening nesterov adamw bc1 bc2 l1 l2 fbeta ftrl gscale

void hip_ok(hipError_t e, const char* what) { TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e)); }

int64_t ctl_words(int64_t W, int64_t NB) { return kHdr + 2 * W * NB + 2 * W; }

struct Ctl {
  int64_t* base = nullptr;
  int64_t W = 0, NB = 0;
  int64_t* ready(int64_t o, int64_t b) const { return base + kHdr + o * NB + b; }
  int64_t* served(int64_t o, int64_t b) const { return base + kHdr + W * NB + o * NB + b; }
  int64_t* sqready(int64_t o) const { return base + kHdr + 2 * W * NB + o; }
  int64_t* fdone(int64_t o) const { return base + kHdr + 2 * W * NB + W + o; }
  int64_t* abort_word() const { return base + 3; }
  int64_t* abort_rank() const { return base + 4; }
};

struct Segment {
  int uid, kind;
  int64_t a, z;  // chunk-local element range
  float *master, *st0, *st1;
};

struct BucketDesc {
  int g_bf16 = 1;
  int64_t esize = 2;
  int64_t chunk = 0;  // elements per owner
  std::vector<int64_t> goff, woff, words_off, scales_off;  // per slot, byte offset of the bucket start
  float* gshard = nullptr;  // clip: local fp32 reduced chunk
  std::vector<Segment> segs;
};

enum Stage { LAND, READY, REDUCED, SERVING, SERVED, PULLING, DONE };

struct Job {
  int64_t round;
  int b, gslot, wslot, flags;
  Stage stage = LAND;
  hipEvent_t land = nullptr, s0 = nullptr, s1 = nullptr, p0 = nullptr, p1 = nullptr;
  Clock::time_point since, t_submit, t_ready, t_allready, t_served, t_allserved;
};

struct ClipRound {
  int nreduced = 0;
  int stage = 0;  // 0 wait zero, 1 zeroed, 2 sq recorded, 3 sq published, 4 factor enqueued, 5 fdone published
  hipEvent_t sq_ev = nullptr, f_ev = nullptr;
  Clock::time_point since;
};

double ms_between(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

class PlaneEngine {
 public:
  PlaneEngine(uintptr_t ctl, int64_t me, int64_t world, int64_t nb, int64_t nslots, bool gpu, int64_t device,
              double timeout_s, double clip_norm, bool average)
      : me_(static_cast<int>(me)), W_(static_cast<int>(world)), NB_(static_cast<int>(nb)),
        nslots_(static_cast<int>(nslots)), gpu_(gpu), dev_(static_cast<int>(device)), timeout_s_(timeout_s),
        clip_(clip_norm), average_(average) {
    TORCH_CHECK(world >= 1 && world <= psamd::kPlaneMaxSrc, "plane world must be in [1, ", psamd::kPlaneMaxSrc, "]");
    ctl_.base = reinterpret_cast<int64_t*>(ctl);
    ctl_.W = world;
    ctl_.NB = nb;
    TORCH_CHECK(psasync::ld(ctl_.base) == kPlaneMagic, "plane control block not initialised");
    buckets_.resize(static_cast<size_t>(nb));
    bases_.assign(static_cast<size_t>(world), 0);
  }
  ~PlaneEngine() { stop(); }

  void set_bases(std::vector<int64_t> bases) {
    TORCH_CHECK(static_cast<int>(bases.size()) == W_, "one arena base per rank");
    for (int r = 0; r < W_; ++r) bases_[static_cast<size_t>(r)] = static_cast<uintptr_t>(bases[static_cast<size_t>(r)]);
  }

  void add_bucket(int64_t b, bool g_bf16, int64_t esize, int64_t chunk, std::vector<int64_t> goff,
                  std::vector<int64_t> woff, std::vector<int64_t> words_off, std::vector<int64_t> scales_off,
                  int64_t gshard) {
    TORCH_CHECK(b >= 0 && b < NB_, "bucket index");
    TORCH_CHECK(static_cast<int>(goff.size()) == nslots_ && static_cast<int>(woff.size()) == nslots_, "slots");
    TORCH_CHECK((chunk * esize) % 16 == 0, "plane chunks must be multiples of 16 B");
    auto& d = buckets_[static_cast<size_t>(b)];
    d.g_bf16 = g_bf16 ? 1 : 0;
    d.esize = esize;
    d.chunk = chunk;
    d.goff = goff;
    d.woff = woff;
    d.words_off = words_off;
    d.scales_off = scales_off;
    d.gshard = reinterpret_cast<float*>(gshard);
  }

  void add_segment(int64_t b, int64_t uid, int64_t kind, int64_t a, int64_t z, int64_t master, int64_t st0,
                   int64_t st1) {
    auto& d = buckets_.at(static_cast<size_t>(b));
    d.segs.push_back(Segment{static_cast<int>(uid), static_cast<int>(kind), a, z, reinterpret_cast<float*>(master),
                             reinterpret_cast<float*>(st0), reinterpret_cast<float*>(st1)});
  }

  // clip: 2 fp32 norm slots at byte offset sq_off of every arena, local scratch for the total,
  // the factor and the sum-of-squares partials
  void set_norm(int64_t sq_off, int64_t total, int64_t factor, int64_t partial) {
    sq_off_ = sq_off;
    total_ = reinterpret_cast<float*>(total);
    factor_ = reinterpret_cast<float*>(factor);
    partial_ = reinterpret_cast<float*>(partial);
  }

  void set_hyper(int64_t round, int64_t uid, std::vector<double> h) {
    TORCH_CHECK(static_cast<int>(h.size()) == kHyper, "hyper vector of ", kHyper);
    std::lock_guard<std::mutex> g(mu_);
    auto& v = hyper_[round];
    if (static_cast<int64_t>(v.size()) <= uid) v.resize(static_cast<size_t>(uid + 1));
    v[static_cast<size_t>(uid)] = h;
  }

  void set_callback(py::object cb) { cb_ = cb; }

  void start() {
    TORCH_CHECK(!th_.joinable(), "plane engine already running");
    quit_ = false;
    th_ = std::thread([this] { run(); });
  }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }

  // training thread: bucket b of ``round`` has been landed (and packed) on ``stream``
  void push(int64_t b, int64_t round, int64_t gslot, int64_t wslot, int64_t flags, int64_t stream) {
    Job j;
    j.round = round;
    j.b = static_cast<int>(b);
    j.gslot = static_cast<int>(gslot);
    j.wslot = static_cast<int>(wslot);
    j.flags = static_cast<int>(flags);
    j.t_submit = j.since = Clock::now();
    if (gpu_) {
      hip_ok(hipSetDevice(dev_), "hipSetDevice");
      // default event flags keep the system-scope release: peers on other GPUs read this data;
      // timing enabled: land -> serve start is the device-side wait for the slowest push
      hip_ok(hipEventCreateWithFlags(&j.land, hipEventDefault), "hipEventCreate");
      hip_ok(hipEventRecord(j.land, reinterpret_cast<hipStream_t>(stream)), "hipEventRecord");
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      TORCH_CHECK(err_.empty(), "plane engine failed: ", err_);
      incoming_.push_back(j);
    }
    cv_.notify_all();
  }

  // make ``stream`` wait until every pull of ``round`` has landed (blocks the host only until
  // the pulls are ENQUEUED, i.e. until every owner served the round)
  void wait_pulled(int64_t round, int64_t stream) {
    hipEvent_t ev = nullptr;
    {
      std::unique_lock<std::mutex> g(mu_);
      const auto deadline = Clock::now() + std::chrono::duration<double>(timeout_s_);
      while (err_.empty() && !round_ev_.count(round) && round > done_round_) {
        if (cv_.wait_until(g, deadline) == std::cv_status::timeout && !round_ev_.count(round) &&
            round > done_round_ && err_.empty()) {
          err_ = "timed out waiting for round " + std::to_string(round) + " to be pulled";
          psasync::st(ctl_.abort_word(), 1);
          break;
        }
      }
      TORCH_CHECK(err_.empty(), "plane engine failed: ", err_);
      auto it0 = round_ev_.find(round);
      if (it0 == round_ev_.end()) return;  // a later round's pull event was already waited on
      ev = it0->second;
      // events of earlier rounds are never waited again
      for (auto it = round_ev_.begin(); it != round_ev_.end() && it->first < round;) {
        if (it->second) retire_events_.push_back(it->second);
        it = round_ev_.erase(it);
      }
    }
    if (gpu_ && ev) hip_ok(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), ev, 0), "hipStreamWaitEvent");
  }

  // one-off copy of ``nbytes`` at byte offset ``off`` from rank ``src``'s arena into ours on
  // ``stream`` (start-up broadcast, checkpoint restore; the caller brackets it with barriers)
  void copy_peer(int64_t src, int64_t off, int64_t nbytes, int64_t stream) {
    TORCH_CHECK(gpu_, "copy_peer is the GPU path");
    psamd::PlaneCopies c{};
    c.nseg = 1;
    c.src[0] = reinterpret_cast<const void*>(bases_[static_cast<size_t>(src)] + off);
    c.dst[0] = reinterpret_cast<void*>(bases_[static_cast<size_t>(me_)] + off);
    hip_ok(hipSetDevice(dev_), "hipSetDevice");
    psamd::launch_plane_gather(c, nbytes, reinterpret_cast<hipStream_t>(stream));
  }

  // pull every owner's chunk of bucket b from weight slot ``wslot`` now, on ``stream``
  void gather_now(int64_t b, int64_t wslot, int64_t stream) {
    TORCH_CHECK(gpu_, "gather_now is the GPU path");
    hip_ok(hipSetDevice(dev_), "hipSetDevice");
    launch_pull(buckets_.at(static_cast<size_t>(b)), static_cast<int>(wslot), reinterpret_cast<hipStream_t>(stream));
  }

  py::dict stats(bool reset) {
    std::lock_guard<std::mutex> g(mu_);
    py::dict d;
    const double n = rounds_done_ > 0 ? static_cast<double>(rounds_done_) : 1.0;
    for (auto& kv : sums_) d[py::str(kv.first)] = kv.second / n;
    d["rounds"] = rounds_done_;
    d["jobs"] = jobs_done_;
    // link throughput of the two one-sided phases: bytes each rank's kernels moved / their
    // device time (serve reads W pushes of its chunk, pull reads W-1 owners' chunks)
    auto rate = [&](const char* bytes, const char* ms) {
      auto b = sums_.find(bytes), t = sums_.find(ms);
      return (b == sums_.end() || t == sums_.end() || t->second <= 0.0) ? 0.0 : b->second / (t->second * 1e6);
    };
    d["serve_GBps"] = rate("serve_bytes", "serve_ms");
    d["pull_GBps"] = rate("pull_bytes", "pull_ms");
    if (reset) {
      sums_.clear();
      rounds_done_ = 0;
      jobs_done_ = 0;
    }
    return d;
  }

  std::string error() {
    std::lock_guard<std::mutex> g(mu_);
    return err_;
  }

  // IPC serve events: create this rank's ring (R per bucket), export handles
  std::vector<py::bytes> ipc_event_handles(int64_t ring) {
    TORCH_CHECK(gpu_ && ring >= 1, "IPC events are the GPU-process path");
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(active_.empty() && incoming_.empty(), "set up IPC events before the first push");
    hip_ok(hipSetDevice(dev_), "hipSetDevice");
    ring_ = static_cast<int>(ring);
    std::vector<py::bytes> out;
    for (int i = 0; i < NB_ * ring_; ++i) {
      hipEvent_t ev;
      hip_ok(hipEventCreateWithFlags(&ev, hipEventInterprocess | hipEventDisableTiming), "hipEventCreate(ipc)");
      own_ev_.push_back(ev);
      hipIpcEventHandle_t h;
      hip_ok(hipIpcGetEventHandle(&h, ev), "hipIpcGetEventHandle");
      out.emplace_back(reinterpret_cast<const char*>(&h), sizeof(h));
    }
    return out;
  }
  // open every peer's ring (handles[r] from rank r; own entry ignored) and switch the round end
  void enable_ipc_events(std::vector<std::vector<py::bytes>> handles) {
    TORCH_CHECK(static_cast<int>(handles.size()) == W_ && ring_ > 0, "one handle list per rank");
    hip_ok(hipSetDevice(dev_), "hipSetDevice");
    peer_ev_.assign(static_cast<size_t>(W_), {});
    for (int r = 0; r < W_; ++r) {
      if (r == me_) continue;
      TORCH_CHECK(static_cast<int>(handles[r].size()) == NB_ * ring_, "ring size mismatch");
      for (auto& hb : handles[r]) {
        std::string st = hb;
        TORCH_CHECK(st.size() == sizeof(hipIpcEventHandle_t), "bad IPC event handle");
        hipIpcEventHandle_t h;
        std::memcpy(&h, st.data(), sizeof(h));
        hipEvent_t ev;
        hip_ok(hipIpcOpenEventHandle(&ev, h), "hipIpcOpenEventHandle");
        peer_ev_[static_cast<size_t>(r)].push_back(ev);
      }
    }
    std::lock_guard<std::mutex> g(mu_);
    ipc_ = true;
  }

  // checkpoint restore at PS clock ``round`` (rounds 0 .. round-1 are complete): this rank's
  // control words say so, as if it had run them -- the peers' waits (ready / served / the clip
  // phase's fdone gate) are monotonic, so a fresh control block would stall the first round
  // after a resume at round >= 2 (e.g. fdone >= round - 1 for clipping) -- and wait_pulled of
  // an earlier round returns at once
  void restore_round(int64_t round) {
    TORCH_CHECK(round >= 0, "round");
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(incoming_.empty(), "restore_round with rounds in flight");
    for (int b = 0; b < NB_; ++b) {
      store_max(ctl_.ready(me_, b), round);
      store_max(ctl_.served(me_, b), round);
    }
    store_max(ctl_.sqready(me_), round);
    store_max(ctl_.fdone(me_), round);
    if (round - 1 > done_round_) done_round_ = round - 1;
    restored_round_ = round;
  }

 private:
  // ------------------------------------------------------------------ engine thread
  void run() {
    if (gpu_) {
      hip_ok(hipSetDevice(dev_), "hipSetDevice");
      hip_ok(hipStreamCreateWithFlags(&serve_s_, hipStreamNonBlocking), "hipStreamCreate");
      hip_ok(hipStreamCreateWithFlags(&pull_s_, hipStreamNonBlocking), "hipStreamCreate");
    }
    psasync::Backoff idle;
    for (;;) {
      {
        std::lock_guard<std::mutex> g(mu_);
        if (quit_) break;
        while (!incoming_.empty()) {
          active_.push_back(incoming_.front());
          incoming_.pop_front();
        }
        for (auto ev : retire_events_) destroy(ev);
        retire_events_.clear();
      }
      bool did = false;
      try {
        if (psasync::ld(ctl_.abort_word()) != 0 && error().empty())
          fail("aborted by rank " + std::to_string(psasync::ld(ctl_.abort_rank())));
        if (error().empty()) {
          // rounds of one bucket move in order: a job never gets ahead of the previous job of
          // its bucket (events of one stream may be observed out of order within a pass)
          std::vector<int> cap(static_cast<size_t>(NB_), static_cast<int>(DONE) + 1);
          for (auto& j : active_) {
            did |= advance(j, cap[static_cast<size_t>(j.b)]);
            cap[static_cast<size_t>(j.b)] = static_cast<int>(j.stage);
          }
          if (clip_ > 0) did |= advance_clip();
          did |= retire();
        }
      } catch (const std::exception& e) {
        fail(e.what());
      }
      if (did) idle.n = 0;
      else idle();
    }
    for (auto& j : active_) release(j);
    active_.clear();
    for (auto& kv : clip_rounds_) {
      destroy(kv.second.sq_ev);
      destroy(kv.second.f_ev);
    }
    clip_rounds_.clear();
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& kv : round_ev_) destroy(kv.second);
      round_ev_.clear();
      for (auto ev : retire_events_) destroy(ev);
      retire_events_.clear();
    }
    if (gpu_) {
      hipStreamSynchronize(serve_s_);
      hipStreamSynchronize(pull_s_);
      hipStreamDestroy(serve_s_);
      hipStreamDestroy(pull_s_);
    }
    for (auto& v : peer_ev_)
      for (auto ev : v) hipEventDestroy(ev);
    peer_ev_.clear();
    for (auto ev : own_ev_) hipEventDestroy(ev);
    own_ev_.clear();
  }

  void fail(const std::string& what) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (err_.empty()) err_ = what;
    }
    if (psasync::ld(ctl_.abort_word()) == 0) {
      psasync::st(ctl_.abort_rank(), me_);
      psasync::st(ctl_.abort_word(), 1);
    }
    cv_.notify_all();
  }

  void check_deadline(const Job& j, const char* what) {
    if (ms_between(j.since, Clock::now()) > timeout_s_ * 1e3)
      throw std::runtime_error(std::string("plane: timed out ") + what + " (bucket " + std::to_string(j.b) +
                               ", round " + std::to_string(j.round) + ")");
  }

  // only this engine writes its own words: a plain monotonic store
  static void store_max(int64_t* p, int64_t v) {
    if (psasync::ld(p) < v) psasync::st(p, v);
  }

  static bool done(hipEvent_t ev) {
    if (ev == nullptr) return true;
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return true;
    if (e == hipErrorNotReady) return false;
    throw std::runtime_error(std::string("plane: event query failed: ") + hipGetErrorString(e));
  }

  void destroy(hipEvent_t& ev) {
    if (ev != nullptr) hipEventDestroy(ev);
    ev = nullptr;
  }

  void release(Job& j) {
    destroy(j.land);
    destroy(j.s0);
    destroy(j.s1);
    destroy(j.p0);
    destroy(j.p1);
  }

  hipEvent_t record(hipStream_t s, bool timing) {
    hipEvent_t ev;
    hip_ok(hipEventCreateWithFlags(&ev, timing ? hipEventDefault : hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipEventRecord(ev, s), "hipEventRecord");
    return ev;
  }

  bool all_at_least(int64_t* (Ctl::*field)(int64_t, int64_t) const, int b, int64_t v) const {
    for (int o = 0; o < W_; ++o)
      if (psasync::ld((ctl_.*field)(o, b)) < v) return false;
    return true;
  }

  std::vector<double> hyper_of(int64_t round, int uid) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = hyper_.find(round);
    if (it == hyper_.end() || static_cast<int>(it->second.size()) <= uid || it->second[uid].empty())
      throw std::runtime_error("plane: no hyper-parameters for round " + std::to_string(round));
    return it->second[static_cast<size_t>(uid)];
  }

  void callback(const char* op, const Job& j) {
    py::gil_scoped_acquire gil;
    try {
      cb_(op, j.b, j.round, j.gslot, j.wslot, j.flags);
    } catch (py::error_already_set& e) {
      throw std::runtime_error(std::string("plane callback ") + op + ": " + e.what());
    }
  }

  // non-blocking steps of job j while it is strictly behind ``limit`` (the stage of the previous
  // job of its bucket; DONE + 1 when there is none); true if it moved
  bool advance(Job& j, int limit) {
    bool moved = false;
    for (;;) {
      if (static_cast<int>(j.stage) >= limit) break;
      const Stage before = j.stage;
      step(j, limit);
      if (j.stage == before) break;
      moved = true;
      j.since = Clock::now();
    }
    return moved;
  }

  void step(Job& j, int limit) {
    auto& bk = buckets_[static_cast<size_t>(j.b)];
    const int64_t want = j.round + 1;
    switch (j.stage) {
      case LAND:
        if (!done(j.land)) return;
        store_max(ctl_.ready(me_, j.b), want);
        j.t_ready = Clock::now();
        j.stage = READY;
        return;
      case READY: {
        if (!all_at_least(&Ctl::ready, j.b, want)) {
          check_deadline(j, "waiting for the peers' pushes");
          return;
        }
        if (clip_ > 0) {
          auto it = clip_rounds_.find(j.round);
          if (it == clip_rounds_.end()) {  // open the round's norm phase (advance_clip)
            clip_rounds_[j.round].since = Clock::now();
            return;
          }
          ClipRound& cr = it->second;
          if (cr.stage < 1) return;  // norm slot not zeroed yet
          // the reduced gradient (bk.gshard) and the factor have ONE buffer per bucket: round r+1
          // may reduce only once round r's clipped serve of this bucket is enqueued (same
          // stream, so the serve reads round r's values before the reduce overwrites them).
          // Without the gate SSP (staleness >= 1) let round r+1 reduce while round r waited
          // for its factor.  ``limit`` is the previous job's stage (DONE + 1 when none).
          if (limit < static_cast<int>(SERVING)) return;
          j.t_allready = Clock::now();
          if (gpu_) launch_reduce(bk, j, serve_s_);
          else callback("reduce", j);
          cr.nreduced += 1;
          j.stage = REDUCED;
          return;
        }
        j.t_allready = Clock::now();
        if (gpu_) {
          j.s0 = record(serve_s_, true);
          launch_serve(bk, j, serve_s_, false);
          j.s1 = record(serve_s_, true);
        } else {
          callback("serve", j);
        }
        j.stage = SERVING;
        publish_enqueued(j);
        return;
      }
      case REDUCED: {
        ClipRound& cr = clip_rounds_[j.round];
        if (cr.stage < 4) return;  // factor not enqueued yet
        if (gpu_) {
          j.s0 = record(serve_s_, true);
          launch_serve(bk, j, serve_s_, true);
          j.s1 = record(serve_s_, true);
        } else {
          callback("serve_clipped", j);
        }
        j.stage = SERVING;
        publish_enqueued(j);
        return;
      }
      case SERVING:
        if (!done(j.s1)) return;
        store_max(ctl_.served(me_, j.b), want);
        j.t_served = Clock::now();
        j.stage = SERVED;
        return;
      case SERVED:
        if (!all_at_least(&Ctl::served, j.b, want)) {
          check_deadline(j, "waiting for the owners to serve");
          return;
        }
        j.t_allserved = Clock::now();
        if (gpu_) {
          if (ipc_) {  // device-side: the pull runs after every owner's serve of this round
            const size_t k = static_cast<size_t>(j.b * ring_ + j.round % ring_);
            hip_ok(hipStreamWaitEvent(pull_s_, j.s1, 0), "hipStreamWaitEvent(own serve)");
            for (int o = 0; o < W_; ++o)
              if (o != me_) hip_ok(hipStreamWaitEvent(pull_s_, peer_ev_[static_cast<size_t>(o)][k], 0),
                                   "hipStreamWaitEvent(peer serve)");
          }
          j.p0 = record(pull_s_, true);
          launch_pull(bk, j.wslot, pull_s_);
          j.p1 = record(pull_s_, true);
        } else {
          callback("pull", j);
        }
        note_pull_enqueued(j);
        j.stage = PULLING;
        return;
      case PULLING:
        if (!done(j.p1)) return;
        account(j);
        release(j);
        j.stage = DONE;
        return;
      case DONE:
        return;
    }
  }

  // IPC mode: record this round's serve event of the bucket and publish served[me][b] now (the
  // serve is enqueued; peers order their pulls after it on the device)
  void publish_enqueued(Job& j) {
    if (!ipc_ || !gpu_) return;
    const size_t k = static_cast<size_t>(j.b * ring_ + j.round % ring_);
    hip_ok(hipEventRecord(own_ev_[k], serve_s_), "hipEventRecord(ipc)");
    store_max(ctl_.served(me_, j.b), j.round + 1);
    j.t_served = Clock::now();
    j.stage = SERVED;
  }

  void note_pull_enqueued(const Job& j) {
    int& n = pulls_enq_[j.round];
    n += 1;
    if (n == NB_) {
      pulls_enq_.erase(j.round);
      hipEvent_t ev = gpu_ ? record(pull_s_, false) : nullptr;
      {
        std::lock_guard<std::mutex> g(mu_);
        round_ev_[j.round] = ev;
        if (j.round > done_round_) done_round_ = j.round;
        hyper_.erase(hyper_.begin(), hyper_.lower_bound(j.round - 1));
      }
      cv_.notify_all();
    }
  }

  void account(const Job& j) {
    float serve_ms = 0.f, pull_ms = 0.f, land_to_serve_ms = 0.f, serve_to_pull_ms = 0.f;
    if (gpu_) {
      hipEventElapsedTime(&serve_ms, j.s0, j.s1);
      hipEventElapsedTime(&pull_ms, j.p0, j.p1);
      // device clock: own push landed -> serve kernel starts (the wait for the slowest peer's
      // push + engine latency), own serve done -> pull starts (the wait for the other owners)
      if (j.land) hipEventElapsedTime(&land_to_serve_ms, j.land, j.s0);
      hipEventElapsedTime(&serve_to_pull_ms, j.s1, j.p0);
    }
    const auto& bk = buckets_[static_cast<size_t>(j.b)];
    const double push_bytes = (j.flags & 1) ? static_cast<double>(bk.chunk) / 8.0 + bk.chunk / psamd::kOnebitChunk * 4.0
                                            : static_cast<double>(bk.chunk * bk.esize);
    std::lock_guard<std::mutex> g(mu_);
    sums_["serve_ms"] += serve_ms;
    sums_["pull_ms"] += pull_ms;
    sums_["land_to_serve_ms"] += land_to_serve_ms;
    sums_["serve_to_pull_ms"] += serve_to_pull_ms;
    sums_["serve_bytes"] += push_bytes * W_;
    sums_["pull_bytes"] += static_cast<double>(bk.chunk * bk.esize) * (W_ - 1);
    sums_["peer_push_wait_ms"] += ms_between(j.t_ready, j.t_allready);
    sums_["peer_serve_wait_ms"] += ms_between(j.t_served, j.t_allserved);
    jobs_done_ += 1;
    if (j.b == NB_ - 1) rounds_done_ += 1;
  }

  bool retire() {
    bool did = false;
    while (!active_.empty() && active_.front().stage == DONE) {
      active_.pop_front();
      did = true;
    }
    return did;
  }

  // ------------------------------------------------------------------ clipping rounds
  bool advance_clip() {
    bool did = false;
    for (auto it = clip_rounds_.begin(); it != clip_rounds_.end();) {
      const int64_t r = it->first;
      ClipRound& cr = it->second;
      const int before = cr.stage;
      if (cr.stage == 0) {
        // peers consumed round r-2's partial from this slot (fdone counts consumed rounds)
        bool ok = true;
        for (int o = 0; o < W_; ++o) ok = ok && psasync::ld(ctl_.fdone(o)) >= r - 1;
        if (ok) {
          if (gpu_) psamd::launch_plane_fill(sq_slot(me_, r), 1, 0.f, serve_s_);
          else callback_round("zero_sq", r);
          cr.stage = 1;
        }
      }
      if (cr.stage == 1 && cr.nreduced == NB_) {
        cr.sq_ev = gpu_ ? record(serve_s_, false) : nullptr;
        cr.stage = 2;
      }
      if (cr.stage == 2 && done(cr.sq_ev)) {
        destroy(cr.sq_ev);
        psasync::st(ctl_.sqready(me_), r + 1);
        cr.stage = 3;
      }
      if (cr.stage == 3) {
        bool ok = true;
        for (int o = 0; o < W_; ++o) ok = ok && psasync::ld(ctl_.sqready(o)) >= r + 1;
        if (ok) {
          if (gpu_) {
            psamd::PlaneCopies c{};
            c.nseg = W_;
            for (int o = 0; o < W_; ++o) c.src[o] = sq_slot(o, r);
            const float mx = static_cast<float>(clip_) * (average_ ? static_cast<float>(W_) : 1.f);
            psamd::launch_plane_clip_factor(c, mx, total_, factor_, serve_s_);
            cr.f_ev = record(serve_s_, false);
          } else {
            callback_round("factor", r);
          }
          cr.stage = 4;
        }
      }
      if (cr.stage == 4 && done(cr.f_ev)) {
        destroy(cr.f_ev);
        psasync::st(ctl_.fdone(me_), r + 1);
        cr.stage = 5;
      }
      if (cr.stage != before) {
        did = true;
        cr.since = Clock::now();
      } else if (cr.stage < 5 && ms_between(cr.since, Clock::now()) > timeout_s_ * 1e3) {
        throw std::runtime_error("plane: timed out in the clip phase of round " + std::to_string(r));
      }
      // drop finished rounds once no job of theirs still needs the factor
      bool needed = false;
      for (auto& j : active_) needed = needed || (j.round == r && j.stage <= REDUCED);
      if (cr.stage == 5 && !needed) it = clip_rounds_.erase(it);
      else ++it;
    }
    return did;
  }

  void callback_round(const char* op, int64_t r) {
    Job j;
    j.round = r;
    j.b = -1;
    j.gslot = j.wslot = j.flags = 0;
    callback(op, j);
  }

  float* sq_slot(int o, int64_t r) const {
    return reinterpret_cast<float*>(bases_[static_cast<size_t>(o)] + sq_off_ + (r & 1) * sizeof(float));
  }

  // ------------------------------------------------------------------ GPU launches
  psamd::MultiGrad sources(const BucketDesc& bk, const Job& j, int64_t off) const {
    psamd::MultiGrad m{};
    m.nsrc = W_;
    m.onebit = (j.flags & 1) ? 1 : 0;
    m.off = off;
    for (int p = 0; p < W_; ++p) {
      const uintptr_t base = bases_[static_cast<size_t>(p)];
      if (m.onebit) {
        m.words[p] = reinterpret_cast<const uint64_t*>(base + bk.words_off[static_cast<size_t>(j.gslot)] +
                                                       me_ * (bk.chunk / 64) * 8);
        m.scales[p] = reinterpret_cast<const float*>(base + bk.scales_off[static_cast<size_t>(j.gslot)] +
                                                     me_ * (bk.chunk / psamd::kOnebitChunk) * 4);
      } else {
        m.g[p] = reinterpret_cast<const void*>(base + bk.goff[static_cast<size_t>(j.gslot)] + me_ * bk.chunk * bk.esize);
      }
    }
    return m;
  }

  void launch_serve(const BucketDesc& bk, const Job& j, hipStream_t s, bool clipped) {
    const float avg = average_ ? 1.f / static_cast<float>(W_) : 1.f;
    const uintptr_t own = bases_[static_cast<size_t>(me_)];
    for (const auto& sg : bk.segs) {
      const std::vector<double> h = hyper_of(j.round, sg.uid);
      psamd::FusedOptArgs a{};
      a.kind = sg.kind;
      a.w = sg.master;
      a.st0 = sg.st0;
      a.st1 = sg.st1;
      a.g_bf16 = bk.g_bf16;
      a.wout = reinterpret_cast<void*>(own + bk.woff[static_cast<size_t>(j.wslot)] + (me_ * bk.chunk + sg.a) * bk.esize);
      a.wout_bf16 = bk.g_bf16;
      a.n = sg.z - sg.a;
      a.lr = h[0]; a.beta1 = h[1]; a.beta2 = h[2]; a.eps = h[3]; a.wd = h[4]; a.momentum = h[5];
      a.dampening = h[6]; a.nesterov = h[7] != 0.0; a.adamw = h[8] != 0.0; a.bc1 = h[9]; a.bc2 = h[10];
      a.l1 = h[11]; a.l2 = h[12]; a.fbeta = h[13]; a.ftrl_mode = static_cast<int>(h[14]);
      a.gscale = static_cast<float>(h[15]) * avg;
      if (clipped) {
        a.g = bk.gshard + sg.a;
        a.g_bf16 = 0;
        a.gscale_ptr = factor_;
        psamd::launch_fused_opt(a, s);
      } else {
        a.gscale_ptr = nullptr;
        psamd::launch_fused_opt_multi(a, sources(bk, j, sg.a), s);
      }
    }
  }

  void launch_reduce(const BucketDesc& bk, const Job& j, hipStream_t s) {
    psamd::launch_reduce_multi(sources(bk, j, 0), bk.g_bf16, bk.chunk, bk.gshard, s);
    const int nblk = psamd::sumsq_blocks(bk.chunk);
    psamd::launch_sumsq_partial(bk.gshard, 0, bk.chunk, partial_, nblk, s);
    psamd::launch_sumsq_finish(partial_, nblk, sq_slot(me_, j.round), 1, s);
  }

  void launch_pull(const BucketDesc& bk, int wslot, hipStream_t s) const {
    psamd::PlaneCopies c{};
    const uintptr_t own = bases_[static_cast<size_t>(me_)];
    for (int o = 0; o < W_; ++o) {
      if (o == me_) continue;
      const int64_t off = bk.woff[static_cast<size_t>(wslot)] + o * bk.chunk * bk.esize;
      c.src[c.nseg] = reinterpret_cast<const void*>(bases_[static_cast<size_t>(o)] + off);
      c.dst[c.nseg] = reinterpret_cast<void*>(own + off);
      c.nseg += 1;
    }
    psamd::launch_plane_gather(c, bk.chunk * bk.esize, s);
  }

  int me_, W_, NB_, nslots_;
  bool gpu_;
  int dev_;
  double timeout_s_, clip_;
  bool average_;
  Ctl ctl_;
  std::vector<uintptr_t> bases_;
  std::vector<BucketDesc> buckets_;
  int64_t sq_off_ = 0;
  float *total_ = nullptr, *factor_ = nullptr, *partial_ = nullptr;
  py::object cb_;

  std::mutex mu_;
  std::condition_variable cv_;
  bool quit_ = true;
  std::string err_;
  std::deque<Job> incoming_;
  std::map<int64_t, std::vector<std::vector<double>>> hyper_;
  std::map<int64_t, hipEvent_t> round_ev_;
  std::vector<hipEvent_t> retire_events_;
  std::map<std::string, double> sums_;
  int64_t rounds_done_ = 0, jobs_done_ = 0;
  int64_t done_round_ = -1;  // rounds <= this one have every pull enqueued
  int64_t restored_round_ = 0;
  // IPC-event round end (enable_ipc_events): served[me][b] is published when the serve is
  // ENQUEUED and the pulls wait on the owners' events on the device -- no rank's host waits for
  // another rank's serve kernel to finish.  Ring of R events per bucket, slot = round % R.
  bool ipc_ = false;
  int ring_ = 0;
  std::vector<hipEvent_t> own_ev_;
  std::vector<std::vector<hipEvent_t>> peer_ev_;

  // engine-thread state
  std::thread th_;
  std::deque<Job> active_;
  std::map<int64_t, int> pulls_enq_;
  std::map<int64_t, ClipRound> clip_rounds_;
  hipStream_t serve_s_ = nullptr, pull_s_ = nullptr;
};

// ------------------------------------------------------------------ device arenas (IPC)
class Arena {
 public:
  Arena(int64_t nbytes, int64_t device) : dev_(static_cast<int>(device)), n_(nbytes) {
    hip_ok(hipSetDevice(dev_), "hipSetDevice");
    hip_ok(hipMalloc(&ptr_, static_cast<size_t>(nbytes)), "hipMalloc(plane arena)");
    hip_ok(hipMemset(ptr_, 0, static_cast<size_t>(nbytes)), "hipMemset");
    hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
  }
  ~Arena() { close(); }
  void close() {
    for (auto p : opened_) hipIpcCloseMemHandle(p);
    opened_.clear();
    if (ptr_ != nullptr) {
      hipSetDevice(dev_);
      hipFree(ptr_);
      ptr_ = nullptr;
    }
  }
  torch::Tensor tensor() {
    auto opts = torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, dev_);
    return torch::from_blob(ptr_, {n_}, [](void*) {}, opts);
  }
  int64_t base() const { return reinterpret_cast<int64_t>(ptr_); }
  py::bytes handle() const {
    hipIpcMemHandle_t h;
    hip_ok(hipIpcGetMemHandle(&h, ptr_), "hipIpcGetMemHandle");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }
  // map a peer's arena into this process (peer may live on another GPU of the node)
  int64_t open(py::bytes hb, int64_t peer_device) {
    std::string s = hb;
    TORCH_CHECK(s.size() == sizeof(hipIpcMemHandle_t), "bad IPC handle");
    hip_ok(hipSetDevice(dev_), "hipSetDevice");
    if (peer_device != dev_) {
      int can = 0;
      hip_ok(hipDeviceCanAccessPeer(&can, dev_, static_cast<int>(peer_device)), "hipDeviceCanAccessPeer");
      TORCH_CHECK(can, "GPU ", dev_, " cannot access peer GPU ", peer_device);
      const hipError_t e = hipDeviceEnablePeerAccess(static_cast<int>(peer_device), 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) hip_ok(e, "hipDeviceEnablePeerAccess");
      (void)hipGetLastError();
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, s.data(), sizeof(h));
    void* p = nullptr;
    hip_ok(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    opened_.push_back(p);
    return reinterpret_cast<int64_t>(p);
  }

 private:
  int dev_;
  int64_t n_;
  void* ptr_ = nullptr;
  std::vector<void*> opened_;
};

// An arena built from physical chunks of at most ``chunk`` bytes (HIP virtual memory management),
// mapped back to back into ONE virtual range, so the local view is contiguous like Arena's.  Why:
// on this stack hipIpcOpenMemHandle hangs for any allocation above 2 GiB (1.99 GiB opens at once,
// 2.01 GiB never returns: profiles/r6_plane_ipc_2gib.txt), and a Llama-3-8B plane arena is ~34 GB.
// Each chunk is exported as a dma-buf file descriptor (the fds travel to the peers over a Unix
// socket, ps_amd/parallel/plane.py); a peer imports every chunk and maps them back to back into a
// virtual range of its own, so it also sees one contiguous arena -- the plane engine's (base +
// offset) addressing is unchanged.
class VmmArena {
 public:
  VmmArena(int64_t nbytes, int64_t device, int64_t chunk) : dev_(static_cast<int>(device)) {
    hip_ok(hipSetDevice(dev_), "hipSetDevice");
    hipMemAllocationProp prop = props(dev_);
    size_t gran = 0;
    hip_ok(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum), "granularity");
    gran_ = gran;
    const size_t ch = round_up(static_cast<size_t>(chunk), gran);
    size_t left = round_up(static_cast<size_t>(nbytes), gran);
    while (left > 0) {
      const size_t sz = left < ch ? left : ch;
      sizes_.push_back(sz);
      left -= sz;
    }
    total_ = 0;
    for (size_t sz : sizes_) total_ += sz;
    hip_ok(hipMemAddressReserve(&base_, total_, gran, nullptr, 0), "hipMemAddressReserve");
    size_t off = 0;
    for (size_t sz : sizes_) {
      hipMemGenericAllocationHandle_t h;
      hip_ok(hipMemCreate(&h, sz, &prop, 0), "hipMemCreate");
      handles_.push_back(h);
      hip_ok(hipMemMap(static_cast<char*>(base_) + off, sz, 0, h, 0), "hipMemMap");
      off += sz;
    }
    set_access(base_, total_);
    hip_ok(hipMemset(base_, 0, total_), "hipMemset");
    hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
    n_ = nbytes;
  }
  ~VmmArena() { close(); }

  // one dma-buf fd per chunk (the caller sends them to the peers, then closes them)
  std::vector<int64_t> export_fds() {
    std::vector<int64_t> fds;
    for (auto h : handles_) {
      int fd = -1;
      hip_ok(hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0),
             "hipMemExportToShareableHandle");
      fds.push_back(fd);
    }
    return fds;
  }
  std::vector<int64_t> chunk_sizes() const { return std::vector<int64_t>(sizes_.begin(), sizes_.end()); }

  // map a peer's chunks (received fds, its chunk sizes) back to back; -> the peer arena's base here
  int64_t open(std::vector<int64_t> fds, std::vector<int64_t> sizes, int64_t peer_device) {
    TORCH_CHECK(fds.size() == sizes.size() && !fds.empty(), "one fd per chunk");
    hip_ok(hipSetDevice(dev_), "hipSetDevice");
    if (peer_device != dev_) {
      int can = 0;
      hip_ok(hipDeviceCanAccessPeer(&can, dev_, static_cast<int>(peer_device)), "hipDeviceCanAccessPeer");
      TORCH_CHECK(can, "GPU ", dev_, " cannot access peer GPU ", peer_device);
    }
    size_t total = 0;
    for (auto sz : sizes) total += static_cast<size_t>(sz);
    Peer pr;
    pr.size = total;
    hip_ok(hipMemAddressReserve(&pr.base, total, gran_, nullptr, 0), "hipMemAddressReserve(peer)");
    size_t off = 0;
    for (size_t i = 0; i < fds.size(); ++i) {
      hipMemGenericAllocationHandle_t h;
      // this HIP reads the descriptor THROUGH the pointer (passing the fd value as a pointer, the
      // CUDA convention, faults at that address)
      int fdv = static_cast<int>(fds[i]);
      hip_ok(hipMemImportFromShareableHandle(&h, &fdv, hipMemHandleTypePosixFileDescriptor),
             "hipMemImportFromShareableHandle");
      pr.handles.push_back(h);
      hip_ok(hipMemMap(static_cast<char*>(pr.base) + off, static_cast<size_t>(sizes[i]), 0, h, 0), "hipMemMap(peer)");
      off += static_cast<size_t>(sizes[i]);
    }
    set_access(pr.base, total);
    peers_.push_back(pr);
    return reinterpret_cast<int64_t>(pr.base);
  }

  void close() {
    if (dev_ < 0) return;
    hipSetDevice(dev_);
    hipDeviceSynchronize();
    for (auto& pr : peers_) release(pr.base, pr.size, pr.handles);
    peers_.clear();
    if (base_ != nullptr) release(base_, total_, handles_);
    base_ = nullptr;
    handles_.clear();
    dev_ = -1;
  }
  torch::Tensor tensor() {
    auto opts = torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, dev_);
    return torch::from_blob(base_, {n_}, [](void*) {}, opts);
  }
  int64_t base() const { return reinterpret_cast<int64_t>(base_); }

 private:
  struct Peer {
    void* base = nullptr;
    size_t size = 0;
    std::vector<hipMemGenericAllocationHandle_t> handles;
  };
  static hipMemAllocationProp props(int dev) {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    return prop;
  }
  static size_t round_up(size_t n, size_t g) { return (n + g - 1) / g * g; }
  void set_access(void* p, size_t n) {
    hipMemAccessDesc d{};
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = dev_;
    d.flags = hipMemAccessFlagsProtReadWrite;
    hip_ok(hipMemSetAccess(p, n, &d, 1), "hipMemSetAccess");
  }
  static void release(void* base, size_t size, std::vector<hipMemGenericAllocationHandle_t>& hs) {
    hipMemUnmap(base, size);
    for (auto h : hs) hipMemRelease(h);
    hs.clear();
    hipMemAddressFree(base, size);
  }
  int dev_;
  int64_t n_ = 0;
  size_t gran_ = 0, total_ = 0;
  void* base_ = nullptr;
  std::vector<size_t> sizes_;
  std::vector<hipMemGenericAllocationHandle_t> handles_;
  std::vector<Peer> peers_;
};

// ------------------------------------------------------------------ IPC events
// An event another process on the node can make its streams wait on (hipEventInterprocess):
// the owner records it after a kernel, a peer that opened the handle enqueues
// hipStreamWaitEvent -- the cross-process dependency lives on the device queues, the peer's
// host only waits until the record was ENQUEUED (a flag in shared memory), never for it to run.
class IpcEvent {
 public:
  explicit IpcEvent(int64_t device) : dev_(static_cast<int>(device)) {
    hip_ok(hipSetDevice(dev_), "hipSetDevice");
    hip_ok(hipEventCreateWithFlags(&ev_, hipEventInterprocess | hipEventDisableTiming), "hipEventCreate(ipc)");
    own_ = true;
  }
  IpcEvent(py::bytes hb, int64_t device) : dev_(static_cast<int>(device)) {
    std::string s = hb;
    TORCH_CHECK(s.size() == sizeof(hipIpcEventHandle_t), "bad IPC event handle");
    hipIpcEventHandle_t h;
    std::memcpy(&h, s.data(), sizeof(h));
    hip_ok(hipSetDevice(dev_), "hipSetDevice");
    hip_ok(hipIpcOpenEventHandle(&ev_, h), "hipIpcOpenEventHandle");
  }
  ~IpcEvent() {
    if (ev_ != nullptr) hipEventDestroy(ev_);
  }
  py::bytes handle() const {
    TORCH_CHECK(own_, "only the creating process exports the handle");
    hipIpcEventHandle_t h;
    hip_ok(hipIpcGetEventHandle(&h, ev_), "hipIpcGetEventHandle");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }
  void record(int64_t stream) { hip_ok(hipEventRecord(ev_, reinterpret_cast<hipStream_t>(stream)), "hipEventRecord"); }
  void wait(int64_t stream) {
    hip_ok(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), ev_, 0), "hipStreamWaitEvent");
  }
  bool query() const {
    const hipError_t e = hipEventQuery(ev_);
    if (e == hipSuccess) return true;
    TORCH_CHECK(e == hipErrorNotReady, "hipEventQuery: ", hipGetErrorString(e));
    return false;
  }
  void synchronize() const { hip_ok(hipEventSynchronize(ev_), "hipEventSynchronize"); }
  int64_t ptr() const { return reinterpret_cast<int64_t>(ev_); }

 private:
  int dev_;
  hipEvent_t ev_ = nullptr;
  bool own_ = false;
};

}  // namespace

void register_plane(pybind11::module& m) {
  auto pm = m.def_submodule("plane", "xGMI parameter-server plane (csrc/plane.cpp)");
  pm.attr("MAX_WORLD") = psamd::kPlaneMaxSrc;
  pm.attr("HYPER") = kHyper;
  pm.def("ctl_size", [](int64_t W, int64_t NB) { return ctl_words(W, NB) * 8; });
  pm.def("ctl_init", [](uintptr_t addr, int64_t W, int64_t NB) {
    int64_t* b = reinterpret_cast<int64_t*>(addr);
    for (int64_t i = 0; i < ctl_words(W, NB); ++i) b[i] = 0;
    b[1] = W;
    b[2] = NB;
    psasync::st(b, kPlaneMagic);
  });
  pm.def("ctl_abort", [](uintptr_t addr, int64_t rank) {
    int64_t* b = reinterpret_cast<int64_t*>(addr);
    psasync::st(b + 4, rank);
    psasync::st(b + 3, 1);
  });
  pm.def("ctl_snapshot", [](uintptr_t addr) {
    int64_t* b = reinterpret_cast<int64_t*>(addr);
    std::vector<int64_t> v(static_cast<size_t>(ctl_words(b[1], b[2])));
    for (size_t i = 0; i < v.size(); ++i) v[i] = psasync::ld(b + i);
    return v;
  });
  // (src, dst, nbytes) copies -- peer arenas included -- as ONE launch on ``stream`` (async PS
  // pushes into owner mailboxes / pulls of published slots / row traffic; <= MAX_WORLD pieces)
  pm.def("copy_many", [](std::vector<std::tuple<int64_t, int64_t, int64_t>> segs, int64_t stream, int64_t device) {
    TORCH_CHECK(static_cast<int>(segs.size()) <= psamd::kPlaneMaxSrc, "too many copy segments");
    psamd::PlaneCopies c{};
    for (auto& t : segs) {
      if (std::get<2>(t) <= 0) continue;
      c.src[c.nseg] = reinterpret_cast<const void*>(std::get<0>(t));
      c.dst[c.nseg] = reinterpret_cast<void*>(std::get<1>(t));
      c.nbytes[c.nseg] = std::get<2>(t);
      TORCH_CHECK(((std::get<0>(t) | std::get<1>(t)) & 15) == 0, "copy_many: 16-B aligned pointers");
      c.nseg += 1;
    }
    hip_ok(hipSetDevice(static_cast<int>(device)), "hipSetDevice");
    psamd::launch_plane_copy(c, reinterpret_cast<hipStream_t>(stream));
  });
  // the owner-side read of the one-sided paths (remote_probe.py): n values at ``src`` into
  // ``out`` (fp32) by the multi-source reduce kernel -- the system-scope acquire at entry and the
  // loads of the async-PS serve (fused_opt_multi) and the plane serve, with one source
  pm.def("read_acquire", [](int64_t src, int64_t n, bool bf16, torch::Tensor out, int64_t stream) {
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == torch::kFloat32 && out.is_contiguous() && out.numel() >= n,
                "read_acquire: fp32 out of >= n elements");
    TORCH_CHECK((src & 15) == 0 && n > 0, "read_acquire: 16-B aligned source");
    psamd::MultiGrad m{};
    m.nsrc = 1;
    m.g[0] = reinterpret_cast<const void*>(src);
    m.off = 0;
    hip_ok(hipSetDevice(out.get_device()), "hipSetDevice");
    psamd::launch_reduce_multi(m, bf16 ? 1 : 0, n, out.data_ptr<float>(), reinterpret_cast<hipStream_t>(stream));
  });
  py::class_<PlaneEngine>(pm, "Engine")
      .def(py::init<uintptr_t, int64_t, int64_t, int64_t, int64_t, bool, int64_t, double, double, bool>())
      .def("set_bases", &PlaneEngine::set_bases)
      .def("add_bucket", &PlaneEngine::add_bucket)
      .def("add_segment", &PlaneEngine::add_segment)
      .def("set_norm", &PlaneEngine::set_norm)
      .def("set_hyper", &PlaneEngine::set_hyper)
      .def("set_callback", &PlaneEngine::set_callback)
      .def("start", &PlaneEngine::start)
      .def("stop", &PlaneEngine::stop, py::call_guard<py::gil_scoped_release>())
      .def("push", &PlaneEngine::push)
      .def("wait_pulled", &PlaneEngine::wait_pulled, py::call_guard<py::gil_scoped_release>())
      .def("copy_peer", &PlaneEngine::copy_peer)
      .def("gather_now", &PlaneEngine::gather_now)
      .def("stats", &PlaneEngine::stats, py::arg("reset") = false)
      .def("error", &PlaneEngine::error)
      .def("restore_round", &PlaneEngine::restore_round)
      .def("ipc_event_handles", &PlaneEngine::ipc_event_handles)
      .def("enable_ipc_events", &PlaneEngine::enable_ipc_events);
  py::class_<IpcEvent>(pm, "IpcEvent")
      .def(py::init<int64_t>())
      .def(py::init<py::bytes, int64_t>())
      .def("handle", &IpcEvent::handle)
      .def("record", &IpcEvent::record)
      .def("wait", &IpcEvent::wait)
      .def("query", &IpcEvent::query)
      .def("synchronize", &IpcEvent::synchronize, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("ptr", &IpcEvent::ptr);
  py::class_<VmmArena>(pm, "VmmArena")
      .def(py::init<int64_t, int64_t, int64_t>())
      .def("tensor", &VmmArena::tensor)
      .def_property_readonly("base", &VmmArena::base)
      .def("export_fds", &VmmArena::export_fds)
      .def("chunk_sizes", &VmmArena::chunk_sizes)
      .def("open", &VmmArena::open)
      .def("close", &VmmArena::close);
  py::class_<Arena>(pm, "Arena")
      .def(py::init<int64_t, int64_t>())
      .def("tensor", &Arena::tensor)
      .def_property_readonly("base", &Arena::base)
      .def("handle", &Arena::handle)
      .def("open", &Arena::open)
      .def("close", &Arena::close);
}
