// pybind11 module ps_amd._native: TCP parameter server / client, id map, batch loader.
// Every blocking call releases the GIL so Python worker threads (prefetch, UI) keep running.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "async_ctl.h"
#include "loader.h"
#include "ps_server.h"

namespace py = pybind11;
using namespace psnative;

namespace {

using F32 = py::array_t<float, py::array::c_style | py::array::forcecast>;
using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;

py::array_t<float> to_array(const Matrix& m) {
  py::array_t<float> a({static_cast<py::ssize_t>(m.rows), static_cast<py::ssize_t>(m.cols)});
  std::memcpy(a.mutable_data(), m.data.data(), m.data.size() * sizeof(float));
  return a;
}

void put_mat(Writer& w, const F32& a) {
  uint32_t rows = 1, cols = 1;
  if (a.ndim() == 1) {
    rows = static_cast<uint32_t>(a.shape(0));
  } else if (a.ndim() == 2) {
    rows = static_cast<uint32_t>(a.shape(0));
    cols = static_cast<uint32_t>(a.shape(1));
  } else if (a.ndim() == 0) {
    rows = cols = 1;
  } else {
    rows = static_cast<uint32_t>(a.shape(0));
    cols = static_cast<uint32_t>(a.size() / a.shape(0));
  }
  w.mat(rows, cols, a.data());
}

void check(uint16_t st, const std::vector<uint8_t>& resp, const char* what) {
  if (st == ST_OK || st == ST_NOT_FOUND) return;
  std::string msg;
  if (!resp.empty()) {
    try {
      Reader r(resp.data(), resp.size());
      msg = r.str();
    } catch (...) {
    }
  }
  if (st == ST_TIMEOUT) throw std::runtime_error(std::string(what) + ": timed out (dead worker?)");
  throw std::runtime_error(std::string(what) + " failed (" + std::to_string(st) + "): " + msg);
}

class Client {
 public:
  Client(const std::string& host, int port, double timeout) : c_(host, port, timeout) {}

  py::object get(const std::string& key) {
    Writer w;
    w.str(key);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_GET, w, &resp);
    }
    check(st, resp, "get");
    if (st == ST_NOT_FOUND) return py::none();
    Reader rd(resp.data(), resp.size());
    return to_array(rd.mat());
  }

  py::list get_list(const std::vector<std::string>& keys) {
    Writer w;
    w.u32(static_cast<uint32_t>(keys.size()));
    for (auto& k : keys) w.str(k);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_GET_LIST, w, &resp);
    }
    check(st, resp, "get_list");
    Reader rd(resp.data(), resp.size());
    const uint32_t n = rd.u32();
    py::list out;
    for (uint32_t i = 0; i < n; ++i) {
      if (rd.u8()) out.append(to_array(rd.mat()));
      else out.append(py::none());
    }
    return out;
  }

  py::tuple upsert(const std::string& key, const F32& a, bool replace) {
    Writer w;
    w.u8(replace ? 1 : 0);
    w.str(key);
    put_mat(w, a);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_UPSERT, w, &resp);
    }
    check(st, resp, "upsert");
    Reader rd(resp.data(), resp.size());
    const bool existed = rd.u8() != 0;
    return py::make_tuple(existed, to_array(rd.mat()));
  }

  py::list upsert_list(const std::vector<std::string>& keys, const std::vector<F32>& arrs, bool replace) {
    if (keys.size() != arrs.size()) throw std::runtime_error("keys/arrays length mismatch");
    Writer w;
    w.u8(replace ? 1 : 0);
    w.u32(static_cast<uint32_t>(keys.size()));
    for (size_t i = 0; i < keys.size(); ++i) {
      w.str(keys[i]);
      put_mat(w, arrs[i]);
    }
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_UPSERT_LIST, w, &resp);
    }
    check(st, resp, "upsert_list");
    Reader rd(resp.data(), resp.size());
    const uint32_t n = rd.u32();
    py::list out;
    for (uint32_t i = 0; i < n; ++i) {
      const bool existed = rd.u8() != 0;
      out.append(py::make_tuple(existed, to_array(rd.mat())));
    }
    return out;
  }

  void push(const std::vector<std::string>& keys, const std::vector<F32>& grads, const std::string& spec,
            int async_flag) {
    if (keys.size() != grads.size()) throw std::runtime_error("keys/grads length mismatch");
    Writer w;
    w.u8(static_cast<uint8_t>(async_flag));
    w.str(spec);
    w.u32(static_cast<uint32_t>(keys.size()));
    for (size_t i = 0; i < keys.size(); ++i) {
      w.str(keys[i]);
      put_mat(w, grads[i]);
    }
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_PUSH, w, &resp);
    }
    check(st, resp, "push");
  }

  uint64_t barrier(uint32_t worker) {
    Writer w;
    w.u32(worker);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_BARRIER, w, &resp);
    }
    check(st, resp, "barrier");
    Reader rd(resp.data(), resp.size());
    return rd.u64();
  }

  uint64_t rendezvous(uint32_t worker) {
    Writer w;
    w.u32(worker);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_RENDEZVOUS, w, &resp);
    }
    check(st, resp, "rendezvous");
    Reader rd(resp.data(), resp.size());
    return rd.u64();
  }

  uint64_t clock(uint32_t worker, uint64_t c) {
    Writer w;
    w.u32(worker);
    w.u64(c);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_CLOCK, w, &resp);
    }
    check(st, resp, "clock");
    Reader rd(resp.data(), resp.size());
    return rd.u64();
  }

  py::array_t<float> row_pull(const std::string& table, uint32_t dim, const I64& keys, float lo, float hi,
                              uint64_t seed) {
    Writer w;
    w.str(table);
    w.u32(dim);
    w.f32(lo);
    w.f32(hi);
    w.u64(seed);
    w.u32(static_cast<uint32_t>(keys.size()));
    w.raw(keys.data(), static_cast<size_t>(keys.size()) * 8);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_ROW_PULL, w, &resp);
    }
    check(st, resp, "row_pull");
    Reader rd(resp.data(), resp.size());
    const uint32_t n = rd.u32();
    py::array_t<float> out({static_cast<py::ssize_t>(n), static_cast<py::ssize_t>(dim)});
    std::vector<float> tmp;
    rd.vec(&tmp, static_cast<size_t>(n) * dim);
    std::memcpy(out.mutable_data(), tmp.data(), tmp.size() * sizeof(float));
    return out;
  }

  void row_push(const std::string& table, uint32_t dim, const I64& keys, const F32& grads, const std::string& spec,
                int async_flag) {
    if (static_cast<size_t>(grads.size()) != static_cast<size_t>(keys.size()) * dim)
      throw std::runtime_error("row_push: grads must be [n, dim]");
    Writer w;
    w.u8(static_cast<uint8_t>(async_flag));
    w.str(spec);
    w.str(table);
    w.u32(dim);
    w.u32(static_cast<uint32_t>(keys.size()));
    w.raw(keys.data(), static_cast<size_t>(keys.size()) * 8);
    w.f32s(grads.data(), static_cast<size_t>(grads.size()));
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_ROW_PUSH, w, &resp);
    }
    check(st, resp, "row_push");
  }

  void simple(Op op, const std::string& s) {
    Writer w;
    w.str(s);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(op, w, &resp);
    }
    check(st, resp, "request");
  }

  std::string stats() {
    Writer w;
    std::vector<uint8_t> resp;
    uint16_t st = c_.call(OP_STATS, w, &resp);
    check(st, resp, "stats");
    Reader rd(resp.data(), resp.size());
    return rd.str();
  }

  void heartbeat(uint32_t worker) {
    Writer w;
    w.u32(worker);
    std::vector<uint8_t> resp;
    check(c_.call(OP_HEARTBEAT, w, &resp), resp, "heartbeat");
  }

  void shutdown() {
    Writer w;
    std::vector<uint8_t> resp;
    c_.call(OP_SHUTDOWN, w, &resp);
  }

  uint64_t bytes_sent() const { return c_.bytes_sent(); }
  uint64_t bytes_recv() const { return c_.bytes_recv(); }

 private:
  PSClient c_;
};

py::object batch_to_dict(Batch& b, int dims, int fields) {
  py::dict d;
  const py::ssize_t n = b.n;
  if (!b.x.empty()) {
    py::array_t<float> x({n, static_cast<py::ssize_t>(dims)});
    std::memcpy(x.mutable_data(), b.x.data(), b.x.size() * 4);
    d["X"] = x;
  }
  if (!b.i.empty()) {
    py::array_t<int64_t> i({n, static_cast<py::ssize_t>(fields)});
    std::memcpy(i.mutable_data(), b.i.data(), b.i.size() * 8);
    d["I"] = i;
  }
  if (!b.v.empty()) {
    py::array_t<float> v({n, static_cast<py::ssize_t>(fields)});
    std::memcpy(v.mutable_data(), b.v.data(), b.v.size() * 4);
    d["V"] = v;
  }
  py::array_t<float> y(n);
  std::memcpy(y.mutable_data(), b.y.data(), b.y.size() * 4);
  d["Y"] = y;
  return d;
}

// ------------------------------------------------------------------ async PS (control + CPU server)
psasync::AsyncCtl* ctl_at(uintptr_t addr) { return reinterpret_cast<psasync::AsyncCtl*>(addr); }

// Owner progress thread of the asynchronous PS for CPU (fp32) shards: the same serve_loop as
// the GPU server (csrc/async_ps_gpu.cpp) with the CPU updaters of the TCP server, one updater
// per key-prefix segment [lo, hi) of the shard.
class CpuAsyncServer {
 public:
  CpuAsyncServer(uintptr_t ctl, int me, int64_t n, uintptr_t master, std::vector<uintptr_t> mbox,
                 std::vector<uintptr_t> pub, double gscale)
      : ctl_(ctl_at(ctl)), me_(me), n_(n), master_(reinterpret_cast<float*>(master)), gscale_(gscale) {
    if (static_cast<int64_t>(mbox.size()) != ctl_->world * psasync::kMbox)
      throw std::runtime_error("async PS: W x kMbox mailboxes expected");
    for (auto p : mbox) mbox_.push_back(reinterpret_cast<const float*>(p));
    for (auto p : pub) pub_.push_back(reinterpret_cast<float*>(p));
    tmp_.resize(static_cast<size_t>(n));
  }
  ~CpuAsyncServer() { stop(); }
  void add_segment(const std::string& spec, int64_t lo, int64_t hi) {
    if (lo < 0 || hi > n_ || lo >= hi) throw std::runtime_error("async PS: bad segment");
    Seg sg;
    sg.lo = lo;
    sg.hi = hi;
    sg.upd = make_updater(spec);
    sg.states.assign(static_cast<size_t>(sg.upd->n_state()), std::vector<float>(static_cast<size_t>(hi - lo), 0.f));
    segs_.push_back(std::move(sg));
  }
  void start() {
    if (segs_.empty()) throw std::runtime_error("async PS: no updater segments");
    stop_ = false;
    th_ = std::thread([this] {
      psasync::serve_loop(ctl_, me_, &stop_, [this](int w, int mslot, int slot, int64_t step) {
        const float* g = mbox_[static_cast<size_t>(w * psasync::kMbox + mslot)];
        for (int64_t i = 0; i < n_; ++i) tmp_[static_cast<size_t>(i)] = g[i] * static_cast<float>(gscale_);
        for (auto& sg : segs_)
          sg.upd->update(master_ + sg.lo, tmp_.data() + sg.lo, static_cast<size_t>(sg.hi - sg.lo), sg.states,
                         static_cast<long>(step));
        std::memcpy(pub_[static_cast<size_t>(slot)], master_, static_cast<size_t>(n_) * sizeof(float));
        applied_ += 1;
      });
    });
  }
  void stop() {
    stop_ = true;
    if (th_.joinable()) th_.join();
  }
  int64_t applied() const { return applied_; }
  // every segment's state tensors, in segment order
  py::list states() {
    py::list out;
    for (auto& sg : segs_)
      for (auto& v : sg.states) {
        py::array_t<float> a(static_cast<py::ssize_t>(v.size()));
        std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(float));
        out.append(a);
      }
    return out;
  }
  void set_states(const std::vector<F32>& st) {
    size_t k = 0;
    for (auto& sg : segs_)
      for (auto& v : sg.states) {
        if (k >= st.size()) return;
        std::memcpy(v.data(), st[k].data(), std::min<size_t>(v.size(), st[k].size()) * 4);
        ++k;
      }
  }

 private:
  struct Seg {
    int64_t lo, hi;
    std::unique_ptr<Updater> upd;
    std::vector<std::vector<float>> states;
  };
  psasync::AsyncCtl* ctl_;
  int me_;
  int64_t n_;
  float* master_;
  double gscale_;
  std::vector<Seg> segs_;
  std::vector<const float*> mbox_;
  std::vector<float*> pub_;
  std::vector<float> tmp_;
  std::atomic<bool> stop_{true};
  std::thread th_;
  int64_t applied_ = 0;
};

// Row service of the asynchronous sparse tables (ps_amd/parallel/async_rows.py): one thread per
// owner and table watching the table's control words (RowCtl below, POSIX shared memory) and
// handing every posted pull request / deposited row push to a Python callback that does the
// owner-side work (hash lookup-or-insert, lazy init, gather / row optimizer on the shard), then
// acknowledging it.  Workers never wait for each other: a pull waits for its owner's service
// only, a push not at all (2-deep mailboxes).
//
// int64 words: [magic, world, stop, pad] req[W][W] resp[W][W] nreq[W][W] pseq[W][W] pack[W][W]
// npush[W][W][kMbox]  -- [o][w] = owner o, worker w
constexpr int64_t kRowMagic = 0x524f57535256ll;  // "ROWSRV"
inline int64_t row_ctl_words(int64_t W) { return 4 + 5 * W * W + W * W * psasync::kMbox; }

class RowPoller {
 public:
  RowPoller(uintptr_t ctl, int me, py::object cb) : b_(reinterpret_cast<int64_t*>(ctl)), me_(me), cb_(cb) {
    if (psasync::ld(b_) != kRowMagic) throw std::runtime_error("row control block not initialised");
    W_ = b_[1];
  }
  ~RowPoller() { stop(); }
  void start() {
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

 private:
  int64_t* w(int k, int64_t o, int64_t wk) const { return b_ + 4 + k * W_ * W_ + o * W_ + wk; }
  int64_t* npush(int64_t o, int64_t wk, int m) const {
    return b_ + 4 + 5 * W_ * W_ + (o * W_ + wk) * psasync::kMbox + m;
  }
  void run() {
    psasync::Backoff idle;
    while (!stop_.load(std::memory_order_acquire) && psasync::ld(b_ + 2) == 0) {
      bool did = false;
      for (int64_t k = 0; k < W_; ++k) {
        const int64_t rq = psasync::ld(w(0, me_, k)), rs = psasync::ld(w(1, me_, k));
        if (rq > rs) {
          if (!call("pull", k, psasync::ld(w(2, me_, k)), 0)) return;
          psasync::st(w(1, me_, k), rq);
          did = true;
        }
        const int64_t ps = psasync::ld(w(3, me_, k)), pa = psasync::ld(w(4, me_, k));
        if (ps > pa) {
          const int m = static_cast<int>(pa % psasync::kMbox);
          if (!call("push", k, psasync::ld(npush(me_, k, m)), m)) return;
          psasync::st(w(4, me_, k), pa + 1);
          did = true;
        }
      }
      if (did) idle.n = 0;
      else idle();
    }
  }
  bool call(const char* op, int64_t worker, int64_t n, int m) {
    py::gil_scoped_acquire gil;
    try {
      cb_(op, worker, n, m);
      return true;
    } catch (py::error_already_set& e) {
      std::lock_guard<std::mutex> g(mu_);
      err_ = std::string(op) + ": " + e.what();
      psasync::st(b_ + 2, 1);  // stop every service of the table: workers time out loudly
      return false;
    }
  }
  int64_t* b_;
  int64_t W_ = 1;
  int me_;
  py::object cb_;
  std::atomic<bool> stop_{true};
  std::thread th_;
  std::mutex mu_;
  std::string err_;
};

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "ps_amd native CPU runtime: TCP parameter server/client, id map, threaded batch loader";

  py::class_<PSServer>(m, "PSServer")
      .def(py::init<int, int, const std::string&, int, double>(), py::arg("port") = 0, py::arg("workers") = 1,
           py::arg("mode") = "bsp", py::arg("staleness") = 0, py::arg("barrier_timeout_s") = 600.0)
      .def("start", &PSServer::start)
      .def("stop", &PSServer::stop, py::call_guard<py::gil_scoped_release>())
      .def("wait", &PSServer::wait, py::call_guard<py::gil_scoped_release>())
      .def("set_bind_any", &PSServer::set_bind_any)
      .def_property_readonly("port", &PSServer::port)
      .def_property_readonly("generation", &PSServer::generation)
      .def_property_readonly("updates", &PSServer::updates);

  py::class_<Client>(m, "PSClient")
      .def(py::init<const std::string&, int, double>(), py::arg("host"), py::arg("port"),
           py::arg("timeout_s") = 30.0)
      .def("get", &Client::get)
      .def("get_list", &Client::get_list)
      .def("upsert", &Client::upsert, py::arg("key"), py::arg("value"), py::arg("replace") = false)
      .def("upsert_list", &Client::upsert_list, py::arg("keys"), py::arg("values"), py::arg("replace") = false)
      .def("push", &Client::push, py::arg("keys"), py::arg("grads"), py::arg("spec"), py::arg("async_flag") = 0)
      .def("barrier", &Client::barrier, py::arg("worker") = 0)
      .def("clock", &Client::clock)
      .def("rendezvous", &Client::rendezvous, py::arg("worker") = 0)
      .def("row_pull", &Client::row_pull, py::arg("table"), py::arg("dim"), py::arg("keys"), py::arg("lo"),
           py::arg("hi"), py::arg("seed"))
      .def("row_push", &Client::row_push, py::arg("table"), py::arg("dim"), py::arg("keys"), py::arg("grads"),
           py::arg("spec"), py::arg("async_flag") = 0)
      .def("register_updater", [](Client& c, const std::string& s) { c.simple(OP_REGISTER, s); })
      .def("save", [](Client& c, const std::string& p) { c.simple(OP_SAVE, p); })
      .def("load", [](Client& c, const std::string& p) { c.simple(OP_LOAD, p); })
      .def("stats", &Client::stats)
      .def("heartbeat", &Client::heartbeat)
      .def("shutdown", &Client::shutdown)
      .def_property_readonly("bytes_sent", &Client::bytes_sent)
      .def_property_readonly("bytes_recv", &Client::bytes_recv);

  // async-PS control block operations (blocking ones release the GIL); ``addr`` is the address
  // of a psasync::AsyncCtl in shared memory (see csrc/include/async_ctl.h)
  auto a = m.def_submodule("async_ctl", "asynchronous parameter-server control block");
  a.attr("SIZE") = sizeof(psasync::AsyncCtl);
  a.attr("MAX_WORLD") = psasync::kMaxW;
  a.attr("SLOTS") = psasync::kSlots;
  a.def("init", [](uintptr_t addr, int64_t world) {
    if (world < 1 || world > psasync::kMaxW) throw std::runtime_error("async PS world out of range");
    psasync::init(ctl_at(addr), world);
  });
  a.def("valid", [](uintptr_t addr) { return psasync::ld(&ctl_at(addr)->magic) == psasync::kMagic; });
  a.def("wait_free", [](uintptr_t addr, int o, int w, double timeout_s) {
    auto* c = ctl_at(addr);
    const auto t0 = std::chrono::steady_clock::now();
    psasync::Backoff bo;
    while (psasync::ld(&c->ack[o][w]) < psasync::ld(&c->seq[o][w])) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
        throw std::runtime_error("async PS: owner did not drain the mailbox in time (dead server?)");
      bo();
    }
  }, py::call_guard<py::gil_scoped_release>());
  // wait until owner o has APPLIED at least ``target`` pushes of worker w: before queueing push
  // number target + 1 into the 1-deep mailbox the worker gates on its OWN push count, not on
  // seq (which the completion thread bumps only after the previous copy landed)
  a.def("wait_ack", [](uintptr_t addr, int o, int w, int64_t target, double timeout_s) {
    auto* c = ctl_at(addr);
    const auto t0 = std::chrono::steady_clock::now();
    psasync::Backoff bo;
    while (psasync::ld(&c->ack[o][w]) < target) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
        throw std::runtime_error("async PS: owner did not apply the previous push in time (dead server?)");
      bo();
    }
  }, py::call_guard<py::gil_scoped_release>());
  // checkpoint restore: the owner's update count (Adam bias correction continues from it)
  a.def("set_version", [](uintptr_t addr, int o, int64_t v) { psasync::st(&ctl_at(addr)->version[o], v); });
  a.def("bump_seq", [](uintptr_t addr, int o, int w) { return psasync::add(&ctl_at(addr)->seq[o][w], 1); });
  a.def("bump_clock", [](uintptr_t addr, int w) { return psasync::add(&ctl_at(addr)->clock[w], 1); });
  a.def("wait_min_ack", [](uintptr_t addr, int64_t target, double timeout_s) {
    auto* c = ctl_at(addr);
    const auto t0 = std::chrono::steady_clock::now();
    psasync::Backoff bo;
    while (psasync::min_ack(c) < target) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
        throw std::runtime_error("async PS: staleness gate timed out (dead worker?)");
      bo();
    }
  }, py::call_guard<py::gil_scoped_release>());
  a.def("pin", [](uintptr_t addr, int o) { return psasync::pin(ctl_at(addr), o); },
        py::call_guard<py::gil_scoped_release>());
  a.def("unpin", [](uintptr_t addr, int o, int s) { psasync::unpin(ctl_at(addr), o, s); });
  a.def("set_stop", [](uintptr_t addr, int64_t v) { psasync::st(&ctl_at(addr)->stop, v); });
  a.def("MBOX", []() { return psasync::kMbox; });

  // generic shared-memory words (acquire / release) for the async row tables
  auto sh = m.def_submodule("shm", "int64 words in shared memory");
  sh.def("ld", [](uintptr_t p) { return psasync::ld(reinterpret_cast<int64_t*>(p)); });
  sh.def("st", [](uintptr_t p, int64_t v) { psasync::st(reinterpret_cast<int64_t*>(p), v); });
  sh.def("add", [](uintptr_t p, int64_t v) { return psasync::add(reinterpret_cast<int64_t*>(p), v); });
  sh.def("wait_ge", [](std::vector<uintptr_t> ps, int64_t v, uintptr_t stop_word, double timeout_s) {
    const auto t0 = std::chrono::steady_clock::now();
    psasync::Backoff bo;
    for (;;) {
      bool ok = true;
      for (auto p : ps) ok = ok && psasync::ld(reinterpret_cast<int64_t*>(p)) >= v;
      if (ok) return;
      if (stop_word && psasync::ld(reinterpret_cast<int64_t*>(stop_word)) != 0)
        throw std::runtime_error("async rows: the service of this table stopped (owner error)");
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
        throw std::runtime_error("async rows: timed out waiting for an owner (dead rank?)");
      bo();
    }
  }, py::call_guard<py::gil_scoped_release>());
  auto rw = m.def_submodule("rows", "asynchronous sparse-row tables: control block + service thread");
  rw.def("ctl_size", [](int64_t W) { return row_ctl_words(W) * 8; });
  rw.def("ctl_init", [](uintptr_t addr, int64_t W) {
    int64_t* b = reinterpret_cast<int64_t*>(addr);
    for (int64_t i = 0; i < row_ctl_words(W); ++i) b[i] = 0;
    b[1] = W;
    psasync::st(b, kRowMagic);
  });
  py::class_<RowPoller>(rw, "Service")
      .def(py::init<uintptr_t, int, py::object>())
      .def("start", &RowPoller::start)
      .def("stop", &RowPoller::stop, py::call_guard<py::gil_scoped_release>())
      .def("error", &RowPoller::error);
  a.def("snapshot", [](uintptr_t addr) {
    auto* c = ctl_at(addr);
    const int W = static_cast<int>(c->world);
    py::dict d;
    py::list clock, version, seq, ack;
    for (int i = 0; i < W; ++i) {
      clock.append(psasync::ld(&c->clock[i]));
      version.append(psasync::ld(&c->version[i]));
      py::list sr, ar;
      for (int j = 0; j < W; ++j) {
        sr.append(psasync::ld(&c->seq[i][j]));
        ar.append(psasync::ld(&c->ack[i][j]));
      }
      seq.append(sr);
      ack.append(ar);
    }
    d["clock"] = clock;
    d["version"] = version;
    d["seq"] = seq;
    d["ack"] = ack;
    return d;
  });
  py::class_<CpuAsyncServer>(m, "CpuAsyncServer")
      .def(py::init<uintptr_t, int, int64_t, uintptr_t, std::vector<uintptr_t>, std::vector<uintptr_t>, double>())
      .def("add_segment", &CpuAsyncServer::add_segment)
      .def("start", &CpuAsyncServer::start)
      .def("stop", &CpuAsyncServer::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("applied", &CpuAsyncServer::applied)
      .def("states", &CpuAsyncServer::states)
      .def("set_states", &CpuAsyncServer::set_states);

  py::class_<IdMap>(m, "IdMap")
      .def(py::init<int64_t>())
      .def("lookup",
           [](IdMap& self, const I64& ids, bool insert) {
             py::array_t<int64_t> out(ids.size());
             {
               py::gil_scoped_release r;
               self.lookup(ids.data(), ids.size(), insert, out.mutable_data());
             }
             return out;
           },
           py::arg("ids"), py::arg("insert") = true)
      .def("size", &IdMap::size)
      .def("items", &IdMap::items)
      .def("restore", [](IdMap& self, const I64& ids, const I64& slots) {
        if (ids.size() != slots.size()) throw std::runtime_error("ids/slots length mismatch");
        self.restore(ids.data(), slots.data(), ids.size());
      });

  py::class_<BatchReader>(m, "BatchReader")
      .def(py::init<const std::string&, const std::string&, int, int, int, int, int, int, int, bool>(),
           py::arg("path"), py::arg("format"), py::arg("batch"), py::arg("dims") = 0, py::arg("fields") = 0,
           py::arg("offset") = 0, py::arg("step") = 1, py::arg("threads") = 2, py::arg("depth") = 4,
           py::arg("drop_last") = false)
      .def("next",
           [](BatchReader& self, double timeout) -> py::object {
             Batch b;
             bool ok;
             {
               py::gil_scoped_release r;
               ok = self.next(&b, timeout);
             }
             if (!ok) return py::none();
             return batch_to_dict(b, self.dims(), self.fields());
           },
           py::arg("timeout_s") = 3.0)
      .def("has_next", &BatchReader::has_next, py::call_guard<py::gil_scoped_release>())
      .def("reset", &BatchReader::reset, py::call_guard<py::gil_scoped_release>());
}
