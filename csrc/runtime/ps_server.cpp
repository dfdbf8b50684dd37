// Native TCP parameter server + client (dedicated-server topology).
//
// Reference: net/PServer.java (gRPC service, server-local KVStore, updater registry keyed by
// spec string, BSP via barrier + update thread, ASP apply-on-push), net/PSClient.java and
// net/PSRouterClient.java.  This is the CPU/TCP-loopback data plane used by BASELINE config 1
// ("2-layer MLP, 1 server + 2 workers") and by any deployment with dedicated server
// processes; the GPU hot path is the co-located collective PS (ps_amd/parallel/colocated.py).
//
// Semantics, with the reference's races fixed:
//   BSP  push = accumulate (sum + count) per key; barrier = generation barrier over W workers;
//        the LAST arriving worker applies every dirty key with grad = sum / count, clears the
//        accumulators (Q3) and opens the next generation; pushes are acknowledged before the
//        worker can reach the barrier (Q2); nobody leaves a barrier before the update is done (Q1).
//   SSP  push applies immediately; ``clock(worker, c)`` blocks while c - min_clock > staleness.
//   ASP  push applies immediately; barrier returns at once (reference isPsAsync).
// Concurrency: one thread per connection; keys sharded over 64 mutex stripes (the reference
// funnels everything through one synchronized KVStore, Q19).
#include "ps_server.h"

#include <netdb.h>
#include <poll.h>

#include <algorithm>
#include <chrono>
#include <fstream>
#include <sstream>

namespace psnative {

// ------------------------------------------------------------------------------- server
PSServer::PSServer(int port, int workers, const std::string& mode, int staleness, double barrier_timeout_s)
    : port_(port), workers_(workers), staleness_(staleness), barrier_timeout_s_(barrier_timeout_s) {
  if (mode == "bsp") mode_ = Mode::BSP;
  else if (mode == "ssp") mode_ = Mode::SSP;
  else if (mode == "asp") mode_ = Mode::ASP;
  else throw std::runtime_error("mode must be bsp|ssp|asp");
  if (workers < 1) throw std::runtime_error("workers must be >= 1");
  clocks_.assign(static_cast<size_t>(workers), 0);
}

PSServer::~PSServer() { stop(); }

void PSServer::start() {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw std::runtime_error("socket() failed");
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (bind_any_) addr.sin_addr.s_addr = htonl(INADDR_ANY);
  addr.sin_port = htons(static_cast<uint16_t>(port_));
  if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
    ::close(listen_fd_);
    throw std::runtime_error("bind() failed on port " + std::to_string(port_));
  }
  socklen_t len = sizeof(addr);
  getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&addr), &len);
  port_ = ntohs(addr.sin_port);
  if (::listen(listen_fd_, 128) != 0) throw std::runtime_error("listen() failed");
  running_ = true;
  accept_thread_ = std::thread([this] { accept_loop(); });
}

void PSServer::stop() {
  if (!running_.exchange(false)) return;
  {
    std::lock_guard<std::mutex> g(barrier_mu_);
    barrier_cv_.notify_all();
  }
  // wake the acceptor, join it, and only then close/reset the fd: closing it while the
  // acceptor still polls it raced on listen_fd_ and could hand a reused fd number to poll()
  // (found by the TSan build, scripts/tsan_native.sh)
  if (listen_fd_ >= 0) ::shutdown(listen_fd_, SHUT_RDWR);
  if (accept_thread_.joinable()) accept_thread_.join();
  if (listen_fd_ >= 0) {
    ::close(listen_fd_);
    listen_fd_ = -1;
  }
  std::vector<std::thread> ts;
  {
    std::lock_guard<std::mutex> g(conn_mu_);
    for (int fd : conn_fds_) ::shutdown(fd, SHUT_RDWR);
    ts.swap(conn_threads_);
  }
  for (auto& t : ts)
    if (t.joinable()) t.join();
}

void PSServer::wait() {
  std::unique_lock<std::mutex> g(stop_mu_);
  stop_cv_.wait(g, [this] { return shutdown_requested_.load() || !running_.load(); });
}

void PSServer::accept_loop() {
  while (running_) {
    pollfd p{listen_fd_, POLLIN, 0};
    int r = ::poll(&p, 1, 200);
    if (r <= 0) continue;
    int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) continue;
    tune_socket(fd);
    std::lock_guard<std::mutex> g(conn_mu_);
    conn_fds_.push_back(fd);
    conn_threads_.emplace_back([this, fd] { serve(fd); });
  }
}

PSServer::Stripe& PSServer::stripe(const std::string& key) {
  return stripes_[std::hash<std::string>{}(key) % kStripes];
}

RowTable& PSServer::row_table(const std::string& name, uint32_t dim) {
  std::lock_guard<std::mutex> g(rt_mu_);
  auto& t = row_tables_[name];
  if (!t) {
    t = std::make_unique<RowTable>();
    t->dim = dim;
  }
  if (t->dim != dim) throw std::runtime_error("row table " + name + ": dim mismatch");
  return *t;
}

const Updater* PSServer::updater(const std::string& spec) {
  std::lock_guard<std::mutex> g(upd_mu_);
  auto it = updaters_.find(spec);
  if (it != updaters_.end()) return it->second.get();
  auto u = make_updater(spec);
  const Updater* raw = u.get();
  updaters_[spec] = std::move(u);
  return raw;
}

void PSServer::apply(Entry& e, const std::string& key, const float* g, size_t n, const Updater* u) {
  if (e.states.size() != static_cast<size_t>(u->n_state())) {
    e.states.assign(static_cast<size_t>(u->n_state()), std::vector<float>(e.w.size(), 0.f));
  }
  e.t += 1;
  u->update(e.w.data(), g, std::min(n, e.w.size()), e.states, e.t);
  updates_.fetch_add(1);
}

void PSServer::serve(int fd) {
  std::vector<uint8_t> payload;
  while (running_) {
    uint32_t hdr[2];
    uint8_t op;
    if (!recv_all(fd, &hdr[0], 4)) break;
    if (hdr[0] != kMagic) break;
    if (!recv_all(fd, &op, 1) || !recv_all(fd, &hdr[1], 4)) break;
    payload.resize(hdr[1]);
    if (hdr[1] && !recv_all(fd, payload.data(), hdr[1])) break;
    Writer out;
    uint16_t status = ST_OK;
    try {
      Reader in(payload.data(), payload.size());
      status = handle(static_cast<Op>(op), in, out);
    } catch (const std::exception& ex) {
      status = ST_ERR;
      out.buf.clear();
      out.str(ex.what());
    }
    Writer resp;
    resp.u32(kMagic);
    resp.u16(status);
    resp.u32(static_cast<uint32_t>(out.buf.size()));
    if (!send_all(fd, resp.buf.data(), resp.buf.size())) break;
    if (!out.buf.empty() && !send_all(fd, out.buf.data(), out.buf.size())) break;
    if (op == OP_SHUTDOWN) {
      shutdown_requested_ = true;
      stop_cv_.notify_all();
    }
  }
  ::close(fd);
}

uint16_t PSServer::handle(Op op, Reader& in, Writer& out) {
  requests_.fetch_add(1);
  switch (op) {
    case OP_GET: {
      const std::string key = in.str();
      auto& s = stripe(key);
      std::lock_guard<std::mutex> g(s.mu);
      auto it = s.map.find(key);
      if (it == s.map.end()) return ST_NOT_FOUND;  // reference 204 "null weights"
      out.mat(it->second.rows, it->second.cols, it->second.w.data());
      return ST_OK;
    }
    case OP_GET_LIST: {
      const uint32_t n = in.u32();
      out.u32(n);
      for (uint32_t i = 0; i < n; ++i) {
        const std::string key = in.str();
        auto& s = stripe(key);
        std::lock_guard<std::mutex> g(s.mu);
        auto it = s.map.find(key);
        if (it == s.map.end()) {
          out.u8(0);
        } else {
          out.u8(1);
          out.mat(it->second.rows, it->second.cols, it->second.w.data());
        }
      }
      return ST_OK;
    }
    case OP_UPSERT:
    case OP_UPSERT_LIST: {
      const uint8_t replace = in.u8();
      const uint32_t n = op == OP_UPSERT ? 1u : in.u32();
      if (op == OP_UPSERT_LIST) out.u32(n);
      for (uint32_t i = 0; i < n; ++i) {
        const std::string key = in.str();
        Matrix m = in.mat();
        auto& s = stripe(key);
        std::lock_guard<std::mutex> g(s.mu);
        auto it = s.map.find(key);
        const bool existed = it != s.map.end();
        if (!existed || replace) {
          Entry& e = s.map[key];
          e.rows = m.rows;
          e.cols = m.cols;
          e.w = std::move(m.data);
          e.acc.clear();
          e.states.clear();
          it = s.map.find(key);
        }
        // first writer wins (net/PServer.java:119-141): the stored value is returned
        out.u8(existed && !replace ? 1 : 0);
        out.mat(it->second.rows, it->second.cols, it->second.w.data());
      }
      return ST_OK;
    }
    case OP_PUSH: {
      const uint8_t async_flag = in.u8();
      const std::string spec = in.str();
      const Updater* u = updater(spec);
      const uint32_t n = in.u32();
      const bool apply_now = mode_ != Mode::BSP || async_flag == 2;  // 2 = force apply
      for (uint32_t i = 0; i < n; ++i) {
        const std::string key = in.str();
        Matrix g = in.mat();
        auto& s = stripe(key);
        std::lock_guard<std::mutex> lk(s.mu);
        auto it = s.map.find(key);
        if (it == s.map.end()) throw std::runtime_error("push to unknown key " + key);
        Entry& e = it->second;
        if (g.data.size() != e.w.size()) throw std::runtime_error("push size mismatch for " + key);
        if (apply_now) {
          apply(e, key, g.data.data(), g.data.size(), u);
        } else {
          if (e.acc.size() != e.w.size()) e.acc.assign(e.w.size(), 0.f);
          for (size_t j = 0; j < g.data.size(); ++j) e.acc[j] += g.data[j];
          e.count += 1;
          e.pending = u;
          s.dirty.insert(key);
        }
      }
      pushes_.fetch_add(n);
      return ST_OK;
    }
    case OP_BARRIER: {
      const uint32_t worker = in.u32();
      (void)worker;
      if (mode_ != Mode::BSP) {
        out.u64(generation_.load());
        return ST_OK;
      }
      std::unique_lock<std::mutex> g(barrier_mu_);
      const uint64_t gen = generation_.load();
      arrived_ += 1;
      if (arrived_ == workers_) {
        apply_pending();  // every worker has pushed and been acknowledged
        arrived_ = 0;
        generation_.fetch_add(1);
        barrier_cv_.notify_all();
      } else {
        const bool ok = barrier_cv_.wait_for(g, std::chrono::duration<double>(barrier_timeout_s_),
                                             [&] { return generation_.load() != gen || !running_.load(); });
        if (!ok) {
          arrived_ -= 1;
          return ST_TIMEOUT;  // a dead worker no longer hangs everyone forever
        }
      }
      out.u64(generation_.load());
      return ST_OK;
    }
    case OP_RENDEZVOUS: {
      // every worker meets here in any consistency mode (Trainer.resume: all present -> worker
      // 0 reloads the store -> all present again, so nobody pulls or pushes across the reload)
      in.u32();
      std::unique_lock<std::mutex> g(barrier_mu_);
      const uint64_t gen = rv_gen_;
      rv_arrived_ += 1;
      if (rv_arrived_ == workers_) {
        rv_arrived_ = 0;
        rv_gen_ += 1;
        barrier_cv_.notify_all();
      } else {
        const bool ok = barrier_cv_.wait_for(g, std::chrono::duration<double>(barrier_timeout_s_),
                                             [&] { return rv_gen_ != gen || !running_.load(); });
        if (!ok) {
          rv_arrived_ -= 1;
          return ST_TIMEOUT;
        }
      }
      out.u64(rv_gen_);
      return ST_OK;
    }
    case OP_CLOCK: {
      const uint32_t worker = in.u32();
      const uint64_t c = in.u64();
      if (worker >= clocks_.size()) throw std::runtime_error("worker id out of range");
      std::unique_lock<std::mutex> g(barrier_mu_);
      clocks_[worker] = c;
      barrier_cv_.notify_all();
      auto min_clock = [&] { return *std::min_element(clocks_.begin(), clocks_.end()); };
      if (mode_ == Mode::SSP) {
        const bool ok = barrier_cv_.wait_for(g, std::chrono::duration<double>(barrier_timeout_s_), [&] {
          return static_cast<int64_t>(c) - static_cast<int64_t>(min_clock()) <= staleness_ || !running_.load();
        });
        if (!ok) return ST_TIMEOUT;
      }
      out.u64(min_clock());
      return ST_OK;
    }
    case OP_ROW_PULL: {
      // str table | u32 dim | f32 lo | f32 hi | u64 seed | u32 n | i64 keys[n]  ->  f32 rows[n*dim]
      const std::string name = in.str();
      const uint32_t dim = in.u32();
      const float lo = in.f32(), hi = in.f32();
      const uint64_t seed = in.u64();
      const uint32_t n = in.u32();
      std::vector<int64_t> keys;
      in.vec(&keys, n);
      RowTable& t = row_table(name, dim);
      std::vector<float> rows(static_cast<size_t>(n) * dim);
      {
        std::lock_guard<std::mutex> g(t.mu);
        for (uint32_t i = 0; i < n; ++i) {
          auto it = t.rows.find(keys[i]);
          if (it == t.rows.end()) {
            Entry e;
            e.rows = 1;
            e.cols = dim;
            e.w.resize(dim, 0.f);
            if (lo != 0.f || hi != 0.f)
              for (uint32_t c = 0; c < dim; ++c)  // word c%4 of the call for c/4 (as the HIP kernel)
                e.w[c] = lo + (hi - lo) * philox_u01(seed, c / 4, c % 4, static_cast<uint64_t>(keys[i]));
            it = t.rows.emplace(keys[i], std::move(e)).first;
          }
          std::memcpy(rows.data() + static_cast<size_t>(i) * dim, it->second.w.data(), dim * sizeof(float));
        }
      }
      out.u32(n);
      out.f32s(rows.data(), rows.size());
      return ST_OK;
    }
    case OP_ROW_PUSH: {
      // u8 async | str spec | str table | u32 dim | u32 n | i64 keys[n] | f32 grads[n*dim]
      const uint8_t async_flag = in.u8();
      const std::string spec = in.str();
      const std::string name = in.str();
      const uint32_t dim = in.u32();
      const uint32_t n = in.u32();
      std::vector<int64_t> keys;
      std::vector<float> grads;
      in.vec(&keys, n);
      in.vec(&grads, static_cast<size_t>(n) * dim);
      const Updater* u = updater(spec);
      const bool apply_now = mode_ != Mode::BSP || async_flag == 2;
      RowTable& t = row_table(name, dim);
      std::lock_guard<std::mutex> g(t.mu);
      for (uint32_t i = 0; i < n; ++i) {
        auto it = t.rows.find(keys[i]);
        if (it == t.rows.end()) throw std::runtime_error("push to a row that was never pulled: " + name);
        Entry& e = it->second;
        const float* gi = grads.data() + static_cast<size_t>(i) * dim;
        if (apply_now) {
          apply(e, name, gi, dim, u);
        } else {
          if (e.acc.size() != dim) e.acc.assign(dim, 0.f);
          for (uint32_t c = 0; c < dim; ++c) e.acc[c] += gi[c];
          e.count += 1;
          e.pending = u;
          t.dirty.insert(keys[i]);
        }
      }
      pushes_.fetch_add(n);
      return ST_OK;
    }
    case OP_REGISTER: {
      updater(in.str());
      return ST_OK;
    }
    case OP_STATS: {
      std::ostringstream os;
      size_t keys = 0, floats = 0;
      for (auto& s : stripes_) {
        std::lock_guard<std::mutex> g(s.mu);
        keys += s.map.size();
        for (auto& kv : s.map) floats += kv.second.w.size();
      }
      os << "{\"keys\":" << keys << ",\"floats\":" << floats << ",\"requests\":" << requests_.load()
         << ",\"pushes\":" << pushes_.load() << ",\"updates\":" << updates_.load()
         << ",\"generation\":" << generation_.load() << ",\"workers\":" << workers_ << ",\"mode\":\""
         << (mode_ == Mode::BSP ? "bsp" : mode_ == Mode::SSP ? "ssp" : "asp") << "\",\"heartbeats\":"
         << heartbeats_.load() << "}";
      out.str(os.str());
      return ST_OK;
    }
    case OP_SAVE: {
      save(in.str());
      return ST_OK;
    }
    case OP_LOAD: {
      load(in.str());
      return ST_OK;
    }
    case OP_HEARTBEAT: {
      in.u32();
      heartbeats_.fetch_add(1);
      return ST_OK;
    }
    case OP_SHUTDOWN:
      return ST_OK;
  }
  return ST_BAD;
}

void PSServer::apply_pending() {
  for (auto& s : stripes_) {
    std::lock_guard<std::mutex> g(s.mu);
    for (const auto& key : s.dirty) {
      Entry& e = s.map[key];
      if (e.count == 0 || e.pending == nullptr) continue;
      const float inv = 1.f / static_cast<float>(e.count);
      for (auto& v : e.acc) v *= inv;
      apply(e, key, e.acc.data(), e.acc.size(), e.pending);
      std::fill(e.acc.begin(), e.acc.end(), 0.f);  // Q3: accumulators cleared every round
      e.count = 0;
    }
    s.dirty.clear();
  }
  std::lock_guard<std::mutex> g(rt_mu_);
  for (auto& kv : row_tables_) {
    RowTable& t = *kv.second;
    std::lock_guard<std::mutex> lk(t.mu);
    for (const int64_t key : t.dirty) {
      Entry& e = t.rows[key];
      if (e.count == 0 || e.pending == nullptr) continue;
      // rows: the gradient of the mean loss over ALL workers' samples, i.e. sum / W even when
      // only some workers touched the row (the reference divides by the pushes it happened to
      // receive, store/KVStore.java:192-200 -- Q3); identical to the co-located path's 1/W
      const float inv = 1.f / static_cast<float>(workers_);
      for (auto& v : e.acc) v *= inv;
      apply(e, kv.first, e.acc.data(), e.acc.size(), e.pending);
      std::fill(e.acc.begin(), e.acc.end(), 0.f);
      e.count = 0;
    }
    t.dirty.clear();
  }
}

// checkpoint: text header + raw floats per key (weights + optimizer states + step)
void PSServer::save(const std::string& path) {
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  Writer w;
  uint32_t nkeys = 0;
  for (auto& s : stripes_) {
    std::lock_guard<std::mutex> g(s.mu);
    for (auto& kv : s.map) {
      const Entry& e = kv.second;
      w.str(kv.first);
      w.u32(e.rows);
      w.u32(e.cols);
      w.u64(static_cast<uint64_t>(e.t));
      w.f32s(e.w.data(), e.w.size());
      w.u32(static_cast<uint32_t>(e.states.size()));
      for (auto& st : e.states) w.f32s(st.data(), st.size());
      ++nkeys;
    }
  }
  // sparse row tables follow the dense keys: u32 ntables | per table: str name | u32 dim |
  // u32 nrows | per row: i64 key | u64 t | f32[dim] w | u32 nstates | f32[dim] per state
  {
    std::lock_guard<std::mutex> g(rt_mu_);
    w.u32(static_cast<uint32_t>(row_tables_.size()));
    for (auto& kv : row_tables_) {
      RowTable& t = *kv.second;
      std::lock_guard<std::mutex> lk(t.mu);
      w.str(kv.first);
      w.u32(t.dim);
      w.u32(static_cast<uint32_t>(t.rows.size()));
      for (auto& r : t.rows) {
        w.u64(static_cast<uint64_t>(r.first));
        w.u64(static_cast<uint64_t>(r.second.t));
        w.f32s(r.second.w.data(), r.second.w.size());
        w.u32(static_cast<uint32_t>(r.second.states.size()));
        for (auto& st : r.second.states) w.f32s(st.data(), st.size());
      }
    }
  }
  Writer h;
  h.u32(kMagic);
  h.u32(nkeys);
  h.u64(generation_.load());
  f.write(reinterpret_cast<const char*>(h.buf.data()), static_cast<std::streamsize>(h.buf.size()));
  f.write(reinterpret_cast<const char*>(w.buf.data()), static_cast<std::streamsize>(w.buf.size()));
}

void PSServer::load(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  Reader r(buf.data(), buf.size());
  if (r.u32() != kMagic) throw std::runtime_error("bad checkpoint magic");
  const uint32_t nkeys = r.u32();
  generation_ = r.u64();
  for (uint32_t i = 0; i < nkeys; ++i) {
    const std::string key = r.str();
    Entry e;
    e.rows = r.u32();
    e.cols = r.u32();
    e.t = static_cast<long>(r.u64());
    const size_t n = static_cast<size_t>(e.rows) * e.cols;
    Matrix m;
    e.w.resize(n);
    for (size_t j = 0; j < n; ++j) {
      uint32_t bits = r.u32();
      std::memcpy(&e.w[j], &bits, 4);
    }
    const uint32_t ns = r.u32();
    e.states.assign(ns, std::vector<float>(n));
    for (auto& st : e.states)
      for (size_t j = 0; j < n; ++j) {
        uint32_t bits = r.u32();
        std::memcpy(&st[j], &bits, 4);
      }
    auto& s = stripe(key);
    std::lock_guard<std::mutex> g(s.mu);
    s.map[key] = std::move(e);
  }
  if (r.done()) return;  // checkpoint without row tables
  const uint32_t ntables = r.u32();
  for (uint32_t ti = 0; ti < ntables; ++ti) {
    const std::string name = r.str();
    const uint32_t dim = r.u32();
    const uint32_t nrows = r.u32();
    RowTable& t = row_table(name, dim);
    std::lock_guard<std::mutex> lk(t.mu);
    t.rows.clear();
    t.dirty.clear();
    for (uint32_t i = 0; i < nrows; ++i) {
      const int64_t key = static_cast<int64_t>(r.u64());
      Entry e;
      e.rows = 1;
      e.cols = dim;
      e.t = static_cast<long>(r.u64());
      r.vec(&e.w, dim);
      const uint32_t ns = r.u32();
      e.states.assign(ns, std::vector<float>());
      for (auto& st : e.states) r.vec(&st, dim);
      t.rows.emplace(key, std::move(e));
    }
  }
}

// ------------------------------------------------------------------------------- client
PSClient::PSClient(const std::string& host, int port, double timeout_s) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("cannot resolve " + host);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  while (true) {
    fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (::connect(fd_, res->ai_addr, res->ai_addrlen) == 0) break;
    ::close(fd_);
    fd_ = -1;
    if (std::chrono::steady_clock::now() > deadline) {
      freeaddrinfo(res);
      throw std::runtime_error("cannot connect to " + host + ":" + std::to_string(port));
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  freeaddrinfo(res);
  tune_socket(fd_);
}

PSClient::~PSClient() {
  if (fd_ >= 0) ::close(fd_);
}

uint16_t PSClient::call(Op op, const Writer& req, std::vector<uint8_t>* resp) {
  std::lock_guard<std::mutex> g(mu_);
  Writer h;
  h.u32(kMagic);
  h.u8(op);
  h.u32(static_cast<uint32_t>(req.buf.size()));
  if (!send_all(fd_, h.buf.data(), h.buf.size()) ||
      (!req.buf.empty() && !send_all(fd_, req.buf.data(), req.buf.size())))
    throw std::runtime_error("PS connection lost (send)");
  uint32_t magic, len;
  uint16_t status;
  if (!recv_all(fd_, &magic, 4) || magic != kMagic || !recv_all(fd_, &status, 2) || !recv_all(fd_, &len, 4))
    throw std::runtime_error("PS connection lost (recv)");
  std::vector<uint8_t> discard;
  std::vector<uint8_t>* dst = resp ? resp : &discard;  // null resp: payload read and dropped
  dst->resize(len);
  if (len && !recv_all(fd_, dst->data(), len)) throw std::runtime_error("PS connection lost (payload)");
  bytes_sent_ += h.buf.size() + req.buf.size();
  bytes_recv_ += 10 + len;
  return status;
}

}  // namespace psnative
