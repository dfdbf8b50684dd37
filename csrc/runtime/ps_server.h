#pragma once
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "ps_updaters.h"
#include "ps_wire.h"

namespace psnative {

struct Entry {
  uint32_t rows = 0, cols = 0;
  std::vector<float> w;
  std::vector<float> acc;  // BSP gradient accumulator
  uint32_t count = 0;      // pushes accumulated this round
  const Updater* pending = nullptr;
  std::vector<std::vector<float>> states;  // optimizer state (m/v, z/n, h, momentum)
  long t = 0;                              // updates applied to this key
};

// Sparse row table (embedding / wide rows): int64 key -> dim floats, created on first pull
// with a deterministic init keyed by (seed, key).
struct RowTable {
  uint32_t dim = 0;
  std::mutex mu;
  std::unordered_map<int64_t, Entry> rows;
  std::unordered_set<int64_t> dirty;
};

class PSServer {
 public:
  enum class Mode { BSP, SSP, ASP };
  PSServer(int port, int workers, const std::string& mode, int staleness, double barrier_timeout_s);
  ~PSServer();
  void start();
  void stop();
  void wait();
  int port() const { return port_; }
  void set_bind_any(bool v) { bind_any_ = v; }
  uint64_t generation() const { return generation_.load(); }
  uint64_t updates() const { return updates_.load(); }

 private:
  static constexpr size_t kStripes = 64;
  struct Stripe {
    std::mutex mu;
    std::unordered_map<std::string, Entry> map;
    std::unordered_set<std::string> dirty;
  };
  void accept_loop();
  void serve(int fd);
  uint16_t handle(Op op, Reader& in, Writer& out);
  void apply(Entry& e, const std::string& key, const float* g, size_t n, const Updater* u);
  void apply_pending();
  void save(const std::string& path);
  void load(const std::string& path);
  Stripe& stripe(const std::string& key);
  RowTable& row_table(const std::string& name, uint32_t dim);
  const Updater* updater(const std::string& spec);

  int port_;
  int workers_;
  Mode mode_ = Mode::BSP;
  int staleness_;
  double barrier_timeout_s_;
  bool bind_any_ = false;
  int listen_fd_ = -1;
  std::atomic<bool> running_{false};
  std::atomic<bool> shutdown_requested_{false};
  std::thread accept_thread_;
  std::mutex conn_mu_;
  std::vector<int> conn_fds_;
  std::vector<std::thread> conn_threads_;
  Stripe stripes_[kStripes];
  std::mutex rt_mu_;
  std::unordered_map<std::string, std::unique_ptr<RowTable>> row_tables_;
  std::mutex upd_mu_;
  std::unordered_map<std::string, std::unique_ptr<Updater>> updaters_;
  std::mutex barrier_mu_;
  std::condition_variable barrier_cv_;
  int arrived_ = 0;
  int rv_arrived_ = 0;     // OP_RENDEZVOUS: its own count and generation, so a load() that
  uint64_t rv_gen_ = 0;   // restores generation_ cannot release a waiter early
  std::atomic<uint64_t> generation_{0};
  std::vector<uint64_t> clocks_;
  std::mutex stop_mu_;
  std::condition_variable stop_cv_;
  std::atomic<uint64_t> requests_{0}, pushes_{0}, updates_{0}, heartbeats_{0};
};

class PSClient {
 public:
  PSClient(const std::string& host, int port, double timeout_s);
  ~PSClient();
  uint16_t call(Op op, const Writer& req, std::vector<uint8_t>* resp);
  uint64_t bytes_sent() const { return bytes_sent_; }
  uint64_t bytes_recv() const { return bytes_recv_; }

 private:
  int fd_ = -1;
  std::mutex mu_;
  uint64_t bytes_sent_ = 0, bytes_recv_ = 0;
};

}  // namespace psnative
