// Threaded batch loader + id map (native runtime of the data pipeline).
//
// Reference: data/DataSet.java (reader threads parse lines into features and feed a bounded
// ArrayBlockingQueue; next() polls with a 3 s timeout), data/DataSource.java (offset/step
// sharding that the reference never configures, Q11), data/LibsvmParser.java and the MNIST
// CSV parser in Mnist.java:45-55.
//
// BatchReader: T reader threads own disjoint line stripes of the same file (line i belongs
// to reader (i / batch) % T), each parses whole batches into flat float / int64 arrays and
// pushes them into a bounded queue; rank sharding is line-level offset/step (line i is kept
// by this worker iff i % step == offset).  Formats:
//   "csv"    label,v1,...,vD              -> X float[B, D], Y float[B]
//   "libsvm" label idx:val idx:val ...    -> I int64[B, F] (first F indices, padded -1),
//                                            V float[B, F], Y float[B]
//   "ctr"    label|f1,...,fNum|c1,...,cCat  (numeric | categorical ids) -> X, E int64, Y
#include "loader.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace psnative {

// ------------------------------------------------------------------------------- IdMap
IdMap::IdMap(int64_t capacity) : capacity_(capacity) { map_.reserve(static_cast<size_t>(std::min<int64_t>(capacity, 1 << 22))); }

void IdMap::lookup(const int64_t* ids, int64_t n, bool insert, int64_t* out) {
  std::lock_guard<std::mutex> g(mu_);
  for (int64_t i = 0; i < n; ++i) {
    auto it = map_.find(ids[i]);
    if (it != map_.end()) {
      out[i] = it->second;
    } else if (insert && static_cast<int64_t>(map_.size()) < capacity_) {
      const int64_t s = static_cast<int64_t>(map_.size());
      map_.emplace(ids[i], s);
      out[i] = s;
    } else {
      out[i] = -1;
    }
  }
}

int64_t IdMap::size() {
  std::lock_guard<std::mutex> g(mu_);
  return static_cast<int64_t>(map_.size());
}

void IdMap::restore(const int64_t* ids, const int64_t* slots, int64_t n) {
  std::lock_guard<std::mutex> g(mu_);
  map_.clear();
  for (int64_t i = 0; i < n; ++i) map_.emplace(ids[i], slots[i]);
}

std::vector<std::pair<int64_t, int64_t>> IdMap::items() {
  std::lock_guard<std::mutex> g(mu_);
  return std::vector<std::pair<int64_t, int64_t>>(map_.begin(), map_.end());
}

// ------------------------------------------------------------------------------- parsing
static bool parse_csv(const std::string& line, int dims, float* x, float* y) {
  const char* p = line.c_str();
  char* end;
  *y = std::strtof(p, &end);
  if (end == p) return false;
  p = end;
  for (int d = 0; d < dims; ++d) {
    while (*p == ',' || *p == ' ') ++p;
    x[d] = std::strtof(p, &end);
    if (end == p) x[d] = 0.f;
    p = end;
  }
  return true;
}

static bool parse_libsvm(const std::string& line, int fields, int64_t* idx, float* val, float* y) {
  const char* p = line.c_str();
  char* end;
  *y = std::strtof(p, &end);
  if (end == p) return false;
  p = end;
  int f = 0;
  while (*p && f < fields) {
    while (*p == ' ' || *p == '\t') ++p;
    if (!*p || *p == '\n') break;
    const long long i = std::strtoll(p, &end, 10);
    if (end == p || *end != ':') break;
    p = end + 1;
    const float v = std::strtof(p, &end);
    p = end;
    idx[f] = i;
    val[f] = v;
    ++f;
  }
  for (; f < fields; ++f) {
    idx[f] = -1;
    val[f] = 0.f;
  }
  return true;
}

static bool parse_ctr(const std::string& line, int num, int cat, float* x, int64_t* e, float* y) {
  const char* p = line.c_str();
  char* end;
  *y = std::strtof(p, &end);
  if (end == p) return false;
  p = end;
  if (*p == '|') ++p;
  for (int d = 0; d < num; ++d) {
    while (*p == ',' || *p == ' ') ++p;
    x[d] = std::strtof(p, &end);
    p = end;
  }
  if (*p == '|') ++p;
  for (int c = 0; c < cat; ++c) {
    while (*p == ',' || *p == ' ') ++p;
    e[c] = std::strtoll(p, &end, 10);
    p = end;
  }
  return true;
}

// ------------------------------------------------------------------------------- reader
BatchReader::BatchReader(const std::string& path, const std::string& format, int batch, int dims, int fields,
                         int offset, int step, int threads, int depth, bool drop_last)
    : path_(path), batch_(batch), dims_(dims), fields_(fields), offset_(offset), step_(std::max(1, step)),
      threads_(std::max(1, threads)), depth_(std::max(1, depth)), drop_last_(drop_last) {
  if (format == "csv") fmt_ = Fmt::CSV;
  else if (format == "libsvm") fmt_ = Fmt::LIBSVM;
  else if (format == "ctr") fmt_ = Fmt::CTR;
  else throw std::runtime_error("format must be csv|libsvm|ctr");
  std::ifstream probe(path_);
  if (!probe) throw std::runtime_error("cannot open " + path_);
  start();
}

BatchReader::~BatchReader() { stop(); }

void BatchReader::start() {
  stop_ = false;
  finished_ = 0;
  for (int t = 0; t < threads_; ++t) workers_.emplace_back([this, t] { run(t); });
}

void BatchReader::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  not_full_.notify_all();
  not_empty_.notify_all();
  for (auto& w : workers_)
    if (w.joinable()) w.join();
  workers_.clear();
  std::lock_guard<std::mutex> g(mu_);
  q_.clear();
}

void BatchReader::reset() {
  stop();
  start();
}

void BatchReader::run(int tid) {
  std::ifstream f(path_);
  std::string line;
  int64_t lineno = -1;
  int64_t kept = -1;  // index among this rank's lines
  Batch b;
  auto alloc = [&] {
    b = Batch();
    b.y.reserve(batch_);
  };
  alloc();
  auto flush = [&](bool final) {
    if (b.n == 0) return;
    if (final && drop_last_ && b.n < batch_) return;
    std::unique_lock<std::mutex> g(mu_);
    not_full_.wait(g, [&] { return stop_ || static_cast<int>(q_.size()) < depth_; });
    if (stop_) return;
    q_.push_back(std::move(b));
    not_empty_.notify_one();
    alloc();
  };
  while (std::getline(f, line)) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (stop_) return;
    }
    ++lineno;
    if (lineno % step_ != offset_) continue;  // rank sharding (DataSource offset/step)
    ++kept;
    if ((kept / batch_) % threads_ != tid) continue;  // reader striping by whole batches
    if (line.empty()) continue;
    float y = 0.f;
    bool ok = false;
    if (fmt_ == Fmt::CSV) {
      const size_t o = b.x.size();
      b.x.resize(o + static_cast<size_t>(dims_));
      ok = parse_csv(line, dims_, b.x.data() + o, &y);
      if (!ok) b.x.resize(o);
    } else if (fmt_ == Fmt::LIBSVM) {
      const size_t o = b.i.size();
      b.i.resize(o + static_cast<size_t>(fields_));
      b.v.resize(o + static_cast<size_t>(fields_));
      ok = parse_libsvm(line, fields_, b.i.data() + o, b.v.data() + o, &y);
      if (!ok) {
        b.i.resize(o);
        b.v.resize(o);
      }
    } else {
      const size_t ox = b.x.size(), oe = b.i.size();
      b.x.resize(ox + static_cast<size_t>(dims_));
      b.i.resize(oe + static_cast<size_t>(fields_));
      ok = parse_ctr(line, dims_, fields_, b.x.data() + ox, b.i.data() + oe, &y);
      if (!ok) {
        b.x.resize(ox);
        b.i.resize(oe);
      }
    }
    if (!ok) continue;
    b.y.push_back(y);
    b.n += 1;
    if (b.n == batch_) flush(false);
  }
  flush(true);
  std::lock_guard<std::mutex> g(mu_);
  finished_ += 1;
  not_empty_.notify_all();
}

bool BatchReader::next(Batch* out, double timeout_s) {
  std::unique_lock<std::mutex> g(mu_);
  const bool ok = not_empty_.wait_for(g, std::chrono::duration<double>(timeout_s),
                                      [&] { return !q_.empty() || finished_ == threads_ || stop_; });
  if (!ok || q_.empty()) return false;
  *out = std::move(q_.front());
  q_.pop_front();
  not_full_.notify_one();
  return true;
}

bool BatchReader::has_next() {
  std::unique_lock<std::mutex> g(mu_);
  not_empty_.wait(g, [&] { return !q_.empty() || finished_ == threads_ || stop_; });
  return !q_.empty();
}

}  // namespace psnative
