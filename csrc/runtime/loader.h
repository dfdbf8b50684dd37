#pragma once
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace psnative {

class IdMap {
 public:
  explicit IdMap(int64_t capacity);
  void lookup(const int64_t* ids, int64_t n, bool insert, int64_t* out);
  int64_t size();
  std::vector<std::pair<int64_t, int64_t>> items();
  void restore(const int64_t* ids, const int64_t* slots, int64_t n);  // checkpoint resume

 private:
  int64_t capacity_;
  std::mutex mu_;
  std::unordered_map<int64_t, int64_t> map_;
};

struct Batch {
  int n = 0;
  std::vector<float> x;    // [n, dims]   (csv / ctr numeric)
  std::vector<int64_t> i;  // [n, fields] (libsvm indices / ctr categorical ids)
  std::vector<float> v;    // [n, fields] (libsvm values)
  std::vector<float> y;    // [n]
};

class BatchReader {
 public:
  BatchReader(const std::string& path, const std::string& format, int batch, int dims, int fields, int offset,
              int step, int threads, int depth, bool drop_last);
  ~BatchReader();
  bool next(Batch* out, double timeout_s);
  bool has_next();
  void reset();
  int dims() const { return dims_; }
  int fields() const { return fields_; }

 private:
  enum class Fmt { CSV, LIBSVM, CTR };
  void start();
  void stop();
  void run(int tid);
  std::string path_;
  Fmt fmt_;
  int batch_, dims_, fields_, offset_, step_, threads_, depth_;
  bool drop_last_;
  std::mutex mu_;
  std::condition_variable not_full_, not_empty_;
  std::deque<Batch> q_;
  std::vector<std::thread> workers_;
  bool stop_ = false;
  int finished_ = 0;
};

}  // namespace psnative
