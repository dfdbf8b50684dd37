// Wire protocol + socket helpers for the native TCP parameter server (ps_server.cpp).
//
// Replaces the reference's gRPC/protobuf PS service (src/main/resources/proto/ps.proto:7-71,
// net/PSClient.java, net/PServer.java) with a length-prefixed binary protocol: float
// payloads travel as raw little-endian float32 (the reference boxes every float into a
// protobuf repeated field and gzips it), and PUSH carries a whole list of keys per request
// instead of one RPC per key (the reference's dominant cost).
//
// Frame:   request  = u32 magic | u8 op | u32 len | payload[len]
//          response = u32 magic | u16 status | u32 len | payload[len]
// Strings: u32 len | bytes.    Matrix: u32 rows | u32 cols | f32[rows*cols]
#pragma once
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace psnative {

constexpr uint32_t kMagic = 0x4D415350u;  // "PSAM"

enum Op : uint8_t {
  OP_GET = 1,
  OP_GET_LIST = 2,
  OP_UPSERT = 3,
  OP_UPSERT_LIST = 4,
  OP_PUSH = 5,
  OP_BARRIER = 6,
  OP_REGISTER = 7,
  OP_STATS = 8,
  OP_SAVE = 9,
  OP_LOAD = 10,
  OP_SHUTDOWN = 11,
  OP_HEARTBEAT = 12,
  OP_CLOCK = 13,
  OP_ROW_PULL = 14,  // sparse row tables: pull (lazy deterministic create) of many int64 keys
  OP_ROW_PUSH = 15,  // sparse row tables: push per-row gradients (BSP accumulate / apply)
  OP_RENDEZVOUS = 16,  // mode-independent W-worker rendezvous (resume hand-off; never touches the BSP generation)
};

enum Status : uint16_t { ST_OK = 200, ST_NOT_FOUND = 204, ST_BAD = 400, ST_TIMEOUT = 408, ST_ERR = 500 };

struct Matrix {
  uint32_t rows = 0, cols = 0;
  std::vector<float> data;
};

class Writer {
 public:
  std::vector<uint8_t> buf;
  void u8(uint8_t v) { buf.push_back(v); }
  void u16(uint16_t v) { raw(&v, 2); }
  void u32(uint32_t v) { raw(&v, 4); }
  void u64(uint64_t v) { raw(&v, 8); }
  void f32s(const float* p, size_t n) { raw(p, n * 4); }
  void f32(float v) { raw(&v, 4); }
  void str(const std::string& s) {
    u32(static_cast<uint32_t>(s.size()));
    raw(s.data(), s.size());
  }
  void mat(uint32_t rows, uint32_t cols, const float* p) {
    u32(rows);
    u32(cols);
    f32s(p, static_cast<size_t>(rows) * cols);
  }
  void raw(const void* p, size_t n) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    buf.insert(buf.end(), b, b + n);
  }
};

class Reader {
 public:
  Reader(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  uint8_t u8() { uint8_t v; get(&v, 1); return v; }
  uint16_t u16() { uint16_t v; get(&v, 2); return v; }
  uint32_t u32() { uint32_t v; get(&v, 4); return v; }
  uint64_t u64() { uint64_t v; get(&v, 8); return v; }
  float f32() { float v; get(&v, 4); return v; }
  // n raw elements of T (int64 keys / float rows) copied out of the frame
  template <typename T>
  void vec(std::vector<T>* out, size_t n) {
    if (n > (1ull << 34)) throw std::runtime_error("vector too large");
    out->resize(n);
    get(out->data(), n * sizeof(T));
  }
  std::string str() {
    uint32_t n = u32();
    need(n);
    std::string s(reinterpret_cast<const char*>(p_ + off_), n);
    off_ += n;
    return s;
  }
  Matrix mat() {
    Matrix m;
    m.rows = u32();
    m.cols = u32();
    const size_t n = static_cast<size_t>(m.rows) * m.cols;
    if (n > (1ull << 34)) throw std::runtime_error("matrix too large");
    m.data.resize(n);
    get(m.data.data(), n * 4);
    return m;
  }
  bool done() const { return off_ == n_; }

 private:
  void need(size_t k) {
    if (off_ + k > n_) throw std::runtime_error("truncated message");
  }
  void get(void* d, size_t k) {
    need(k);
    std::memcpy(d, p_ + off_, k);
    off_ += k;
  }
  const uint8_t* p_;
  size_t n_;
  size_t off_ = 0;
};

inline bool send_all(int fd, const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  while (n) {
    ssize_t k = ::send(fd, b, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    b += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

inline bool recv_all(int fd, void* p, size_t n) {
  uint8_t* b = static_cast<uint8_t*>(p);
  while (n) {
    ssize_t k = ::recv(fd, b, n, 0);
    if (k <= 0) return false;
    b += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

inline void tune_socket(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int sz = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
}

}  // namespace psnative
