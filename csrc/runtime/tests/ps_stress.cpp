// Concurrency stress test of the native TCP parameter server (SURVEY §5.2 c: host-side
// ThreadSanitizer build of the C++ server).  Built by scripts/tsan_native.sh with
// -fsanitize=thread; also a plain correctness check without it.
//
// W worker threads, each with its own PSClient connection, run R BSP rounds against one
// PSServer: upsert (insert-if-absent, first writer wins), push a gradient of ones for K keys
// with the SGD spec "simple@eta:1.0@", barrier.  The server averages the W pushes per key
// and applies one update per round, so after R rounds every key holds  init - R  exactly.
// An SSP phase then checks the clock bound: no CLOCK call returns while the caller is more
// than `s` clocks ahead of the slowest worker.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../ps_server.h"

using namespace psnative;

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  const int W = argc > 1 ? std::atoi(argv[1]) : 4;
  const int R = argc > 2 ? std::atoi(argv[2]) : 20;
  const int K = argc > 3 ? std::atoi(argv[3]) : 16;
  const int D = 8;

  // ---------------------------------------------------------------- BSP rounds
  PSServer srv(0, W, "bsp", 0, 60.0);
  srv.start();
  const int port = srv.port();
  std::atomic<int> errors{0};
  std::vector<std::thread> ts;
  for (int w = 0; w < W; ++w) {
    ts.emplace_back([&, w] {
      try {
        PSClient c("127.0.0.1", port, 60.0);
        {
          Writer r;
          r.str("simple@eta:1.0@");
          if (c.call(OP_REGISTER, r, nullptr) != ST_OK) errors++;
        }
        std::vector<float> init(D, 5.0f), ones(D, 1.0f);
        for (int k = 0; k < K; ++k) {  // every worker races the insert-if-absent
          Writer u;
          u.u8(0);
          u.str("k" + std::to_string(k));
          u.mat(1, D, init.data());
          if (c.call(OP_UPSERT, u, nullptr) != ST_OK) errors++;
        }
        for (int round = 0; round < R; ++round) {
          Writer p;
          p.u8(0);  // sync push
          p.str("simple@eta:1.0@");
          p.u32(static_cast<uint32_t>(K));
          for (int k = 0; k < K; ++k) {
            p.str("k" + std::to_string(k));
            p.mat(1, D, ones.data());
          }
          if (c.call(OP_PUSH, p, nullptr) != ST_OK) errors++;
          Writer b;
          b.u32(static_cast<uint32_t>(w));
          if (c.call(OP_BARRIER, b, nullptr) != ST_OK) errors++;
        }
      } catch (const std::exception& e) {
        std::fprintf(stderr, "worker %d: %s\n", w, e.what());
        errors++;
      }
    });
  }
  for (auto& t : ts) t.join();
  ts.clear();
  if (errors.load()) return fail("BSP worker errors");
  {
    PSClient c("127.0.0.1", port, 60.0);
    for (int k = 0; k < K; ++k) {
      Writer g;
      g.str("k" + std::to_string(k));
      std::vector<uint8_t> resp;
      if (c.call(OP_GET, g, &resp) != ST_OK) return fail("GET");
      Reader rd(resp.data(), resp.size());
      Matrix m = rd.mat();
      for (float v : m.data)
        if (v != 5.0f - static_cast<float>(R)) {
          std::fprintf(stderr, "key k%d = %f, expected %f\n", k, v, 5.0f - R);
          return fail("BSP result");
        }
    }
  }
  if (srv.generation() != static_cast<uint64_t>(R)) return fail("BSP generation count");
  srv.stop();

  // ---------------------------------------------------------------- SSP clock bound
  const int S = 1;
  PSServer ssp(0, W, "ssp", S, 60.0);
  ssp.start();
  std::vector<std::atomic<long>> clock(W);
  for (auto& c : clock) c = 0;
  std::atomic<int> violations{0};
  for (int w = 0; w < W; ++w) {
    ts.emplace_back([&, w] {
      try {
        PSClient c("127.0.0.1", ssp.port(), 60.0);
        for (long t = 1; t <= R; ++t) {
          if ((w + t) % 3 == 0) std::this_thread::sleep_for(std::chrono::microseconds(200 * (w + 1)));
          clock[w] = t;
          Writer r;
          r.u32(static_cast<uint32_t>(w));
          r.u64(static_cast<uint64_t>(t));
          if (c.call(OP_CLOCK, r, nullptr) != ST_OK) errors++;
          long mn = t;
          for (int o = 0; o < W; ++o) mn = std::min(mn, clock[o].load());
          // the call returned: we may run clock t+1 only if t - min <= S
          if (t - mn > S) violations++;
        }
      } catch (const std::exception& e) {
        std::fprintf(stderr, "ssp worker %d: %s\n", w, e.what());
        errors++;
      }
    });
  }
  for (auto& t : ts) t.join();
  ssp.stop();
  if (errors.load()) return fail("SSP worker errors");
  if (violations.load()) return fail("SSP bound violated");
  std::printf("ps_stress ok: %d workers x %d rounds x %d keys (BSP exact), SSP s=%d bound held\n", W, R, K, S);
  return 0;
}
