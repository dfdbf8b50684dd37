// ThreadSanitizer stress of the asynchronous-PS control protocol (csrc/include/async_ctl.h):
// W owner threads run serve_loop, W worker threads push into kMbox-deep mailboxes, bump clocks, and
// pin / copy / unpin published slots under an SSP(s) gate.  The "GPU" is plain host memory
// here, written and read with ordinary loads/stores, so TSan checks that the acquire/release
// hand-offs order every mailbox and slot access (a missing fence is a reported data race).
// Invariants asserted: every push applied exactly once; a pinned slot is never rewritten while
// pinned (readers verify the slot's version stamp before and after the copy); the SSP bound
// clock(w) - clock(v) <= s + 1 holds whenever observed.
//
//   build + run: scripts/tsan_native.sh async
#include <atomic>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "async_ctl.h"

using namespace psasync;

int main(int argc, char** argv) {
  const int W = argc > 1 ? std::atoi(argv[1]) : 3;
  const int steps = argc > 2 ? std::atoi(argv[2]) : 200;
  const int s = argc > 3 ? std::atoi(argv[3]) : 1;
  const int L = 64;  // shard length
  AsyncCtl* c = new AsyncCtl;
  init(c, W);
  // per owner: W x kMbox mailboxes of L floats, 3 slots of L floats + a version stamp per slot
  std::vector<std::vector<float>> mbox(W * W * kMbox, std::vector<float>(L, 0.f));
  std::vector<std::vector<float>> slot(W * kSlots, std::vector<float>(L, 0.f));
  std::vector<int64_t> stamp(W * kSlots, 0);
  std::vector<float> master(W * L, 0.f);
  std::vector<int64_t> applied(W, 0);
  std::atomic<bool> stop{false};
  std::vector<std::thread> th;
  for (int o = 0; o < W; ++o)
    th.emplace_back([&, o] {
      serve_loop(c, o, &stop, [&](int w, int ms, int sl, int64_t step) {
        for (int i = 0; i < L; ++i) master[o * L + i] += mbox[(o * W + w) * kMbox + ms][i];
        for (int i = 0; i < L; ++i) slot[o * kSlots + sl][i] = master[o * L + i];
        stamp[o * kSlots + sl] = step;
        applied[o] += 1;
      });
    });
  std::atomic<int> violations{0};
  std::vector<std::thread> wk;
  for (int w = 0; w < W; ++w)
    wk.emplace_back([&, w] {
      std::vector<float> replica(L);
      for (int t = 0; t < steps; ++t) {
        for (int o = 0; o < W; ++o) {
          Backoff bo;
          const int64_t k = ld(&c->seq[o][w]);  // this worker's push number (only it bumps seq)
          while (ld(&c->ack[o][w]) + kMbox <= k) bo();  // mailbox slot k % kMbox still unapplied
          for (int i = 0; i < L; ++i) mbox[(o * W + w) * kMbox + k % kMbox][i] = 1.f;  // gradient of 1
          add(&c->seq[o][w], 1);
        }
        const int64_t clk = add(&c->clock[w], 1);
        {  // SSP gate on applied pushes
          Backoff bo;
          while (min_ack(c) < clk - s) bo();
        }
        for (int v = 0; v < W; ++v)
          if (ld(&c->clock[w]) - ld(&c->clock[v]) > s + 1) violations++;
        for (int o = 0; o < W; ++o) {
          const int sl = pin(c, o);
          const int64_t before = stamp[o * kSlots + sl];
          for (int i = 0; i < L; ++i) replica[i] = slot[o * kSlots + sl][i];
          if (stamp[o * kSlots + sl] != before) violations++;  // rewritten while pinned
          unpin(c, o, sl);
        }
      }
    });
  for (auto& t : wk) t.join();
  // drain, stop the owners
  for (int o = 0; o < W; ++o)
    for (int w = 0; w < W; ++w) {
      Backoff bo;
      while (ld(&c->ack[o][w]) < steps) bo();
    }
  stop = true;
  for (auto& t : th) t.join();
  int bad = violations.load();
  for (int o = 0; o < W; ++o) {
    if (applied[o] != static_cast<int64_t>(W) * steps) bad++;
    for (int i = 0; i < L; ++i)
      if (master[o * L + i] != static_cast<float>(W * steps)) bad++;
  }
  std::printf("async_ctl stress: W=%d steps=%d s=%d violations=%d\n", W, steps, s, bad);
  delete c;
  return bad == 0 ? 0 : 1;
}
