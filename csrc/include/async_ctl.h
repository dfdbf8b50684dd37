// Control block of the asynchronous parameter server (ASP / SSP without lockstep collectives).
//
// Reference: the async PServer applies every push on arrival and its barrier returns at once
// (net/PServer.java:176-184, 242-248; net/PSClient.java:159-161).  There is no staleness bound
// in the reference; here SSP(s) bounds it.
//
// Data plane (one node): every rank owns a contiguous range shard of the flat parameter space.
// The owner keeps per-worker gradient MAILBOXES (kMbox = 2 deep: push k of worker w lands in
// mailbox slot k % 2, so a worker only waits when its push k-2 is still unapplied) and 3
// PUBLISHED weight slots in its own device memory; the other ranks write their gradient slice
// straight into the owner's mailbox and read the owner's current slot back with peer copies over
// xGMI (IPC-mapped buffers) -- one-sided, so no rank ever waits for another rank to reach a
// matching collective.
//
// Control plane: this block, in POSIX shared memory, all fields int64 accessed with acquire /
// release atomics:
//   seq[o][w]   pushes worker w has deposited in owner o's mailbox (bumped after the copy landed)
//   ack[o][w]   pushes owner o has applied from worker w (the mailbox is free when ack == seq)
//   version[o]  updates applied to shard o;   cur[o]  slot holding the newest weights of shard o
//   pins[o][s]  readers currently copying slot s of shard o (the owner never overwrites a pinned
//               slot -- no torn reads)
//   clock[w]    steps worker w has pushed
// SSP(s): before a worker at clock c pulls, every ack[o][w] must be >= c - s, i.e. the weights it
// reads contain every update of every worker from clocks < c - s.  s = 0 gives BSP semantics
// without any collective; ASP skips the gate.
#pragma once
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <thread>

namespace psasync {

constexpr int64_t kMagic = 0x50534153594e4331ll;  // "PSASYNC1"
constexpr int kMaxW = 64;
constexpr int kSlots = 3;
constexpr int kMbox = 2;  // mailbox depth per (owner, worker)

struct AsyncCtl {
  int64_t magic;
  int64_t world;
  int64_t stop;
  int64_t pad;
  int64_t clock[kMaxW];
  int64_t seq[kMaxW][kMaxW];
  int64_t ack[kMaxW][kMaxW];
  int64_t version[kMaxW];
  int64_t cur[kMaxW];
  int64_t pins[kMaxW][4];
};

inline int64_t ld(const int64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void st(int64_t* p, int64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
inline int64_t add(int64_t* p, int64_t v) { return __atomic_add_fetch(p, v, __ATOMIC_ACQ_REL); }

inline void init(AsyncCtl* c, int64_t world) {
  char* b = reinterpret_cast<char*>(c);
  for (size_t i = 0; i < sizeof(AsyncCtl); ++i) b[i] = 0;
  c->world = world;
  st(&c->magic, kMagic);
}

// Spin politely: a few hundred pause iterations, then yield, then short sleeps.
struct Backoff {
  int n = 0;
  void operator()() {
    ++n;
    if (n < 256) {
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    } else if (n < 1024) {
      std::this_thread::yield();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
};

// A slot of owner o that holds no reader and is not the current one (-1 if none right now).
// The full fence pairs with the one in pin(): "owner publishes cur, then reads pins" against
// "reader bumps pins, then reads cur" is the store-buffer pattern -- with acquire/release alone
// both could read the stale value (x86 store buffer) and the owner would overwrite a slot a
// reader is copying.
inline int free_slot(AsyncCtl* c, int o) {
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  const int64_t cur = ld(&c->cur[o]);
  for (int s = 0; s < kSlots; ++s)
    if (s != cur && ld(&c->pins[o][s]) == 0) return s;
  return -1;
}

// Reader side: pin the current slot of owner o (re-checked after the pin so the owner cannot
// have moved on and reused it in between).
inline int pin(AsyncCtl* c, int o) {
  Backoff bo;
  for (;;) {
    const int64_t s = ld(&c->cur[o]);
    add(&c->pins[o][s], 1);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);  // see free_slot()
    if (ld(&c->cur[o]) == s) return static_cast<int>(s);
    add(&c->pins[o][s], -1);
    bo();
  }
}

inline void unpin(AsyncCtl* c, int o, int s) { add(&c->pins[o][s], -1); }

inline int64_t min_ack(AsyncCtl* c) {
  int64_t m = INT64_MAX;
  const int W = static_cast<int>(c->world);
  for (int o = 0; o < W; ++o)
    for (int w = 0; w < W; ++w) {
      const int64_t a = ld(&c->ack[o][w]);
      if (a < m) m = a;
    }
  return m;
}

// Owner progress loop: apply every deposited push in arrival order (round-robin over workers
// for fairness), publish into a free slot, then acknowledge.  ``apply(w, mslot, slot, step)``
// runs the optimizer on the master shard with worker w's mailbox slot ``mslot`` (= push number
// % kMbox) and writes the new weights into published ``slot``; it returns only once the result
// is globally visible (stream synchronised).
template <class Apply>
void serve_loop(AsyncCtl* c, int me, const std::atomic<bool>* stop, Apply&& apply) {
  const int W = static_cast<int>(c->world);
  int start = 0;
  Backoff idle;
  while (!stop->load(std::memory_order_acquire) && ld(&c->stop) == 0) {
    bool did = false;
    for (int k = 0; k < W; ++k) {
      const int w = (start + k) % W;
      const int64_t s = ld(&c->seq[me][w]);
      const int64_t a = ld(&c->ack[me][w]);
      if (s <= a) continue;
      int slot;
      Backoff wait_slot;
      while ((slot = free_slot(c, me)) < 0) {
        if (stop->load(std::memory_order_acquire) || ld(&c->stop)) return;
        wait_slot();
      }
      const int64_t v = ld(&c->version[me]);
      apply(w, static_cast<int>(a % kMbox), slot, v + 1);
      st(&c->cur[me], slot);
      st(&c->version[me], v + 1);
      st(&c->ack[me][w], a + 1);
      did = true;
    }
    start = (start + 1) % W;
    if (did) idle.n = 0;
    else idle();
  }
}

}  // namespace psasync
