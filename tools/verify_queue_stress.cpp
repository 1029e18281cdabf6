// The asynchronous verify's queue (ciruela_amd/csrc/verify_queue.hpp) on the
// host with a test hasher in place of the GPU batch -- built under
// ThreadSanitizer and under ASan + UBSan by tests/test_verify_queue.py.
// The test hasher's digest is a keyed mix of the block bytes (not a BLAKE2b:
// this checks the queue's bookkeeping, not the hash); it can be held closed
// to make the queue's states deterministic, and fails every batch that holds
// a block of the poison length with CIR_EIO.
//   verify_queue_stress <rounds> <seed>   -> prints "ok ..." and exits 0
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "verify_queue.hpp"

#if defined(__SANITIZE_THREAD__)
#include <pthread.h>
#include <time.h>
// gcc 11's ThreadSanitizer does not intercept pthread_cond_clockwait, which
// libstdc++ uses for condition_variable::wait_until on steady_clock (the
// queue's batching window): the waiter's unlock goes unseen and every later
// lock of the mutex is reported as a double lock / race.  This test binary
// routes the call through pthread_cond_timedwait, which TSan intercepts,
// with the monotonic deadline carried over to the realtime clock.
extern "C" int pthread_cond_clockwait(pthread_cond_t* c, pthread_mutex_t* m, clockid_t clk,
                                      const struct timespec* abs) {
  struct timespec now_c, now_r, r;
  clock_gettime(clk, &now_c);
  clock_gettime(CLOCK_REALTIME, &now_r);
  long long ns = (long long)(abs->tv_sec - now_c.tv_sec) * 1000000000LL +
                 (abs->tv_nsec - now_c.tv_nsec) + now_r.tv_nsec;
  r.tv_sec = now_r.tv_sec + (time_t)(ns / 1000000000LL);
  r.tv_nsec = (long)(ns % 1000000000LL);
  if (r.tv_nsec < 0) {
    r.tv_nsec += 1000000000L;
    r.tv_sec -= 1;
  }
  return pthread_cond_timedwait(c, m, &r);
}
#endif

using cir::VerifyQueue;

static constexpr size_t kPoison = 4242;

static void digest(const uint8_t* p, size_t n, uint8_t out[32]) {
  uint64_t h[4] = {0x6a09e667f3bcc908ull ^ n, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                   0xa54ff53a5f1d36f1ull};
  for (size_t i = 0; i < n; ++i) {
    uint64_t& x = h[i & 3];
    x = (x ^ p[i]) * 0x100000001b3ull;
    x ^= x >> 29;
  }
  memcpy(out, h, 32);
}

// the hasher the queue calls from its worker: optionally held closed, slow,
// or failing on the poison length
struct TestHasher {
  std::mutex mu;
  std::condition_variable cv;
  bool open = true;
  std::atomic<int> batches{0};
  std::atomic<int> max_us{0};
  void hold() {
    std::lock_guard<std::mutex> lk(mu);
    open = false;
  }
  void release() {
    {
      std::lock_guard<std::mutex> lk(mu);
      open = true;
    }
    cv.notify_all();
  }
  VerifyQueue::HashFn fn() {
    return [this](int, const uint8_t* arena, const uint64_t* off, const uint32_t* len, size_t n,
                  uint8_t* out, std::string* err) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return open; });
      }
      ++batches;
      if (const int us = max_us.load()) std::this_thread::sleep_for(std::chrono::microseconds(rand() % us));
      for (size_t i = 0; i < n; ++i)
        if (len[i] == kPoison) {
          *err = "poisoned batch";
          return (int)CIR_EIO;
        }
      for (size_t i = 0; i < n; ++i) digest(arena + off[i], len[i], out + 32 * i);
      return (int)CIR_OK;
    };
  }
};

#define CHECK(c)                                                              \
  do {                                                                        \
    if (!(c)) {                                                               \
      fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c);   \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

struct Block {
  std::vector<uint8_t> data;
  uint8_t expected[32];
  bool good;
};

static Block make_block(std::mt19937_64& rng, size_t n, bool good) {
  Block b;
  b.data.resize(n);
  for (auto& c : b.data) c = (uint8_t)rng();
  digest(b.data.data(), n, b.expected);
  b.good = good;
  if (!good) b.expected[rng() % 32] ^= 1 + (uint8_t)(rng() % 255);
  return b;
}

static uint64_t stat(VerifyQueue& q, int k) {
  uint64_t s[CIR_VERIFY_STATS_FIELDS];
  q.stats(s);
  return s[k];
}
enum { kHeld, kPeak, kPending, kOutcomes, kExpired, kForgotten, kRefused, kBatches };

static void stage(const char* what) {
  fprintf(stderr, "stage: %s\n", what);
  fflush(stderr);
}

// deterministic states with the hasher held closed
static void deterministic(std::mt19937_64& rng) {
  stage("refusal");
  TestHasher th;
  VerifyQueue q(th.fn());
  std::string err;
  q.window(100000, 4096);
  q.limits(64 << 10, 0, true);
  th.hold();
  Block a = make_block(rng, 40 << 10, true), b = make_block(rng, 40 << 10, false);
  uint64_t ta = 0, tb = 0, te = 0;
  CHECK(q.submit(1, a.data.data(), a.data.size(), a.expected, &ta, &err) == 0);
  CHECK(q.submit(1, b.data.data(), b.data.size(), b.expected, &tb, &err) == CIR_EAGAIN);
  CHECK(err.find("verify queue full") == 0);
  Block e = make_block(rng, 0, true);
  CHECK(q.submit(1, e.data.data(), 0, e.expected, &te, &err) == 0);  // 0 bytes always fit
  CHECK(stat(q, kHeld) == (40u << 10) && stat(q, kPending) == 2 && stat(q, kRefused) == 1);
  CHECK(q.poll(ta, &err) == 0);
  th.release();
  CHECK(q.wait(ta, &err) == 1);
  CHECK(q.poll(ta, &err) == CIR_ENOTFOUND);  // consumed
  CHECK(q.wait(te, &err) == 1);
  CHECK(q.submit(1, b.data.data(), b.data.size(), b.expected, &tb, &err) == 0);
  CHECK(q.wait(tb, &err) == 2);
  CHECK(stat(q, kHeld) == 0 && stat(q, kPeak) == (40u << 10));
  // a block larger than the bound is taken when nothing else is held
  Block big = make_block(rng, 100 << 10, true);
  uint64_t tbig = 0;
  CHECK(q.submit(1, big.data.data(), big.data.size(), big.expected, &tbig, &err) == 0);
  CHECK(q.wait(tbig, &err) == 1);

  // blocking: a submitter without room waits until the worker frees it
  stage("blocking");
  q.limits(64 << 10, 0, false);
  th.hold();
  CHECK(q.submit(1, a.data.data(), a.data.size(), a.expected, &ta, &err) == 0);
  std::atomic<bool> entered{false}, returned{false};
  std::thread blocked([&] {
    uint64_t t = 0;
    std::string e2;
    entered = true;
    CHECK(q.submit(1, a.data.data(), a.data.size(), a.expected, &t, &e2) == 0);
    returned = true;
    CHECK(q.wait(t, &e2) == 1);
  });
  while (!entered) std::this_thread::yield();
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  CHECK(!returned);  // still waiting for room: the hasher is closed
  th.release();
  blocked.join();
  CHECK(q.wait(ta, &err) == 1);

  // forget: pending (with a waiter), finished, unknown
  stage("forget");
  th.hold();
  uint64_t tf = 0;
  CHECK(q.submit(1, a.data.data(), a.data.size(), a.expected, &tf, &err) == 0);
  int waited = 99;
  std::thread waiter([&] {
    std::string e2;
    waited = q.wait(tf, &e2);
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(5));
  CHECK(q.forget(tf, &err) == 0);
  waiter.join();
  CHECK(waited == CIR_ENOTFOUND);
  th.release();
  uint64_t tg = 0, th2 = 0;
  q.window(0, 4096);
  CHECK(q.submit(1, b.data.data(), b.data.size(), b.expected, &tg, &err) == 0);
  CHECK(q.submit(1, e.data.data(), 0, e.expected, &th2, &err) == 0);
  CHECK(q.wait(th2, &err) == 1);
  while (q.poll(tg, &err) == 0) std::this_thread::yield();  // (consumes it when done)
  CHECK(q.forget(tg, &err) == CIR_ENOTFOUND);
  uint64_t ti = 0;
  CHECK(q.submit(1, b.data.data(), b.data.size(), b.expected, &ti, &err) == 0);
  while (stat(q, kPending)) std::this_thread::yield();
  CHECK(q.forget(ti, &err) == 0);  // finished, not consumed
  CHECK(q.poll(ti, &err) == CIR_ENOTFOUND && q.forget(ti, &err) == CIR_ENOTFOUND);
  CHECK(q.forget(123456789, &err) == CIR_ENOTFOUND);
  CHECK(stat(q, kForgotten) == 2 && stat(q, kOutcomes) == 0);

  // expiry: at most 16 outcomes held, the newest kept
  stage("expiry");
  q.limits(0, 16, false);
  std::vector<uint64_t> tk(64);
  std::vector<Block> bl;
  for (int i = 0; i < 64; ++i) bl.push_back(make_block(rng, 1000 + i, i % 3 != 1));
  for (int i = 0; i < 64; ++i)
    CHECK(q.submit(1, bl[i].data.data(), bl[i].data.size(), bl[i].expected, &tk[i], &err) == 0);
  CHECK(q.wait(tk[63], &err) == 1 + !bl[63].good);
  CHECK(stat(q, kOutcomes) <= 16 && stat(q, kExpired) >= 64 - 1 - 16);
  CHECK(q.poll(tk[0], &err) == CIR_ENOTFOUND);
  for (int i = 48; i < 63; ++i) CHECK(q.poll(tk[i], &err) == 1 + !bl[i].good);

  // a failed batch: every ticket in it reports the hasher's code and text
  stage("failed batch");
  th.hold();
  q.window(100000, 4096);
  Block p1 = make_block(rng, kPoison, true), p2 = make_block(rng, 10, true);
  uint64_t tp1 = 0, tp2 = 0;
  CHECK(q.submit(1, p1.data.data(), kPoison, p1.expected, &tp1, &err) == 0);
  CHECK(q.submit(1, p2.data.data(), 10, p2.expected, &tp2, &err) == 0);
  th.release();
  CHECK(q.wait(tp2, &err) == CIR_EIO && err == "poisoned batch");
  CHECK(q.poll(tp1, &err) == CIR_EIO && err == "poisoned batch");
  // two hash types never share a batch
  stage("hash types");
  q.window(0, 4096);
  const int b0 = th.batches.load();
  uint64_t u1 = 0, u2 = 0;
  th.hold();
  CHECK(q.submit(1, p2.data.data(), 10, p2.expected, &u1, &err) == 0);
  CHECK(q.submit(2, p2.data.data(), 10, p2.expected, &u2, &err) == 0);
  th.release();
  CHECK(q.wait(u1, &err) == 1 && q.wait(u2, &err) == 1);
  CHECK(th.batches.load() - b0 == 2);
  // idle past a second: the spare arenas are given back, and the queue
  // works as before afterwards
  stage("idle trim");
  std::this_thread::sleep_for(std::chrono::milliseconds(1200));
  uint64_t tz = 0;
  CHECK(q.submit(1, big.data.data(), big.data.size(), big.expected, &tz, &err) == 0);
  CHECK(q.wait(tz, &err) == 1);
  // a bound past what can be allocated: it caps admission only, so blocks
  // still verify in arenas of the usual size; a block whose own arena
  // cannot be allocated is CIR_ENOMEM and holds nothing (its bytes are
  // never read: the allocation comes first); the queue works on
  stage("bound larger than memory");
  q.limits(1ull << 62, 0, false);
  uint64_t tn = 0;
  CHECK(q.submit(1, p2.data.data(), 10, p2.expected, &tn, &err) == 0);
  CHECK(q.wait(tn, &err) == 1);
  stage("arena that cannot be allocated");
  CHECK(q.submit(1, p2.data.data(), 1ull << 61, p2.expected, &tn, &err) == CIR_ENOMEM);
  CHECK(stat(q, kHeld) == 0);
  q.limits(0, 0, false);
  CHECK(q.submit(1, p2.data.data(), 10, p2.expected, &tn, &err) == 0);
  CHECK(q.wait(tn, &err) == 1);
}

// random traffic from several threads against a byte bound, blocking or
// not, with forgets; every outcome kept must be right and the bound held
static void random_traffic(std::mt19937_64& seed_rng, int round) {
  stage(round & 1 ? "random traffic, non-blocking" : "random traffic, blocking");
  TestHasher th;
  th.max_us = 200;
  auto q = std::make_unique<VerifyQueue>(th.fn());
  const bool nb = round & 1;
  const uint64_t cap = (uint64_t)(64 + seed_rng() % 1024) << 10;
  q->limits(cap, 0, nb);
  q->window((uint32_t)(seed_rng() % 400), (uint32_t)(1 + seed_rng() % 64));
  const int nthreads = 2 + (int)(seed_rng() % 4);
  std::atomic<int> bad{0};
  std::vector<std::thread> th_;
  for (int t = 0; t < nthreads; ++t) {
    const uint64_t s = seed_rng();
    th_.emplace_back([&, s] {
      std::mt19937_64 rng(s);
      std::string err;
      std::vector<std::pair<uint64_t, bool>> mine;
      for (int i = 0; i < 150; ++i) {
        const size_t n = rng() % 5 == 0 ? 0 : rng() % 70000;
        Block b = make_block(rng, n, rng() % 4 != 0);
        uint64_t tk = 0;
        int rc;
        while ((rc = q->submit(1 + (int)(rng() % 2), b.data.data(), n, b.expected, &tk, &err)) ==
               CIR_EAGAIN)
          std::this_thread::yield();
        if (rc) ++bad;
        if (rng() % 10 == 0) {
          if (q->forget(tk, &err) != 0) ++bad;
        } else {
          mine.push_back({tk, b.good});
        }
        if (rng() % 7 == 0 && !mine.empty()) {  // poll one now and then
          const auto& m = mine.back();
          const int v = q->poll(m.first, &err);
          if (v == 1 || v == 2) {
            if ((v == 1) != m.second) ++bad;
            mine.pop_back();
          } else if (v != 0) {
            ++bad;
          }
        }
      }
      for (auto& m : mine) {
        const int v = q->wait(m.first, &err);
        if (v != (m.second ? 1 : 2)) ++bad;
      }
    });
  }
  for (auto& t : th_) t.join();
  CHECK(bad.load() == 0);
  CHECK(stat(*q, kPeak) <= std::max<uint64_t>(cap, 70000));
  // (a batch of forgotten tickets only may still be in flight)
  for (int i = 0; i < 10000 && stat(*q, kHeld); ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  CHECK(stat(*q, kHeld) == 0 && stat(*q, kPending) == 0 && stat(*q, kOutcomes) == 0);
  // destroyed with work queued: the destructor drains it
  th.hold();
  std::string err;
  Block b = make_block(seed_rng, 100, true);
  uint64_t tk = 0;
  CHECK(q->submit(1, b.data.data(), 100, b.expected, &tk, &err) == 0);
  th.release();
  q.reset();
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 4;
  std::mt19937_64 rng(argc > 2 ? strtoull(argv[2], nullptr, 10) : 1);
  deterministic(rng);
  for (int r = 0; r < rounds; ++r) random_traffic(rng, r);
  printf("ok %d rounds\n", rounds);
  return 0;
}
