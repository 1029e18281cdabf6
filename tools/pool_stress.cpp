// The host worker pool (ciruela_amd/csrc/pool.hpp) under ThreadSanitizer:
// CALLERS threads each make ROUNDS parallel_run-style calls of random width
// over a random number of items pulled from an atomic index (as the staged
// paths' readers do); every item must be processed exactly once per call,
// and no call may hang while the others keep the pool busy; a job that
// throws is waited for everywhere before run() rethrows.
//   pool_stress CALLERS ROUNDS
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <random>
#include <stdexcept>
#include <thread>
#include <vector>

#include "pool.hpp"

int main(int argc, char** argv) {
  const int callers = argc > 1 ? atoi(argv[1]) : 8;
  const int rounds = argc > 2 ? atoi(argv[2]) : 200;
  cir::WorkerPool pool;
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int c = 0; c < callers; ++c)
    th.emplace_back([&, c] {
      std::mt19937 rng(c + 1);
      for (int r = 0; r < rounds; ++r) {
        const unsigned width = 1 + rng() % 24;
        const size_t items = rng() % 300;
        std::vector<std::atomic<int>> seen(items);
        for (auto& s : seen) s.store(0);
        std::atomic<size_t> next{0};
        const unsigned spin = rng() % 2000;
        pool.run(width, [&] {
          for (size_t i; (i = next.fetch_add(1)) < items;) {
            for (volatile unsigned k = 0; k < spin; k = k + 1) {
            }
            seen[i].fetch_add(1);
          }
        });
        for (auto& s : seen)
          if (s.load() != 1) bad.fetch_add(1);
      }
    });
  for (auto& t : th) t.join();
  // concurrent callers get workers of their own: CALLERS calls of width 12
  // at once grow the pool to about CALLERS x 11
  {
    std::vector<std::thread> wide;
    std::atomic<int> inside{0}, peak{0};
    for (int c = 0; c < callers; ++c)
      wide.emplace_back([&] {
        std::atomic<int> next{0};
        pool.run(12, [&] {
          for (int i; (i = next.fetch_add(1)) < 12;) {
            const int now = inside.fetch_add(1) + 1;
            int p = peak.load();
            while (now > p && !peak.compare_exchange_weak(p, now)) {
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(20));
            inside.fetch_sub(1);
          }
        });
      });
    for (auto& t : wide) t.join();
    if (peak.load() < callers * 6) {
      printf("FAIL: %d concurrent calls of width 12 peaked at %d items in flight\n", callers,
             peak.load());
      return 1;
    }
  }
  // a job that throws, in a worker's copy or in the caller's: run() returns
  // only once no copy is running (the job's state is the caller's stack)
  // and rethrows; every item is still taken exactly once
  int threw_caller = 0, threw_worker = 0;
  for (int r = 0; r < 200; ++r) {
    const size_t items = 64;
    std::vector<std::atomic<int>> seen(items);
    for (auto& s : seen) s.store(0);
    std::atomic<size_t> next{0};
    std::atomic<int> running{0};
    const std::thread::id caller = std::this_thread::get_id();
    const bool in_caller = r % 2 == 0;
    bool threw = false;
    try {
      pool.run(8, [&] {
        running.fetch_add(1);
        for (size_t i; (i = next.fetch_add(1)) < items;) {
          seen[i].fetch_add(1);
          if (i == 17 && (std::this_thread::get_id() == caller) == in_caller) {
            running.fetch_sub(1);
            throw std::runtime_error("item 17");
          }
          std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        running.fetch_sub(1);
      });
    } catch (const std::runtime_error&) {
      threw = true;
    }
    if (running.load() != 0) {
      printf("FAIL: run() returned with %d copies of the job running\n", running.load());
      return 1;
    }
    // (item 17 may have gone to the other side: then nothing threw)
    for (auto& s : seen)
      if (s.load() > 1) bad.fetch_add(1);
    if (threw) ++(in_caller ? threw_caller : threw_worker);
  }
  if (threw_caller == 0 || threw_worker == 0) {
    printf("FAIL: exceptions seen from the caller %d, from workers %d\n", threw_caller,
           threw_worker);
    return 1;
  }
  if (bad.load() || pool.workers() > cir::WorkerPool::kMaxWorkers) {
    printf("FAIL: %d items not processed exactly once\n", bad.load());
    return 1;
  }
  printf("%d callers x %d rounds ok, %zu workers\n", callers, rounds, pool.workers());
  return 0;
}
