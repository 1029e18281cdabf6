// The host worker pool (ciruela_amd/csrc/pool.hpp) under ThreadSanitizer:
// CALLERS threads each make ROUNDS parallel_run-style calls of random width
// over a random number of items pulled from an atomic index (as the staged
// paths' readers do); every item must be processed exactly once per call,
// and no call may hang while the others keep the pool busy.
//   pool_stress CALLERS ROUNDS
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <random>
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
  if (bad.load() || pool.workers() > cir::WorkerPool::kMaxWorkers) {
    printf("FAIL: %d items not processed exactly once\n", bad.load());
    return 1;
  }
  printf("%d callers x %d rounds ok, %zu workers\n", callers, rounds, pool.workers());
  return 0;
}
