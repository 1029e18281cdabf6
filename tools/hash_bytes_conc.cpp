// Concurrent callers of the drop-in BlockHash::hash_bytes (cir_blake2b256)
// from C threads, without Python in the way: T threads each hash M blocks
// of B bytes, one call per block; prints the wall time per call against one
// thread's.  The library coalesces callers that arrive while a launch runs
// (runtime.cpp single_coalesced).  Every digest is checked against the
// first thread's single-call result for the same block.
//
//   build/hash_bytes_conc [block_bytes=32768] [calls_per_thread=64]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

#include "ciruela_blockhash.h"

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t bs = argc > 1 ? (size_t)atoll(argv[1]) : 32768;
  const int m = argc > 2 ? atoi(argv[2]) : 64;
  const int nblk = 256;
  std::vector<uint8_t> data((size_t)nblk * bs);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (auto& b : data) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    b = (uint8_t)x;
  }
  std::vector<uint8_t> want((size_t)nblk * 32);
  for (int i = 0; i < nblk; ++i)
    if (cir_blake2b256(data.data() + (size_t)i * bs, bs, want.data() + 32 * i)) {
      fprintf(stderr, "cir_blake2b256: %s\n", cir_last_error());
      return 1;
    }
  double one = 0;
  for (int threads : {1, 2, 4, 8, 16, 32, 64}) {
    std::vector<std::thread> th;
    std::vector<int> bad(threads, 0);
    const double t0 = now_s();
    for (int t = 0; t < threads; ++t)
      th.emplace_back([&, t] {
        uint8_t out[32];
        for (int k = 0; k < m; ++k) {
          const int i = (t * 7 + k) % nblk;
          if (cir_blake2b256(data.data() + (size_t)i * bs, bs, out) ||
              memcmp(out, want.data() + 32 * i, 32) != 0)
            ++bad[t];
        }
      });
    for (auto& t : th) t.join();
    const double dt = now_s() - t0;
    int nbad = 0;
    for (int b : bad) nbad += b;
    const double per = dt / (threads * m) * 1e6;
    if (threads == 1) one = per;
    printf("threads %2d: %5d calls of %zu B in %8.2f ms = %7.1f us per call (%.1fx one thread)%s\n",
           threads, threads * m, bs, dt * 1e3, per, one / per, nbad ? " MISMATCH" : "");
    if (nbad) return 1;
  }
  return 0;
}
