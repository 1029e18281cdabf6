// The daemon's per-block verify under load, from C threads: C "connections"
// each receive 32 KiB blocks one at a time and hand each to the bounded
// asynchronous verify (cir_verify_submit, non-blocking, as INTEGRATION.md §3
// wires FetchBlock::poll, src/daemon/tracking/fetch_blocks.rs:77); a full
// queue (CIR_EAGAIN) is a refused fetch, retried after a short back-off; one
// block in 20 carries a wrong expected digest (the mismatch branch, :91-103)
// and one in 100 is abandoned while it verifies (cir_verify_forget, a peer
// that went away).  Every outcome must match the block's expected state.
// Prints blocks/s, GB/s, latency percentiles (submit -> outcome) and the
// queue's own counters (cir_verify_stats).
//
//   build/verify_daemon_sim [connections=8] [seconds=5] [max_bytes_mib=64] [window_us=200]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <thread>
#include <vector>

#include "ciruela_blockhash.h"

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int conns = argc > 1 ? atoi(argv[1]) : 8;
  const double seconds = argc > 2 ? atof(argv[2]) : 5.0;
  const uint64_t max_bytes = (uint64_t)(argc > 3 ? atoi(argv[3]) : 64) << 20;
  const uint32_t window_us = argc > 4 ? (uint32_t)atoi(argv[4]) : 200;
  constexpr size_t kBs = 32768;
  constexpr int kPool = 4096;  // distinct blocks, reused
  cir_ctx* ctx = nullptr;
  if (cir_init(&ctx, 1u, 64ull << 20)) {
    fprintf(stderr, "cir_init: %s\n", cir_last_error());
    return 1;
  }
  std::vector<uint8_t> pool((size_t)kPool * kBs);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (auto& b : pool) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    b = (uint8_t)x;
  }
  // the index's digests of the pool (one batch on the GPU)
  std::vector<uint64_t> off(kPool);
  std::vector<uint32_t> len(kPool, (uint32_t)kBs);
  for (int i = 0; i < kPool; ++i) off[i] = (uint64_t)i * kBs;
  std::vector<uint8_t> want((size_t)kPool * 32);
  if (cir_hash_blocks(ctx, pool.data(), off.data(), len.data(), kPool, want.data())) {
    fprintf(stderr, "cir_hash_blocks: %s\n", cir_last_error());
    return 1;
  }
  if (cir_verify_limits(ctx, max_bytes, 0, CIR_VERIFY_NONBLOCK) ||
      cir_verify_window(ctx, window_us, 4096)) {
    fprintf(stderr, "verify setup: %s\n", cir_last_error());
    return 1;
  }
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> done_blocks{0}, refused{0}, wrong{0}, errors{0}, forgotten{0};
  std::vector<std::vector<double>> lat(conns);
  std::vector<std::thread> th;
  const double t0 = now_s();
  for (int c = 0; c < conns; ++c)
    th.emplace_back([&, c] {
      struct Pending {
        uint64_t ticket;
        double t;
        bool good;
      };
      std::deque<Pending> inflight;
      uint64_t k = (uint64_t)c * 7919;
      uint8_t bad[32];
      auto reap = [&](bool all) {
        while (!inflight.empty()) {
          Pending& p = inflight.front();
          int st = 0;
          const int rc = all ? cir_verify_wait(ctx, p.ticket, &st) : cir_verify_poll(ctx, p.ticket, &st);
          if (rc) {
            ++errors;
            inflight.pop_front();
            continue;
          }
          if (!all && st == 0) return;  // oldest still pending
          if ((st == 1) != p.good) ++wrong;  // wait: 1/0, poll: 1/2
          lat[c].push_back(now_s() - p.t);
          ++done_blocks;
          inflight.pop_front();
        }
      };
      while (!stop.load(std::memory_order_relaxed)) {
        const int i = (int)(k++ % kPool);
        const bool good = k % 20 != 3;
        const uint8_t* exp = want.data() + 32 * i;
        if (!good) {
          memcpy(bad, exp, 32);
          bad[k % 32] ^= 0x5a;
          exp = bad;
        }
        uint64_t ticket = 0;
        const double ts = now_s();
        int rc;
        while ((rc = cir_verify_submit(ctx, CIR_HASH_BLAKE2B_256, pool.data() + (size_t)i * kBs, kBs,
                                       exp, &ticket)) == CIR_EAGAIN) {
          ++refused;  // a refused fetch: back off, fetch again
          std::this_thread::sleep_for(std::chrono::microseconds(50));
          if (stop.load(std::memory_order_relaxed)) break;
        }
        if (rc == CIR_EAGAIN) break;
        if (rc) {
          ++errors;
          continue;
        }
        if (k % 100 == 17) {  // the peer went away while the block verifies
          if (cir_verify_forget(ctx, ticket)) ++errors;
          ++forgotten;
        } else {
          inflight.push_back({ticket, ts, good});
        }
        reap(false);
      }
      reap(true);
    });
  std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
  stop = true;
  for (auto& t : th) t.join();
  const double dt = now_s() - t0;
  std::vector<double> all;
  for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double q) { return all.empty() ? 0.0 : all[(size_t)(q * (all.size() - 1))] * 1e6; };
  uint64_t st[CIR_VERIFY_STATS_FIELDS] = {};
  cir_verify_stats(ctx, st);
  printf("connections %d, %.1f s, max_bytes %llu MiB, window %u us: %llu blocks verified "
         "(%.0f blocks/s, %.2f GB/s), latency p50 %.0f us p90 %.0f us p99 %.0f us\n",
         conns, dt, (unsigned long long)(max_bytes >> 20), window_us,
         (unsigned long long)done_blocks.load(), done_blocks / dt, done_blocks * kBs / dt / 1e9,
         pct(0.5), pct(0.9), pct(0.99));
  printf("  refused %llu, forgotten %llu, wrong outcomes %llu, errors %llu; queue: peak %llu MiB "
         "held, %llu batches, %llu outcomes held at the end, %llu bytes held at the end\n",
         (unsigned long long)refused.load(), (unsigned long long)forgotten.load(),
         (unsigned long long)wrong.load(), (unsigned long long)errors.load(),
         (unsigned long long)(st[1] >> 20), (unsigned long long)st[7], (unsigned long long)st[3],
         (unsigned long long)st[0]);
  const bool ok = wrong == 0 && errors == 0 && st[1] <= max_bytes;
  printf("%s\n", ok ? "ok" : "FAIL");
  return ok ? 0 : 1;
}
