// StripePrefix (ciruela_amd/csrc/stripes.hpp) against a brute-force prefix:
// random totals, stripe sizes and device counts; every device walks its
// round-robin stripes in order in random batches, the devices interleaved at
// random.  After every update the reported prefix must equal the true
// complete prefix (so a batch that extends it is never held back, the first
// open stripe's partial batches and the last stripe's completion included),
// and a report is made exactly when that prefix grows.
//   stripe_prefix_fuzz <cases> <seed>   -> prints "ok <updates> <reports>"
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "stripes.hpp"

int main(int argc, char** argv) {
  const int cases = argc > 1 ? atoi(argv[1]) : 200;
  std::mt19937_64 rng(argc > 2 ? strtoull(argv[2], nullptr, 10) : 1);
  auto pick = [&](uint64_t lo, uint64_t hi) { return lo + rng() % (hi - lo + 1); };
  uint64_t updates = 0, reports = 0;
  for (int c = 0; c < cases; ++c) {
    const uint64_t total = pick(1, 400);
    const uint64_t stripe = pick(1, 40);
    const size_t nd = (size_t)pick(2, 8);
    cir::StripePrefix sp(total, stripe);
    std::vector<uint64_t> done(total, 0);  // per block
    // per device: its stripes, the current one and blocks done in it
    std::vector<std::vector<size_t>> mine(nd);
    for (size_t st = 0; st < sp.stripes(); ++st) mine[st % nd].push_back(st);
    std::vector<size_t> cur(nd, 0);
    std::vector<uint64_t> got(nd, 0);
    uint64_t last_true = 0;
    for (;;) {
      std::vector<size_t> live;
      for (size_t i = 0; i < nd; ++i)
        if (cur[i] < mine[i].size()) live.push_back(i);
      if (live.empty()) break;
      const size_t i = live[rng() % live.size()];
      const size_t st = mine[i][cur[i]];
      const uint64_t len = sp.stripe_len(st);
      const uint64_t step = pick(1, std::max<uint64_t>(1, len / 2 + 1));
      const uint64_t n = std::min(len, got[i] + step);
      for (uint64_t b = got[i]; b < n; ++b) done[st * stripe + b] = 1;
      got[i] = n;
      if (n == len) {
        ++cur[i];
        got[i] = 0;
      }
      uint64_t truth = 0;
      while (truth < total && done[truth]) ++truth;
      uint64_t p = ~0ull;
      const bool r = sp.update(st, n, &p);
      ++updates;
      if (r != (truth > last_true) || (r && p != truth) || sp.reported() != truth) {
        fprintf(stderr,
                "case %d: total %llu stripe %llu nd %zu: stripe %zu n %llu -> report %d prefix "
                "%llu, truth %llu (last %llu)\n",
                c, (unsigned long long)total, (unsigned long long)stripe, nd, st,
                (unsigned long long)n, (int)r, (unsigned long long)p, (unsigned long long)truth,
                (unsigned long long)last_true);
        return 1;
      }
      reports += r;
      last_true = truth;
    }
    if (sp.reported() != total) {
      fprintf(stderr, "case %d: final prefix %llu of %llu\n", c,
              (unsigned long long)sp.reported(), (unsigned long long)total);
      return 1;
    }
  }
  printf("ok %llu %llu\n", (unsigned long long)updates, (unsigned long long)reports);
  return 0;
}
