// The complete prefix of a scan's global block order while several devices
// hash interleaved stripes of it (hash_files, scan.cpp).
//
// The order is cut into stripes of `stripe` blocks, dealt round-robin to the
// devices; each device reports, per stripe, how many of its blocks are done
// (monotone within a stripe).  The emitter may write every file whose blocks
// all lie in the prefix [0, prefix) in which every block is done, so every
// report that extends the prefix must reach it -- including a batch that only
// partly advances the first open stripe, and the completion of the last one.
// Host-only; tools/stripe_prefix_fuzz.cpp checks it against a brute-force
// prefix in the CPU suite.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace cir {

class StripePrefix {
 public:
  StripePrefix(uint64_t total_blocks, uint64_t stripe_blocks)
      : total_(total_blocks),
        stripe_(std::max<uint64_t>(1, stripe_blocks)),
        got_((size_t)((total_blocks + stripe_ - 1) / stripe_), 0) {}

  size_t stripes() const { return got_.size(); }
  uint64_t stripe_blocks() const { return stripe_; }
  // blocks in stripe st (the last one may be short)
  uint64_t stripe_len(size_t st) const {
    return std::min<uint64_t>(stripe_, total_ - (uint64_t)st * stripe_);
  }

  // Stripe st now has n blocks done.  Returns true and sets *prefix when the
  // complete prefix grew past what the last true return reported.
  bool update(size_t st, uint64_t n, uint64_t* prefix) {
    got_[st] = n;
    while (first_open_ < got_.size() && got_[first_open_] == stripe_len(first_open_)) ++first_open_;
    const uint64_t p =
        first_open_ < got_.size() ? (uint64_t)first_open_ * stripe_ + got_[first_open_] : total_;
    if (p <= reported_) return false;
    reported_ = p;
    *prefix = p;
    return true;
  }

  uint64_t reported() const { return reported_; }

 private:
  uint64_t total_, stripe_;
  std::vector<uint64_t> got_;
  size_t first_open_ = 0;
  uint64_t reported_ = 0;  // the prefix the last true update() returned
};

}  // namespace cir
