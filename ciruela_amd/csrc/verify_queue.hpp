// The asynchronous per-block verify's queue (cir_verify_submit / poll / wait
// / forget / window / limits / stats; row f2, the daemon's per-block caller,
// src/daemon/tracking/fetch_blocks.rs:77).
//
// FetchBlock::poll hashes each received block as it arrives.  submit() packs
// one block (one copy) into the arena of the batch being formed for its hash
// type and returns a ticket at once; a worker thread takes the oldest batch
// once it is full (max_batch blocks, or its arena) or `window` after its
// first block, and hands it to `hash` -- in the library, one host batch of
// cir_hash_blocks_ht straight from that arena; callers poll or wait for their
// ticket.  One batch costs about one chain's latency whatever its size below
// a few thousand blocks, so blocks that arrive together share
// it.
//
// Bounds (limits()): the block bytes accepted and not yet verified stay
// within max_bytes -- a submit that would pass it sends the forming batches
// to the worker and waits for room or, non-blocking, returns CIR_EAGAIN
// without taking the block (the daemon's backpressure); at most max_results
// finished outcomes are held for their tickets, the oldest dropped beyond
// that; forget() drops a ticket the caller no longer wants (the reference
// retries such a block elsewhere, :91-103).
//
// Host-only and independent of HIP: tools/verify_queue_stress.cpp drives it
// with a test hasher under ThreadSanitizer in the CPU suite.
#pragma once

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "ciruela_blockhash.h"

namespace cir {

class VerifyQueue {
 public:
  // hash(ht, arena, off, len, n, out) -> 0 or a CIR_E* code (*err: detail):
  // the 32-byte digests of the n blocks arena[off[i], off[i] + len[i]).
  using HashFn = std::function<int(int ht, const uint8_t* arena, const uint64_t* off,
                                   const uint32_t* len, size_t n, uint8_t* out, std::string* err)>;
  static constexpr uint64_t kMaxBytes = 256ull << 20;  // two batches of 4096 x 32 KiB
  static constexpr uint64_t kMaxResults = 1ull << 20;
  // a batch's arena: half the byte bound (a batch forms while the previous
  // one is verified), at most one full batch of 32 KiB blocks -- the bound
  // caps what is admitted, not what one batch allocates, so a large bound
  // costs nothing up front; only a block larger than this gets an arena of
  // its own size
  static constexpr uint64_t kArenaMax = 4096ull * 32768;

  explicit VerifyQueue(HashFn hash) : hash_(std::move(hash)) {
    worker_ = std::thread([this] { run(); });
  }
  // verifies what is queued, then joins the worker
  ~VerifyQueue() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
  }
  VerifyQueue(const VerifyQueue&) = delete;
  VerifyQueue& operator=(const VerifyQueue&) = delete;

  // 0 with *ticket, CIR_EAGAIN (non-blocking, no room; *err says why) or
  // CIR_ENOMEM (a new batch's arena could not be allocated)
  int submit(int ht, const uint8_t* data, size_t n, const uint8_t* expected, uint64_t* ticket,
             std::string* err) {
    std::unique_lock<std::mutex> lk(mu_);
    // room: a block always fits an empty queue, whatever its size.  Without
    // room, the batches being formed go to the worker now instead of waiting
    // out their window: nothing larger can join them until room frees anyway.
    while (held_ && held_ + n > max_bytes_) {
      bool sealed = false;
      for (auto& q : queue_)
        if (!q->sealed) q->sealed = sealed = true;
      if (sealed) cv_.notify_one();
      if (nonblocking_) {
        ++refused_;
        *err = "verify queue full (" + std::to_string(held_) + " of " + std::to_string(max_bytes_) +
               " bytes held)";
        return CIR_EAGAIN;
      }
      room_cv_.wait(lk);
    }
    Batch* b = nullptr;
    for (auto it = queue_.rbegin(); it != queue_.rend(); ++it)
      if (!(*it)->sealed && (*it)->ht == ht) {
        b = it->get();
        break;
      }
    if (b && b->used + n > b->cap) {
      b->sealed = true;  // full: this block opens the next batch
      b = nullptr;
    }
    if (!b) {
      auto nb = std::make_unique<Batch>();
      nb->ht = ht;
      // one batch's arena (arena_bytes(); a spare arena of a verified batch
      // is reused: its pages are already faulted in), or -- when that much
      // cannot be allocated -- one just for this block
      if (!arena_for(*nb, std::max<uint64_t>(n, arena_bytes())) &&
          (n >= arena_bytes() || !arena_for(*nb, std::max<uint64_t>(n, 1)))) {
        *err = "verify batch arena of " + std::to_string(std::max<uint64_t>(n, 1)) + " bytes";
        return CIR_ENOMEM;
      }
      nb->first = std::chrono::steady_clock::now();
      b = nb.get();
      queue_.push_back(std::move(nb));
    }
    const uint64_t at = b->used;
    b->used += n;
    b->off.push_back(at);
    b->len.push_back((uint32_t)n);
    b->expected.insert(b->expected.end(), expected, expected + 32);
    const uint64_t t = next_ticket_++;
    b->tickets.push_back(t);
    if (b->tickets.size() >= max_batch_) b->sealed = true;
    pending_.insert(t);
    held_ += n;
    peak_ = std::max(peak_, held_);
    *ticket = t;
    // the block's bytes are copied outside the lock, into the space just
    // reserved; the worker hashes a batch only once its writers are done
    ++b->writers;
    lk.unlock();
    cv_.notify_one();
    if (n) memcpy(b->arena.get() + at, data, n);
    lk.lock();
    if (--b->writers == 0) writers_cv_.notify_all();
    return CIR_OK;
  }

  // 0 pending, 1 match, 2 mismatch (consumed when reported), a CIR_E* code
  // of the failed batch, or CIR_ENOTFOUND (*err set for both)
  int poll(uint64_t ticket, std::string* err) {
    std::lock_guard<std::mutex> lk(mu_);
    if (pending_.count(ticket)) return 0;
    auto r = done_.find(ticket);
    if (r == done_.end()) {
      *err = "unknown, consumed, forgotten or expired ticket";
      return CIR_ENOTFOUND;
    }
    return take(r, err);
  }

  // blocks: 1 match, 2 mismatch, or an error code as poll()
  int wait(uint64_t ticket, std::string* err) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!pending_.count(ticket) && !done_.count(ticket)) {
      *err = "unknown, consumed, forgotten or expired ticket";
      return CIR_ENOTFOUND;
    }
    done_cv_.wait(lk, [&] { return !pending_.count(ticket); });
    // (consumed by another caller's poll, forgotten or expired meanwhile)
    auto r = done_.find(ticket);
    if (r == done_.end()) {
      *err = "ticket consumed, forgotten or expired while waiting";
      return CIR_ENOTFOUND;
    }
    return take(r, err);
  }

  // 0, or CIR_ENOTFOUND.  A pending ticket is still hashed with its batch
  // (its bytes are released with it) but its outcome is never held.
  int forget(uint64_t ticket, std::string* err) {
    std::lock_guard<std::mutex> lk(mu_);
    if (pending_.erase(ticket)) {
      ++forgotten_;
      done_cv_.notify_all();
      return CIR_OK;
    }
    auto r = done_.find(ticket);
    if (r == done_.end()) {
      *err = "unknown, consumed, forgotten or expired ticket";
      return CIR_ENOTFOUND;
    }
    errors_.erase(ticket);
    done_.erase(r);
    ++forgotten_;
    return CIR_OK;
  }

  void window(uint32_t window_us, uint32_t max_batch) {
    std::lock_guard<std::mutex> lk(mu_);
    window_us_ = window_us;
    max_batch_ = std::max<uint32_t>(1, max_batch);
  }

  // 0 = the default for either bound
  void limits(uint64_t max_bytes, uint64_t max_results, bool nonblocking) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      max_bytes_ = max_bytes ? max_bytes : kMaxBytes;
      max_results_ = max_results ? max_results : kMaxResults;
      nonblocking_ = nonblocking;
      evict();
    }
    room_cv_.notify_all();
  }

  void stats(uint64_t out[CIR_VERIFY_STATS_FIELDS]) {
    std::lock_guard<std::mutex> lk(mu_);
    const uint64_t v[CIR_VERIFY_STATS_FIELDS] = {held_,         peak_,    pending_.size(),
                                                 done_.size(),  expired_, forgotten_,
                                                 refused_,      batches_};
    memcpy(out, v, sizeof(v));
  }

 private:
  // a batch being formed or waiting for the worker: its blocks packed into
  // one arena as they were submitted
  struct Batch {
    int ht = 0;
    std::unique_ptr<uint8_t[]> arena;  // cap bytes, the first `used` taken
    uint64_t cap = 0, used = 0;
    int writers = 0;  // submitters still copying into the arena
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
    std::vector<uint8_t> expected;
    std::vector<uint64_t> tickets;
    std::chrono::steady_clock::time_point first;
    bool sealed = false;  // full (or pressed for room): taken without waiting
  };

  // a held outcome, consumed; caller holds mu_
  int take(std::map<uint64_t, int>::iterator it, std::string* err) {
    const uint64_t ticket = it->first;
    const int r = it->second;
    done_.erase(it);
    if (r < 0) {
      *err = errors_[ticket];
      errors_.erase(ticket);
    }
    return r;
  }

  // the standard arena of a batch (see kArenaMax); caller holds mu_
  uint64_t arena_bytes() const {
    return std::max<uint64_t>(1, std::min<uint64_t>(max_bytes_ / 2, kArenaMax));
  }

  // b gets an arena of at least `bytes`: a spare one when one is big enough;
  // false if it cannot be allocated (caller holds mu_)
  bool arena_for(Batch& b, uint64_t bytes) {
    for (auto it = spare_.begin(); it != spare_.end(); ++it)
      if (it->second >= bytes) {
        b.arena = std::move(it->first);
        b.cap = it->second;
        spare_.erase(it);
        return true;
      }
    // not value-initialised: untouched pages cost nothing
    b.arena.reset(new (std::nothrow) uint8_t[bytes]);
    b.cap = b.arena ? bytes : 0;
    return b.arena != nullptr;
  }

  void evict() {  // caller holds mu_
    while (done_.size() > max_results_) {
      errors_.erase(done_.begin()->first);
      done_.erase(done_.begin());
      ++expired_;
    }
  }

  void run() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      // idle for a second with spare arenas: give their memory back
      if (queue_.empty() && !stop_ && !spare_.empty() &&
          !cv_.wait_for(lk, std::chrono::seconds(1), [&] { return stop_ || !queue_.empty(); }))
        spare_.clear();
      cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
      if (queue_.empty()) return;  // stopped and drained
      Batch* b = queue_.front().get();
      const auto deadline = b->first + std::chrono::microseconds(window_us_);
      cv_.wait_until(lk, deadline, [&] { return stop_ || b->sealed; });
      std::unique_ptr<Batch> bp = std::move(queue_.front());
      queue_.pop_front();
      bp->sealed = true;  // (no more appends)
      writers_cv_.wait(lk, [&] { return bp->writers == 0; });  // every block copied in
      lk.unlock();
      const size_t n = bp->tickets.size();
      static const uint8_t empty = 0;
      std::string err;
      std::unique_ptr<uint8_t[]> got(new (std::nothrow) uint8_t[32 * n]);
      const int rc = got ? hash_(bp->ht, bp->used ? bp->arena.get() : &empty, bp->off.data(),
                                 bp->len.data(), n, got.get(), &err)
                         : (err = "verify batch digests", CIR_ENOMEM);
      const uint64_t bytes = bp->used;
      lk.lock();
      for (size_t i = 0; i < n; ++i) {
        const uint64_t t = bp->tickets[i];
        if (!pending_.erase(t)) continue;  // forgotten meanwhile: no outcome held
        if (rc) {
          done_[t] = rc;
          errors_[t] = err;
        } else {
          done_[t] = memcmp(got.get() + 32 * i, bp->expected.data() + 32 * i, 32) == 0 ? 1 : 2;
        }
      }
      held_ -= bytes;
      ++batches_;
      evict();
      // keep the arena for a later batch (at most two spares, within the
      // byte bound's two batches); the rest is freed outside the lock
      if (spare_.size() < 2 && bp->cap <= arena_bytes())
        spare_.emplace_back(std::move(bp->arena), bp->cap);
      room_cv_.notify_all();
      done_cv_.notify_all();
      lk.unlock();
      bp.reset();
      lk.lock();
    }
  }

  HashFn hash_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_, room_cv_, writers_cv_;
  std::deque<std::unique_ptr<Batch>> queue_;
  std::unordered_set<uint64_t> pending_;  // submitted, outcome not yet known
  std::map<uint64_t, int> done_;          // outcome held: 1 match, 2 mismatch, < 0 error
  std::unordered_map<uint64_t, std::string> errors_;
  std::vector<std::pair<std::unique_ptr<uint8_t[]>, uint64_t>> spare_;  // arenas and sizes
  uint64_t next_ticket_ = 1;
  uint64_t held_ = 0, peak_ = 0;  // block bytes accepted and not yet verified
  uint64_t max_bytes_ = kMaxBytes, max_results_ = kMaxResults;
  bool nonblocking_ = false;
  uint32_t window_us_ = 200, max_batch_ = 4096;
  uint64_t expired_ = 0, forgotten_ = 0, refused_ = 0, batches_ = 0;
  bool stop_ = false;
  std::thread worker_;  // last: started after every member above exists
};

}  // namespace cir
