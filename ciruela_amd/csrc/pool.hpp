// The host worker pool behind parallel_run (runtime.hpp): the staged host
// paths' reader and copy threads (scan.cpp run_reads, runtime.cpp
// parallel_pieces / parallel_items) persist across batches instead of being
// created and joined per batch.  Header-only so that a CPU stress test can
// build it alone under ThreadSanitizer (tools/pool_stress.cpp).
#pragma once
#include <algorithm>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <mutex>
#include <system_error>
#include <thread>
#include <vector>

namespace cir {

// A call queues n-1 tickets for its job and runs the job itself; a worker
// takes a ticket, runs the job and counts it off.  The job pulls its items
// from shared state and returns when none are left, so once the caller's own
// run returns, tickets nobody has started are dropped rather than waited
// for: a busy pool delays a call by at most the tickets already running.
// Exceptions: a job that throws (in the caller or in a worker) is still
// waited for everywhere it runs, and run() rethrows the first exception once
// no copy is left running; a worker thread that cannot be created leaves its
// ticket to the running workers or to the caller's own run.
class WorkerPool {
 public:
  static constexpr size_t kMaxWorkers = 256;

  WorkerPool() = default;
  WorkerPool(const WorkerPool&) = delete;
  WorkerPool& operator=(const WorkerPool&) = delete;
  // (the process-wide pool is never destroyed; a pool that is waits for its
  // workers, which must be idle: no run() in progress)
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
  }

  void run(unsigned n, const std::function<void()>& fn) {
    if (n <= 1) {
      fn();
      return;
    }
    Job job;
    job.fn = &fn;
    {
      std::lock_guard<std::mutex> lk(mu_);
      unsigned queued = 0;
      try {
        for (; queued + 1 < n; ++queued) q_.push_back(&job);
      } catch (...) {
        // out of memory part-way: take this job's tickets back (the last
        // `queued` entries: the lock is held) and run it on this thread only
        // -- a ticket left queued would point at `job` after it is gone
        for (; queued > 0; --queued) q_.pop_back();
      }
      job.pending = queued;
      // a worker for every ticket queued or running, concurrent callers
      // included (several devices' readers at once)
      const size_t want = std::min<size_t>(busy_ + q_.size(), kMaxWorkers);
      try {
        while (th_.size() < want) th_.emplace_back([this] { loop(); });
      } catch (...) {
        // (no thread for now -- system_error, or bad_alloc for its state or
        // the vector: the tickets wait for a free worker or are dropped once
        // the caller's own run has done the work)
      }
    }
    cv_.notify_all();
    std::exception_ptr mine;
    try {
      fn();
    } catch (...) {
      mine = std::current_exception();
    }
    std::unique_lock<std::mutex> lk(mu_);
    for (auto it = q_.begin(); it != q_.end();) {
      if (*it == &job) {
        it = q_.erase(it);
        --job.pending;
      } else {
        ++it;
      }
    }
    job.done.wait(lk, [&] { return job.pending == 0; });
    if (!mine) mine = job.error;
    lk.unlock();
    if (mine) std::rethrow_exception(mine);
  }

  size_t workers() {
    std::lock_guard<std::mutex> lk(mu_);
    return th_.size();
  }

 private:
  struct Job {
    const std::function<void()>* fn = nullptr;
    unsigned pending = 0;  // tickets queued or running (under mu_)
    std::condition_variable done;
    std::exception_ptr error;  // the first a worker's copy threw (under mu_)
  };

  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stopping
      Job* j = q_.front();
      q_.pop_front();
      ++busy_;
      lk.unlock();
      std::exception_ptr e;
      try {
        (*j->fn)();
      } catch (...) {
        e = std::current_exception();
      }
      lk.lock();
      if (e && !j->error) j->error = e;
      --busy_;
      if (--j->pending == 0) j->done.notify_all();
    }
  }

  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job*> q_;
  std::vector<std::thread> th_;
  size_t busy_ = 0;  // workers running a ticket
  bool stop_ = false;
};

}  // namespace cir
