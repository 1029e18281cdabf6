// Host runtime of the block-hash path: per-device state, error plumbing and
// the pinned double-buffered staging engine shared by the host-memory entry
// points (cir_hash_blocks / cir_hash_file / cir_hash_memory / cir_scan_v1).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <sys/types.h>

#include <array>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "ciruela_blockhash.h"
#include "kernels.hpp"
#include "verify_queue.hpp"

namespace cir {

int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

// No C++ exception crosses the C ABI (a Rust caller unwinding through it is
// undefined behaviour; a C caller would be terminated): every int-returning
// entry point is a function-try-block ending in CIR_CATCH_BOUNDARY.  A failed
// host allocation (std::bad_alloc) or a thread that could not start
// (std::system_error, resource_unavailable_try_again) becomes CIR_ENOMEM,
// anything else CIR_EIO, with the exception's text in cir_last_error.
int boundary_error() noexcept;
#define CIR_CATCH_BOUNDARY \
  catch (...) {            \
    return cir::boundary_error(); \
  }

#define CIR_HIP(expr)                                  \
  do {                                                 \
    hipError_t cir_e_ = (expr);                        \
    if (cir_e_ != hipSuccess) return hip_fail(cir_e_, #expr); \
  } while (0)

// Restores the calling thread's current HIP device on scope exit.  Every
// public entry point that switches device holds one, so a caller working on
// GPU k finds GPU k current again after any cir_* call (the header's NULL
// stream means "the current device's null stream").
class DeviceGuard {
 public:
  DeviceGuard() {
    if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
  }
  ~DeviceGuard() {
    if (prev_ >= 0) (void)hipSetDevice(prev_);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;

 private:
  int prev_ = -1;
};

// One staging slot: a pinned host buffer and its device twin, plus the
// descriptor and digest buffers of the blocks packed into it.
struct Slot {
  uint8_t* h_data = nullptr;
  uint8_t* d_data = nullptr;
  uint64_t cap = 0;
  uint64_t* h_off = nullptr;
  uint32_t* h_len = nullptr;
  uint8_t* h_out = nullptr;
  uint64_t* d_off = nullptr;
  uint32_t* d_len = nullptr;
  uint8_t* d_out = nullptr;
  uint64_t cap_blk = 0;
  hipEvent_t copied = nullptr;  // H2D of this slot finished (copy stream)
  hipEvent_t done = nullptr;    // digests of this slot are back in h_out
  // timing events (created on first use, recorded only while the device's
  // record_times is set: CIR_TRACE, or cir_debug_scan_timing during a scan)
  hipEvent_t t_copy0 = nullptr, t_copy1 = nullptr, t_hash0 = nullptr, t_done = nullptr;
  bool timed = false;  // this slot's last submit recorded them
  bool busy = false;
};

// CIR_TRACE set to a non-empty value other than "0": per-batch timings on stderr.
bool trace_enabled();

// Host threads for the staged paths' copies and reads (scan readers when the
// caller asks for auto threads, the host-memory batches' packing): at most
// kMaxCopyThreads, and at most 3/4 of the CPUs this process may use (its
// cgroup CPU quota, else its affinity mask), so the threads that submit the
// uploads keep a CPU.  Config 5 on three boxes of a 16-CPU share
// (profiles/r03_s2/cfg5_threads/): 12 readers 39.1-44.1 GiB/s, 16 readers
// 32.2-42.1 (the uploads slowed to 6.4-6.7 ms per 256 MiB batch from 5.1-5.9).
unsigned host_copy_threads();
// The scan's auto_threads over ndev devices: kMaxCopyThreads readers per
// device (each device's range is read by threads / ndev of them), within 3/4
// of the process's CPUs but never fewer than the one-device count.
unsigned host_copy_threads(size_t ndev);

// How host threads fill the pinned staging slots (CIR_STAGE_COPY):
//   nt (the default): non-temporal 16-B stores -- file bytes are pread()
//     into a per-thread 512 KiB bounce buffer that stays in the core's L2
//     and streamed from there -- so a slot is written without
//     read-for-ownership and leaves no dirty lines in the CPU caches for the
//     upload's DMA reads to meet;
//   direct: pread() / memcpy() straight into the slot.
// Config 5 (50 GiB tmpfs tree, one box, alternating processes,
// profiles/r04/cfg5_copy/): direct 43.8-45.4 GiB/s with every 256 MiB
// upload at 4.8-6.2 ms while the readers run; nt 47.8-48.6 GiB/s, every
// upload 4.75 ms (the link's rate) and the reads faster too.
bool stage_copy_nt();
// Run `work` on n threads at once -- the caller and n-1 threads of a
// process-wide pool that persists across calls (created on first use, grown
// on demand) -- and return when every copy has returned.  `work` must pull
// its items from shared state (an atomic index) and return once none are
// left: copies still queued when the caller's own copy returns are dropped.
// Round 4: the host paths created their reader / copy threads per batch.
void parallel_run(unsigned n, const std::function<void()>& work);
// Run fn(i) for every i in [0, n), each on a thread of its own (one per
// device state), and return once all have returned.  A thread that cannot
// be created runs its i on the calling thread instead; an exception thrown
// by any fn(i) is rethrown after every thread has been joined (the entry
// point's CIR_CATCH_BOUNDARY turns it into a code).
void fan_out(size_t n, const std::function<void(size_t)>& fn);
// CIR_STAGE_RAMP=0: the staged host paths (scan, hash_file, hash_memory)
// start with whole-slot batches instead of ramping up from 1/8 of a slot.
bool scan_ramp();
// n bytes into a staging slot from memory / from fd at off (pread
// semantics: the count read, 0 at EOF, -1 with errno), with streaming
// stores when nt (the caller reads stage_copy_nt() once per call or batch).
void copy_staged(uint8_t* dst, const uint8_t* src, size_t n, bool nt);
ssize_t pread_staged(int fd, uint8_t* dst, size_t n, off_t off, bool nt);

struct Device {
  int id = 0;
  hipStream_t compute = nullptr;
  hipStream_t copy = nullptr;  // == compute in a CIR_INIT_ONE_SHOT context
  // per-batch timing of the staged path (slot_submit records t_* events)
  bool record_times = false;
  hipEvent_t t_ref = nullptr;  // a scan's time origin on the copy stream
  // staging slots: the batch entry points cycle through two; the directory
  // scan through all three (reads of batch k+1 overlap the H2D of k and k-1).
  static constexpr int kSlots = 3;
  Slot slot[kSlots];
  std::mutex mu;  // one host-path user at a time per device
  // device scratch of the descriptor ordering (cir_hash_blocks_dev); users on
  // different streams are ordered through `order_free`.
  std::mutex order_mu;
  void* order_scratch = nullptr;
  size_t order_cap = 0;
  hipEvent_t order_free = nullptr;
  // scratch of the bounds pass of the *_dev_bounded entry points (checked
  // lengths and flags, order.hip launch_desc_bound), kept across calls like
  // the ordering scratch; users on different streams are ordered through
  // `bound_free` (created on first use).  Taken before order_mu.
  std::mutex bound_mu;
  void* bound_scratch = nullptr;
  size_t bound_cap = 0;
  hipEvent_t bound_free = nullptr;
  // An ordered batch runs its quad part on `qstream` (a high-priority
  // stream: a hardware queue of its own) and its lane part on the caller's
  // stream, forked and joined with events (runtime.cpp create_part_streams).
  hipStream_t qstream = nullptr;
  hipEvent_t part_fork = nullptr, q_join = nullptr;
  // relayed quad chains (used on qstream only; allocated at full capacity
  // by cir_init)
  dev::RelayScratch relay;
  void* relay_mem = nullptr;
  // incremental footer chain (cir_scan_v1): own stream, state, text buffers
  std::mutex chain_mu;  // one incremental footer (scan) at a time per device
  hipStream_t chain = nullptr;
  uint64_t* chain_state = nullptr;  // 16 x u64
  uint8_t* chain_h[2] = {nullptr, nullptr};
  uint8_t* chain_d[2] = {nullptr, nullptr};
  size_t chain_cap[2] = {0, 0};
  hipEvent_t chain_done[2] = {nullptr, nullptr};
  // low-latency single-block hash (cir_blake2b256): own stream, a pinned
  // device-mapped input buffer, device scratch and a mapped digest slot
  std::mutex single_mu;
  hipStream_t single = nullptr;
  uint8_t* single_h = nullptr;
  uint8_t* single_d = nullptr;
  uint8_t* single_out = nullptr;
  size_t single_cap = 0;
  // concurrent cir_blake2b256 callers coalesced into one batch: pinned
  // descriptors + digests (h) and their device twins (d), room for
  // single_batch_cap requests
  uint8_t* single_desc_h = nullptr;
  uint8_t* single_desc_d = nullptr;
  size_t single_batch_cap = 0;
  // per-part timing of ordered batches (cir_debug_desc_timing): one set of
  // six events per recorded batch -- ordering start / end on the caller's
  // stream, quad part start / end, lane part start / end -- under order_mu
  bool timing = false;
  std::vector<std::array<hipEvent_t, 6>> tev;
  size_t tev_used = 0;
  ~Device();
  int ensure_slot(Slot& s, uint64_t bytes, uint64_t nblk);
  int ensure_timing(Slot& s);
};

// Every slot a staged loop submitted is waited for before the loop lets go
// of its device, on every return path: a loop that fails part-way (a read
// error, a failed launch) leaves no busy slot behind -- the next loop on the
// device would find it busy and retire it as one of its own batches (a
// striped scan then reported a wrapped-around progress count and emitted
// files before their digests were back).  Declare it after the device lock
// and the DeviceGuard, so it runs first with the device current.
struct SlotDrain {
  Device& d;
  ~SlotDrain() {
    for (Slot& s : d.slot)
      if (s.busy) {
        (void)hipEventSynchronize(s.done);
        s.busy = false;
      }
  }
};

// A batch of blocks already packed in a slot's host buffer:
// block k = h_data[h_off[k] .. h_off[k] + h_len[k]).
// Staging engine: the caller packs a slot, submit() uploads and hashes it
// asynchronously, wait() returns the digests in h_out.
int slot_submit(Device& d, Slot& s, uint64_t bytes, uint64_t nblk, int ht = CIR_HASH_BLAKE2B_256);
int hash_desc_ordered(Device& d, const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                      uint64_t n, uint8_t* out, hipStream_t s, int ht = CIR_HASH_BLAKE2B_256,
                      bool warm_only = false);
bool valid_hash_type(int ht);
int slot_wait(Device& d, Slot& s);

}  // namespace cir

namespace cir {
// cir_debug_scan_timing: one row per staged batch of the last scans, one
// phase record per scan (fields: include/ciruela_blockhash.h)
constexpr int kScanBatchFields = 10;
constexpr int kScanPhaseFields = 10;
static_assert(kScanBatchFields == CIR_SCAN_BATCH_FIELDS && kScanPhaseFields == CIR_SCAN_PHASE_FIELDS,
              "scan stats layout");
struct ScanStats {
  std::mutex mu;
  bool on = false;
  std::vector<std::array<double, kScanBatchFields>> batches;
  std::array<double, kScanPhaseFields> phases{};
  size_t scans = 0;
};
}  // namespace cir


struct cir_ctx {
  std::vector<std::unique_ptr<cir::Device>> devs;
  uint64_t staging = 0;
  // where cir_scan_v1 hashes an index's footer: CIR_FOOTER_HOST (one host
  // thread beside the scan) or CIR_FOOTER_GPU (the resumable single-chain
  // kernel on device 0's chain stream)
  int footer = CIR_FOOTER_HOST;
  cir::ScanStats stats;
  // cir_verify_submit's queue and worker (verify_queue.hpp), created on
  // first use; declared last, so it is stopped (its worker drained and
  // joined) before anything its hashing uses goes away
  std::mutex av_mu;
  std::unique_ptr<cir::VerifyQueue> av;
};

namespace cir {
Device* stream_device(cir_ctx* ctx, hipStream_t s);
}  // namespace cir
