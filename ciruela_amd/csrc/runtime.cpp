// C ABI of the block-hash path: context, device-resident entry points and the
// host-memory entry points (pinned double-buffered staging, one worker thread
// per device).  See include/ciruela_blockhash.h for the reference interface
// each entry point replaces.
#include "runtime.hpp"

#include "pool.hpp"

#include <emmintrin.h>
#include <errno.h>
#include <sched.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <exception>
#include <new>
#include <system_error>
#include <thread>
#include <unordered_map>

namespace cir {

static thread_local std::string t_last_error;

int fail(int code, const std::string& msg) {
  t_last_error = msg;
  return code;
}

int boundary_error() noexcept {
  int code = CIR_EIO;
  const char* what = "unknown exception";
  try {
    throw;  // the exception being handled by the entry point's catch (...)
  } catch (const std::bad_alloc& e) {
    code = CIR_ENOMEM;
    what = e.what();
  } catch (const std::system_error& e) {
    if (e.code() == std::errc::resource_unavailable_try_again) code = CIR_ENOMEM;
    what = e.what();
  } catch (const std::exception& e) {
    what = e.what();
  } catch (...) {
  }
  try {
    t_last_error = std::string("C++ exception in the library: ") + what;
  } catch (...) {
  }
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(e == hipErrorOutOfMemory ? CIR_ENOMEM : CIR_EHIP,
              std::string(what) + ": " + hipGetErrorString(e));
}

Device::~Device() {
  DeviceGuard guard;
  (void)hipSetDevice(id);
  for (Slot& s : slot) {
    if (s.done) (void)hipEventSynchronize(s.done);
    (void)hipHostFree(s.h_data);
    (void)hipHostFree(s.h_off);
    (void)hipHostFree(s.h_len);
    (void)hipHostFree(s.h_out);
    (void)hipFree(s.d_data);
    (void)hipFree(s.d_off);
    (void)hipFree(s.d_len);
    (void)hipFree(s.d_out);
    if (s.copied) (void)hipEventDestroy(s.copied);
    if (s.done) (void)hipEventDestroy(s.done);
    for (hipEvent_t e : {s.t_copy0, s.t_copy1, s.t_hash0, s.t_done})
      if (e) (void)hipEventDestroy(e);
  }
  if (t_ref) (void)hipEventDestroy(t_ref);
  if (chain) (void)hipStreamSynchronize(chain);
  for (int k = 0; k < 2; ++k) {
    (void)hipHostFree(chain_h[k]);
    (void)hipFree(chain_d[k]);
    if (chain_done[k]) (void)hipEventDestroy(chain_done[k]);
  }
  (void)hipFree(chain_state);
  if (chain) (void)hipStreamDestroy(chain);
  for (auto& set : tev)
    for (hipEvent_t e : set)
      if (e) (void)hipEventDestroy(e);
  if (bound_free) (void)hipEventSynchronize(bound_free);
  (void)hipFree(bound_scratch);
  if (bound_free) (void)hipEventDestroy(bound_free);
  if (order_free) (void)hipEventSynchronize(order_free);
  (void)hipFree(order_scratch);
  if (order_free) (void)hipEventDestroy(order_free);
  if (qstream) (void)hipStreamSynchronize(qstream);
  (void)hipFree(relay_mem);
  if (part_fork) (void)hipEventDestroy(part_fork);
  if (q_join) (void)hipEventDestroy(q_join);
  if (qstream) (void)hipStreamDestroy(qstream);
  if (single) (void)hipStreamSynchronize(single);
  (void)hipHostFree(single_h);
  (void)hipHostFree(single_out);
  (void)hipFree(single_d);
  (void)hipHostFree(single_desc_h);
  (void)hipFree(single_desc_d);
  if (single) (void)hipStreamDestroy(single);
  if (compute) (void)hipStreamDestroy(compute);
  if (copy && copy != compute) (void)hipStreamDestroy(copy);
}

bool trace_enabled() {
  static const bool on = [] {
    const char* v = std::getenv("CIR_TRACE");
    return v && *v && strcmp(v, "0") != 0;
  }();
  return on;
}

// 12 vs 16 in one lease, alternating builds (profiles/r03_s2/cfg5_threads/
// ab_copy_threads_12_vs_16.log): config 5 43.7 / 38.5 vs 38.3 / 35.3 GiB/s,
// config 2 from host memory 51.0 / 51.7 vs 50.6 / 50.9.
constexpr unsigned kMaxCopyThreads = 12;

// CPUs this process may run on: the affinity mask, capped by the cgroup CPU
// quota (v2: "max" or "quota period" in /sys/fs/cgroup/cpu.max; v1:
// cpu.cfs_quota_us / cpu.cfs_period_us, -1 = none).
static unsigned usable_cpus() {
  unsigned n = 0;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = (unsigned)CPU_COUNT(&set);
  if (n == 0) n = std::max(1u, std::thread::hardware_concurrency());
  long long quota = -1, period = 0;
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0)
      quota = strtoll(q, nullptr, 10);
    fclose(f);
  } else if (FILE* fq = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
    if (fscanf(fq, "%lld", &quota) != 1) quota = -1;
    fclose(fq);
    if (FILE* fp = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
      if (fscanf(fp, "%lld", &period) != 1) period = 0;
      fclose(fp);
    }
  }
  if (quota > 0 && period > 0)
    n = std::min<unsigned>(n, (unsigned)std::max<long long>(1, quota / period));
  return n;
}

unsigned host_copy_threads() {
  static const unsigned n = std::max(1u, std::min(kMaxCopyThreads, usable_cpus() * 3u / 4u));
  return n;
}

unsigned host_copy_threads(size_t ndev) {
  if (ndev <= 1) return host_copy_threads();
  const unsigned share = std::max(host_copy_threads(), usable_cpus() * 3u / 4u);
  return (unsigned)std::min<size_t>(share, (size_t)kMaxCopyThreads * ndev);
}

bool stage_copy_nt() {  // read per API call / batch: tests switch it within one process
  const char* v = std::getenv("CIR_STAGE_COPY");
  return !(v && strcmp(v, "direct") == 0);
}

static WorkerPool& pool() {  // never destroyed: a context's threads may still use it at exit
  static WorkerPool* p = new WorkerPool;
  return *p;
}

void parallel_run(unsigned n, const std::function<void()>& work) { pool().run(n, work); }

void fan_out(size_t n, const std::function<void(size_t)>& fn) {
  std::vector<std::exception_ptr> errs(n);
  auto one = [&](size_t i) {
    try {
      fn(i);
    } catch (...) {
      errs[i] = std::current_exception();
    }
  };
  std::vector<std::thread> th;
  std::vector<size_t> here;
  th.reserve(n);
  here.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    try {
      th.emplace_back(one, i);
    } catch (...) {
      // no thread (system_error, or bad_alloc for its state): run it on this
      // one below.  (`here` was reserved: the push cannot throw, so no
      // exception leaves while `th` holds joinable threads.)
      here.push_back(i);
    }
  }
  for (size_t i : here) one(i);
  for (auto& t : th) t.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}

bool scan_ramp() {  // read per call
  const char* v = std::getenv("CIR_STAGE_RAMP");
  return !(v && strcmp(v, "0") == 0);
}

// 16-B aligned non-temporal stores; the unaligned head and the tail with
// plain stores; sfence so the bytes are globally visible before the caller
// hands the slot to the copy engine.
static void stream_copy(uint8_t* dst, const uint8_t* src, size_t n) {
  while (n && (reinterpret_cast<uintptr_t>(dst) & 15u)) {
    *dst++ = *src++;
    --n;
  }
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128((const __m128i*)(src + i));
    const __m128i b = _mm_loadu_si128((const __m128i*)(src + i + 16));
    const __m128i c = _mm_loadu_si128((const __m128i*)(src + i + 32));
    const __m128i e = _mm_loadu_si128((const __m128i*)(src + i + 48));
    _mm_stream_si128((__m128i*)(dst + i), a);
    _mm_stream_si128((__m128i*)(dst + i + 16), b);
    _mm_stream_si128((__m128i*)(dst + i + 32), c);
    _mm_stream_si128((__m128i*)(dst + i + 48), e);
  }
  memcpy(dst + i, src + i, n - i);
  _mm_sfence();
}

void copy_staged(uint8_t* dst, const uint8_t* src, size_t n, bool nt) {
  if (nt && n >= 4096)
    stream_copy(dst, src, n);
  else
    memcpy(dst, src, n);
}

// One bounce buffer per reading thread (the pool's workers persist, so each
// keeps its buffer warm in its core's L2).
constexpr size_t kBounce = 512u << 10;

ssize_t pread_staged(int fd, uint8_t* dst, size_t n, off_t off, bool nt) {
  if (!nt || n < 4096) return ::pread(fd, dst, n, off);
  thread_local std::unique_ptr<uint8_t[]> tl_bounce;
  if (!tl_bounce) tl_bounce.reset(new uint8_t[kBounce]);
  uint8_t* b = tl_bounce.get();
  size_t got = 0;
  ssize_t last = 0;
  while (got < n) {
    const size_t want = std::min(kBounce, n - got);
    last = ::pread(fd, b, want, off + (off_t)got);
    if (last < 0 && errno == EINTR) continue;
    if (last <= 0) break;
    stream_copy(dst + got, b, (size_t)last);
    got += (size_t)last;
    if ((size_t)last < want) break;  // a short read (EOF): the caller decides
  }
  if (got > 0) return (ssize_t)got;
  return last;  // 0 at EOF, -1 with errno
}

int Device::ensure_slot(Slot& s, uint64_t bytes, uint64_t nblk) {
  if (!s.copied) {
    CIR_HIP(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
    CIR_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  }
  const auto t0 = std::chrono::steady_clock::now();
  bool grew = false;
  if (bytes > s.cap) {
    grew = true;
    (void)hipHostFree(s.h_data);
    (void)hipFree(s.d_data);
    s.h_data = nullptr;
    s.d_data = nullptr;
    s.cap = 0;
    // (zero-copy staging -- the hash kernels reading the pinned buffer over
    // PCIe instead of an SDMA copy first -- ran config 5 at 30.0 vs 35.7
    // GiB/s and config 2 from host memory at 33.7 vs 51.5: profiles/r02/zero_copy/)
    CIR_HIP(hipHostMalloc(&s.h_data, bytes, hipHostMallocDefault));
    CIR_HIP(hipMalloc(&s.d_data, bytes));
    s.cap = bytes;
  }
  if (nblk > s.cap_blk) {
    (void)hipHostFree(s.h_off);
    (void)hipHostFree(s.h_len);
    (void)hipHostFree(s.h_out);
    (void)hipFree(s.d_off);
    (void)hipFree(s.d_len);
    (void)hipFree(s.d_out);
    s.h_off = nullptr;
    s.h_len = nullptr;
    s.h_out = nullptr;
    s.d_off = nullptr;
    s.d_len = nullptr;
    s.d_out = nullptr;
    s.cap_blk = 0;
    CIR_HIP(hipHostMalloc(&s.h_off, nblk * 8, hipHostMallocDefault));
    CIR_HIP(hipHostMalloc(&s.h_len, nblk * 4, hipHostMallocDefault));
    CIR_HIP(hipHostMalloc(&s.h_out, nblk * 32, hipHostMallocDefault));
    CIR_HIP(hipMalloc(&s.d_off, nblk * 8));
    CIR_HIP(hipMalloc(&s.d_len, nblk * 4));
    CIR_HIP(hipMalloc(&s.d_out, nblk * 32));
    s.cap_blk = nblk;
    grew = true;
  }
  if (grew && trace_enabled())
    fprintf(stderr, "cir alloc slot %d: %.1f MiB data, %llu blocks in %.2f ms\n",
            (int)(&s - slot), s.cap / 1048576.0, (unsigned long long)s.cap_blk,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
                .count());
  return CIR_OK;
}

int Device::ensure_timing(Slot& s) {
  for (hipEvent_t* e : {&s.t_copy0, &s.t_copy1, &s.t_hash0, &s.t_done})
    if (!*e) CIR_HIP(hipEventCreate(e));
  if (!t_ref) CIR_HIP(hipEventCreate(&t_ref));
  return CIR_OK;
}

// The two parts of an ordered batch: the quad part on a non-blocking stream
// of the greatest priority, the lane part on the caller's stream.  HIP pools
// hardware queues per priority, so the quad part never shares a queue with
// the caller's (or any other normal-priority) stream, and its workgroups are
// dispatched first.  Measured against the alternatives (round 2,
// profiles/r02/queue_probe_*.log: config 3 at 1 / 4 contexts per process):
// plain streams 866 / 616 GiB/s (the parts serialised whenever they shared a
// hardware queue), both parts on CU-masked streams 840 / 768, this 867 / 758
// (830 after the gate and the counting sort).
static hipError_t create_part_streams(Device& d) {
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e != hipSuccess) return e;
  return hipStreamCreateWithPriority(&d.qstream, hipStreamNonBlocking, greatest);
}

// The relay scratch (kernels.hpp RelayScratch), allocated at full capacity
// by cir_init: chain values, then the flags, zeroed once (each relay's
// finisher zeroes its groups' flags again).  Every relay runs on the
// quad-part stream, so relays of different callers never overlap on it.
// Caller holds d.order_mu with d's device current and the part streams
// created.
static int ensure_relay(Device& d) {
  if (d.relay_mem) return CIR_OK;
  CIR_HIP(hipMalloc(&d.relay_mem, dev::relay_scratch_bytes(dev::kRelayMaxGroups)));
  d.relay.state = (uint64_t*)d.relay_mem;
  d.relay.flags = (uint32_t*)((uint8_t*)d.relay_mem + (size_t)dev::kRelayMaxGroups * 1024u);
  d.relay.groups = dev::kRelayMaxGroups;
  // zeroed before any relay can run (once per device; the relays themselves
  // all run on the quad-part stream, in order)
  CIR_HIP(hipMemsetAsync(d.relay.flags, 0, (size_t)dev::kRelayMaxGroups * 4u,
                         d.qstream ? d.qstream : d.compute));
  CIR_HIP(hipStreamSynchronize(d.qstream ? d.qstream : d.compute));
  return CIR_OK;
}

// The part streams and their events, created by cir_init (caller holds
// d.order_mu with d's device current).
static int ensure_part_streams(Device& d, bool quad_stream) {
  if (d.order_free) return CIR_OK;
  if (quad_stream) CIR_HIP(create_part_streams(d));
  CIR_HIP(hipEventCreateWithFlags(&d.part_fork, hipEventDisableTiming));
  CIR_HIP(hipEventCreateWithFlags(&d.q_join, hipEventDisableTiming));
  CIR_HIP(hipEventCreateWithFlags(&d.order_free, hipEventDisableTiming));
  return CIR_OK;
}

// The context's state of the device `s` belongs to (NULL: the calling
// thread's current device), or null if the context does not hold it.
Device* stream_device(cir_ctx* ctx, hipStream_t s) {
  int id = 0;
  if ((s ? hipStreamGetDevice(s, &id) : hipGetDevice(&id)) != hipSuccess) return nullptr;
  for (auto& p : ctx->devs)
    if (p->id == id) return p.get();
  return nullptr;
}

// Descriptor batch, longest chain first: device sort (order.hip) into the
// device's ordering scratch, then the general kernel through the permutation.
bool valid_hash_type(int ht) { return ht == CIR_HASH_BLAKE2B_256 || ht == CIR_HASH_SHA512_256; }

int hash_desc_ordered(Device& d, const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                      uint64_t n, uint8_t* out, hipStream_t s, int ht, bool warm_only) {
  // Every batch is ordered (even a single chain: an index footer is one long
  // chain and runs in quad mode).
  if (n == 0) return CIR_OK;
  if (n > (uint64_t)INT32_MAX)  // 32-bit chain indices in the order (order.hip)
    return fail(CIR_EINVAL, "more than 2^31-1 descriptors in one ordered batch");
  std::lock_guard<std::mutex> lk(d.order_mu);
  // Streams, events and the ordering scratch live on d's device, whatever
  // the caller's current device is; the caller's device is restored on exit.
  DeviceGuard guard;
  CIR_HIP(hipSetDevice(d.id));
  const size_t need = dev::order_scratch_bytes(n);
  // the ordering scratch grows with the batch (the one allocation left on
  // this path: a batch larger than any before waits for the previous user)
  if (need > d.order_cap) {
    CIR_HIP(hipEventSynchronize(d.order_free));
    (void)hipFree(d.order_scratch);
    d.order_scratch = nullptr;
    d.order_cap = 0;
    CIR_HIP(hipMalloc(&d.order_scratch, need));
    d.order_cap = need;
  }
  // cir_init's warm-up: the scratch sized for n descriptors, one hashed
  if (warm_only) n = 1;
  CIR_HIP(hipStreamWaitEvent(s, d.order_free, 0));
  // diagnostics: a fresh event set per batch while timing is on (at most
  // kMaxTimedBatches per enable)
  constexpr size_t kMaxTimedBatches = 256;
  // (the set counts as recorded only once every event of it is: a batch that
  // fails part-way leaves it to the next batch)
  const hipEvent_t* tev = nullptr;
  if (d.timing && ht != CIR_HASH_SHA512_256 && d.tev_used < kMaxTimedBatches) {
    if (d.tev_used == d.tev.size()) {
      std::array<hipEvent_t, 6> set{};
      for (hipEvent_t& e : set) CIR_HIP(hipEventCreate(&e));
      d.tev.push_back(set);
    }
    tev = d.tev[d.tev_used].data();
    CIR_HIP(hipEventRecord(tev[0], s));
  }
  uint32_t* perm = nullptr;
  uint32_t* n_long = nullptr;
  CIR_HIP(dev::launch_order_desc(len, n, d.order_scratch, d.order_cap, &perm, &n_long, s));
  if (tev) CIR_HIP(hipEventRecord(tev[1], s));
  if (ht == CIR_HASH_SHA512_256)
    CIR_HIP(dev::launch_sha_desc(arena, off, len, perm, n, out, s));
  else
    CIR_HIP(dev::launch_mixed(arena, off, len, perm, n_long, n, out, s, d.qstream ? d.qstream : s,
                              d.part_fork, d.q_join,
                              d.relay_mem ? &d.relay : nullptr, tev ? tev + 2 : nullptr));
  CIR_HIP(hipEventRecord(d.order_free, s));
  if (tev) ++d.tev_used;
  return CIR_OK;
}

// Upload a packed slot and hash it.  chunk_bs == 0: descriptor batch
// (h_off/h_len, nblk blocks); otherwise the slot holds `bytes` consecutive
// bytes of one file split into chunk_bs blocks (nblk = ceil(bytes / bs)).
static int slot_submit_impl(Device& d, Slot& s, uint64_t bytes, uint64_t nblk,
                            uint64_t chunk_bs, int ht) {
  s.timed = d.record_times || trace_enabled();
  if (s.timed) {
    int rc = d.ensure_timing(s);
    if (rc) return rc;
    CIR_HIP(hipEventRecord(s.t_copy0, d.copy));
  }
  const uint8_t* src = s.d_data;
  CIR_HIP(hipMemcpyAsync(s.d_data, s.h_data, bytes, hipMemcpyHostToDevice, d.copy));
  if (chunk_bs == 0) {
    CIR_HIP(hipMemcpyAsync(s.d_off, s.h_off, nblk * 8, hipMemcpyHostToDevice, d.copy));
    CIR_HIP(hipMemcpyAsync(s.d_len, s.h_len, nblk * 4, hipMemcpyHostToDevice, d.copy));
  }
  if (s.timed) CIR_HIP(hipEventRecord(s.t_copy1, d.copy));
  CIR_HIP(hipEventRecord(s.copied, d.copy));
  CIR_HIP(hipStreamWaitEvent(d.compute, s.copied, 0));
  if (s.timed) CIR_HIP(hipEventRecord(s.t_hash0, d.compute));
  if (chunk_bs == 0) {
    int rc = hash_desc_ordered(d, src, s.d_off, s.d_len, nblk, s.d_out, d.compute, ht);
    if (rc) return rc;
  } else
    CIR_HIP(dev::launch_chunks(src, bytes, chunk_bs, s.d_out, d.compute));
  CIR_HIP(hipMemcpyAsync(s.h_out, s.d_out, nblk * 32, hipMemcpyDeviceToHost, d.compute));
  // t_done before done: slot_wait's synchronize on done then covers it
  if (s.timed) CIR_HIP(hipEventRecord(s.t_done, d.compute));
  CIR_HIP(hipEventRecord(s.done, d.compute));
  s.busy = true;
  return CIR_OK;
}

int slot_submit(Device& d, Slot& s, uint64_t bytes, uint64_t nblk, int ht) {
  return slot_submit_impl(d, s, bytes, nblk, 0, ht);
}

int slot_wait(Device& d, Slot& s) {
  (void)d;
  if (!s.busy) return CIR_OK;
  s.busy = false;
  CIR_HIP(hipEventSynchronize(s.done));
  return CIR_OK;
}

static int check_device(int id) {
  hipDeviceProp_t prop;
  CIR_HIP(hipGetDeviceProperties(&prop, id));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(CIR_ENODEV, std::string("device ") + std::to_string(id) + " is " +
                                prop.gcnArchName + ", this build targets gfx950 only");
  return CIR_OK;
}

// ---- host-memory batch: cir_hash_blocks --------------------------------

// Run piece(off, len) over [0, n) in 8 MiB pieces on host_copy_threads() host threads
// (a staging batch is 256 MiB: one copying thread moves ~10 GB/s, the
// upload takes ~55 GB/s).  Returns 0 or the first negative piece result;
// a piece must return len on success.
static int64_t parallel_pieces(uint64_t n, const std::function<int64_t(uint64_t, uint64_t)>& piece) {
  constexpr uint64_t kPiece = 8ull << 20;
  const uint64_t np = (n + kPiece - 1) / kPiece;
  const unsigned nt = (unsigned)std::min<uint64_t>(np, host_copy_threads());
  std::atomic<uint64_t> next{0};
  std::atomic<int64_t> err{0};
  auto work = [&] {
    for (uint64_t p; (p = next.fetch_add(1)) < np && err.load() == 0;) {
      const uint64_t off = p * kPiece, len = std::min(kPiece, n - off);
      const int64_t r = piece(off, len);
      if (r != (int64_t)len) {
        int64_t z = 0;
        err.compare_exchange_strong(z, r < 0 ? r : -(int64_t)EIO);
      }
    }
  };
  parallel_run(std::max(1u, nt), work);
  return err.load();
}

// fn(i0, i1) over [0, n) items in groups, on host_copy_threads() host threads when the
// batch moves at least 16 MiB (bytes); one thread otherwise.
static void parallel_items(size_t n, uint64_t bytes, const std::function<void(size_t, size_t)>& fn) {
  const unsigned nt = bytes < (16ull << 20) ? 1u : host_copy_threads();
  if (nt <= 1 || n < 2) {
    fn(0, n);
    return;
  }
  const size_t grain = std::max<size_t>(1, n / (8 * nt));
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (size_t i0; (i0 = next.fetch_add(grain)) < n;) fn(i0, std::min(n, i0 + grain));
  };
  parallel_run(nt, work);
}


// Hash blocks [b0, b1) of a host arena on device d, packing them 16-byte
// aligned into the two staging slots (pack slot k+1 while slot k hashes).
static int run_blocks(cir_ctx* ctx, Device& d, const uint8_t* arena, const uint64_t* off,
                      const uint32_t* len, size_t b0, size_t b1, uint8_t* out, int ht) {
  std::lock_guard<std::mutex> lk(d.mu);
  DeviceGuard guard;
  CIR_HIP(hipSetDevice(d.id));
  SlotDrain drain{d};  // an early return leaves no slot busy
  const uint64_t cap = ctx->staging;
  const uint64_t cap_blk = std::max<uint64_t>(cap / 512, 4096);
  const bool nt = stage_copy_nt();
  size_t next = b0;
  size_t pending_first[2] = {0, 0}, pending_n[2] = {0, 0};
  int k = 0;
  while (next < b1 || d.slot[0].busy || d.slot[1].busy) {
    Slot& s = d.slot[k];
    if (s.busy) {
      int rc = slot_wait(d, s);
      if (rc) return rc;
      memcpy(out + 32 * pending_first[k], s.h_out, 32 * pending_n[k]);
    }
    if (next < b1) {
      // size this batch
      uint64_t bytes = 0;
      size_t n = 0;
      while (next + n < b1 && n < cap_blk) {
        const uint64_t need = ((bytes + 15) & ~15ull) + len[next + n];
        if (n > 0 && need > cap) break;
        bytes = need;
        ++n;
      }
      int rc = d.ensure_slot(s, std::max<uint64_t>(std::max<uint64_t>(bytes, cap), 16),
                             std::max<uint64_t>(n, cap_blk));
      if (rc) return rc;
      uint64_t pos = 0;
      for (size_t i = 0; i < n; ++i) {
        pos = (pos + 15) & ~15ull;
        s.h_off[i] = pos;
        s.h_len[i] = len[next + i];
        pos += len[next + i];
      }
      // gather the blocks into the slot on several threads
      const size_t base = next;
      parallel_items(n, pos, [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i)
          copy_staged(s.h_data + s.h_off[i], arena + off[base + i], s.h_len[i], nt);
      });
      rc = slot_submit(d, s, std::max<uint64_t>(pos, 1), n, ht);
      if (rc) return rc;
      pending_first[k] = next;
      pending_n[k] = n;
      next += n;
    }
    k ^= 1;
  }
  return CIR_OK;
}

// Run fn(device, part) on every device of ctx in its own thread; return the
// first failure.
static int for_each_device(cir_ctx* ctx, const std::function<int(cir::Device&, size_t)>& fn) {
  const size_t nd = ctx->devs.size();
  if (nd == 1) return fn(*ctx->devs[0], 0);
  std::vector<int> rc(nd, 0);
  std::vector<std::string> err(nd);
  fan_out(nd, [&](size_t i) {
    rc[i] = fn(*ctx->devs[i], i);
    if (rc[i]) err[i] = t_last_error;
  });
  for (size_t i = 0; i < nd; ++i)
    if (rc[i]) return fail(rc[i], err[i]);
  return CIR_OK;
}

// ---- Hashes::hash_file over a byte source ------------------------------

// read(dst, n) must fill exactly n bytes or return < 0 (errno-style) / the
// short count at EOF.
using Reader = std::function<int64_t(uint8_t*, uint64_t)>;

// The digests of a host path, built in place in one malloc'd buffer that is
// handed to the caller as is (cir_free): sized once when the source's length
// is known, grown by realloc otherwise (a large block is remapped, not
// copied).  Round 4: a std::vector grown batch by batch, zero-filled, then
// copied into the returned buffer cost config 2 from host memory ~2 % (three
// extra passes over its 32 MB of digests).
struct HashBuf {
  uint8_t* p = nullptr;
  size_t len = 0, cap = 0;
  HashBuf() = default;
  HashBuf(const HashBuf&) = delete;
  HashBuf& operator=(const HashBuf&) = delete;
  ~HashBuf() { free(p); }
  bool reserve(size_t n) {
    if (n <= cap) return true;
    uint8_t* q = (uint8_t*)realloc(p, n);
    if (!q) return false;
    p = q;
    cap = n;
    return true;
  }
  // n more bytes at the end (contents undefined); null if out of memory
  uint8_t* extend(size_t n) {
    if (len + n > cap && !reserve(std::max(len + n, cap * 2))) return nullptr;
    uint8_t* at = p + len;
    len += n;
    return at;
  }
};

// size_hint: the source's length when known (a lower bound for a file that
// may grow), kSizeUnknown otherwise (a pipe); `exact`: the source ends there
// (memory, a known range).
constexpr uint64_t kSizeUnknown = ~0ull;
static int run_file_dev(cir_ctx* ctx, Device& d, const Reader& rd, uint64_t bs,
                        uint64_t* size_out, HashBuf& hashes, int ht,
                        uint64_t size_hint = kSizeUnknown, bool exact = false) {
  std::lock_guard<std::mutex> lk(d.mu);
  DeviceGuard guard;
  CIR_HIP(hipSetDevice(d.id));
  SlotDrain drain{d};  // an early return leaves no slot busy
  const uint64_t block_chunk = std::max<uint64_t>(bs, ctx->staging / bs * bs);
  uint64_t chunk = block_chunk;
  // A source shorter than one block is one short block: a slot of its own
  // size, not of the block size (a huge block size over a small input would
  // otherwise pin and allocate a block-sized slot).  A file whose size is
  // only a lower bound (it may grow while it is read) gets one byte of room
  // more: a slot that fills up means it grew, and the slot is regrown to
  // the block form with the bytes read so far.
  const bool hinted = size_hint != kSizeUnknown;
  if (!hinted) size_hint = 0;
  const bool one_short = (exact || hinted) && size_hint < bs;
  bool may_grow = one_short && !exact;
  if (one_short)
    chunk = std::max<uint64_t>(16, (std::min(bs, size_hint + (may_grow ? 1 : 0)) + 15) & ~15ull);
  uint64_t chunk_blk = one_short ? 1 : chunk / bs;
  // the first batches ramp up (1/8, 1/4, 1/2 of a slot, then whole slots),
  // as the scan's do: the first upload starts after a short fill
  auto first_fill = [&] {
    return scan_ramp() ? std::max<uint64_t>(bs, block_chunk / 8 / bs * bs) : block_chunk;
  };
  // (a file that may grow reads one byte past its size, never more than one
  // block: more bytes than that and it regrows below)
  uint64_t fill = !one_short ? first_fill() : may_grow ? size_hint + 1 : chunk;
  uint64_t total = 0;
  bool eof = false;
  size_t pending_at[2] = {0, 0}, pending_n[2] = {0, 0};
  int k = 0;
  hashes.len = 0;
  if (size_hint && !hashes.reserve(32 * ((size_hint + bs - 1) / bs)))
    return fail(CIR_ENOMEM, "digest buffer");
  while (!eof || d.slot[0].busy || d.slot[1].busy) {
    Slot& s = d.slot[k];
    if (s.busy) {
      int rc = slot_wait(d, s);
      if (rc) return rc;
      memcpy(hashes.p + 32 * pending_at[k], s.h_out, 32 * pending_n[k]);
    }
    if (!eof) {
      int rc = d.ensure_slot(s, chunk, chunk_blk);
      if (rc) return rc;
      uint64_t got = 0;
      uint64_t want = fill;
      fill = std::min(chunk, fill * 2);
      for (;;) {
        while (got < want) {
          const int64_t r = rd(s.h_data + got, want - got);
          if (r < 0) return fail(CIR_EIO, std::string("read: ") + strerror((int)-r));
          if (r == 0) {
            eof = true;
            break;
          }
          got += (uint64_t)r;
        }
        if (!may_grow || eof || got < want) break;
        // the file grew past its size at the start: the block form from here
        // (this slot regrown around the bytes already read)
        may_grow = false;
        std::unique_ptr<uint8_t[]> head(new (std::nothrow) uint8_t[got]);
        if (!head) return fail(CIR_ENOMEM, "read buffer");
        memcpy(head.get(), s.h_data, got);
        chunk = block_chunk;
        chunk_blk = chunk / bs;
        rc = d.ensure_slot(s, chunk, chunk_blk);
        if (rc) return rc;
        memcpy(s.h_data, head.get(), got);
        want = std::max(got, first_fill());
        fill = std::min(chunk, want * 2);
      }
      if (got > 0) {
        const uint64_t n = (got + bs - 1) / bs;
        pending_at[k] = hashes.len / 32;
        pending_n[k] = n;
        if (!hashes.extend(32 * n)) return fail(CIR_ENOMEM, "digest buffer");
        if (ht == CIR_HASH_BLAKE2B_256) {
          rc = slot_submit_impl(d, s, got, n, bs, ht);
        } else {  // descriptor form: one descriptor per block of the chunk
          for (uint64_t b = 0; b < n; ++b) {
            s.h_off[b] = b * bs;
            s.h_len[b] = (uint32_t)std::min<uint64_t>(bs, got - b * bs);
          }
          rc = slot_submit_impl(d, s, got, n, 0, ht);
        }
        if (rc) return rc;
        total += got;
      }
    }
    k ^= 1;
  }
  *size_out = total;
  return CIR_OK;
}

static int run_file(cir_ctx* ctx, const Reader& rd, uint64_t bs, uint64_t* size_out,
                    HashBuf& hashes, int ht, uint64_t size_hint = kSizeUnknown,
                    bool exact = false) {
  return run_file_dev(ctx, *ctx->devs[0], rd, bs, size_out, hashes, ht, size_hint, exact);
}

// read(dst, n, off): exactly n bytes at offset off (known to exist), or < 0.
using PosReader = std::function<int64_t(uint8_t*, uint64_t, uint64_t)>;

// A source of known size on a context with several devices: the blocks are
// split into one contiguous range per device (equal counts), each hashed by
// its own thread through that device's staging slots.
static int run_split(cir_ctx* ctx, const PosReader& prd, uint64_t total, uint64_t bs,
                     HashBuf& hashes, int ht) {
  const uint64_t nblk = (total + bs - 1) / bs;
  const size_t nd = std::min<size_t>(ctx->devs.size(), nblk);
  hashes.len = 0;
  if (!hashes.extend(32 * nblk)) return fail(CIR_ENOMEM, "digest buffer");
  std::vector<uint64_t> lo(nd), hi(nd);
  for (size_t i = 0; i < nd; ++i) {
    lo[i] = nblk * i / nd;
    hi[i] = nblk * (i + 1) / nd;
  }
  std::vector<int> rc(nd, 0);
  std::vector<std::string> err(nd);
  fan_out(nd, [&](size_t i) {
    const uint64_t beg = lo[i] * bs, end = std::min(hi[i] * bs, total);
    uint64_t pos = beg;
    Reader rd = [&](uint8_t* dst, uint64_t n) -> int64_t {
      const uint64_t k = std::min(n, end - pos);
      if (k == 0) return 0;
      const int64_t r = prd(dst, k, pos);
      if (r < 0) return r;
      pos += k;
      return (int64_t)k;
    };
    HashBuf h;
    uint64_t got = 0;
    rc[i] = run_file_dev(ctx, *ctx->devs[i], rd, bs, &got, h, ht, end - beg, /*exact=*/true);
    if (!rc[i] && h.len != 32 * (hi[i] - lo[i])) rc[i] = fail(CIR_EIO, "short range");
    if (rc[i])
      err[i] = t_last_error;
    else
      memcpy(hashes.p + 32 * lo[i], h.p, h.len);
  });
  for (size_t i = 0; i < nd; ++i)
    if (rc[i]) return fail(rc[i], err[i]);
  return CIR_OK;
}

// hand the digest buffer over (no copy); none for no digests
static int export_hashes(HashBuf& h, uint8_t** out, size_t* n) {
  *n = h.len / 32;
  *out = nullptr;
  if (h.len == 0) return CIR_OK;
  *out = h.p;
  h.p = nullptr;
  h.len = h.cap = 0;
  return CIR_OK;
}

// Everything a device state needs, created here rather than by the first
// call that uses it: the asynchronous *_dev entry points then never allocate
// or synchronise, and the first scan / host batch of a process runs as fast
// as the later ones (round 3: the staging slots' allocation and the first
// kernel launches were ~0.1 s of config 5's first scan).
//   * the staging, part and footer-chain streams, their events and the relay
//     scratch (zeroed with one synchronised memset);
//   * the three staging slots at the context's staging size (pinned host +
//     device buffers, descriptor and digest buffers for a full batch) -- or,
//     with `lazy` (CIR_STAGING_LAZY), two 64 KiB slots for the warm-up only,
//     grown by the first host-path call -- and the ordering scratch for one
//     full batch;
//   * one tiny chunk-form hash and one ordered descriptor batch on the
//     compute stream, which load the code object and touch every buffer;
//   * one small upload on the staging and on the footer-chain stream.
// Caller holds a DeviceGuard.
static int init_device(Device& d, uint64_t staging, bool lazy, bool one_shot) {
  // CIR_TRACE: each step's ms on stderr (the one-shot CLI's start-up budget)
  const bool tr = trace_enabled();
  auto t = std::chrono::steady_clock::now();
  auto step = [&](const char* what) {
    if (!tr) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "cir_init dev %d: %s %.2f ms\n", d.id, what,
            std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  };
  CIR_HIP(hipSetDevice(d.id));
  CIR_HIP(hipStreamCreateWithFlags(&d.compute, hipStreamNonBlocking));
  // one-shot: uploads share the compute stream, the footer-chain stream is
  // created by the first GPU-footer scan (scan.cpp), no quad-part stream
  if (one_shot)
    d.copy = d.compute;
  else {
    CIR_HIP(hipStreamCreateWithFlags(&d.copy, hipStreamNonBlocking));
    CIR_HIP(hipStreamCreateWithFlags(&d.chain, hipStreamNonBlocking));
  }
  CIR_HIP(hipMalloc(&d.chain_state, 16 * 8));
  for (int b = 0; b < 2; ++b)
    CIR_HIP(hipEventCreateWithFlags(&d.chain_done[b], hipEventDisableTiming));
  {
    std::lock_guard<std::mutex> lk(d.order_mu);
    int rc = ensure_part_streams(d, !one_shot);
    if (rc == CIR_OK) rc = ensure_relay(d);
    if (rc) return rc;
  }
  step("streams, events, relay scratch");
  const uint64_t cap_blk = std::max<uint64_t>(staging / 512, 4096);
  const uint64_t slot_bytes = lazy ? (64ull << 10) : std::max<uint64_t>(staging, 16);
  for (int k = 0; k < (one_shot ? 1 : lazy ? 2 : Device::kSlots); ++k) {
    const int rc = d.ensure_slot(d.slot[k], slot_bytes, lazy ? 4096 : cap_blk);
    if (rc) return rc;
  }
  step("staging slots");
  Slot& s = d.slot[0];
  CIR_HIP(hipMemsetAsync(s.d_data, 0, 4096, d.compute));
  CIR_HIP(hipMemsetAsync(s.d_off, 0, 8, d.compute));
  CIR_HIP(hipMemsetAsync(s.d_len, 0, 4, d.compute));
  CIR_HIP(dev::launch_chunks(s.d_data, 4096, 1024, s.d_out, d.compute));
  CIR_HIP(hipStreamSynchronize(d.compute));
  step("first kernel (code object load)");
  const int rc = hash_desc_ordered(d, s.d_data, s.d_off, s.d_len, cap_blk, s.d_out, d.compute,
                                   CIR_HASH_BLAKE2B_256, /*warm_only=*/true);
  if (rc) return rc;
  CIR_HIP(hipStreamSynchronize(d.compute));
  step("ordered descriptor batch");
  // the process's first host->device copy on a stream takes 7-11 ms more
  // than the next (profiles/r03_s2/cli/: a 10 MiB batch's upload 7.7-10.7 ms
  // in a fresh CLI process, ~0.2 ms later): pay it here for the staging and
  // footer-chain streams, with copies big enough to take the DMA engine path
  const size_t warm = (size_t)std::min<uint64_t>(slot_bytes, 4ull << 20);
  CIR_HIP(hipMemcpyAsync(s.d_data, s.h_data, warm, hipMemcpyHostToDevice, d.copy));
  if (d.chain)
    CIR_HIP(hipMemcpyAsync(d.slot[1].d_data, d.slot[1].h_data, warm, hipMemcpyHostToDevice,
                           d.chain));
  CIR_HIP(hipStreamSynchronize(d.copy));
  if (d.chain) CIR_HIP(hipStreamSynchronize(d.chain));
  step("first uploads");
  return CIR_OK;
}

// Open the given devices, one host thread each (a device's warm-up waits on
// its own streams only); the first failure in device order is returned.
static int init_devices(std::vector<std::unique_ptr<Device>>& devs, uint64_t staging, bool lazy,
                        bool one_shot) {
  if (devs.size() == 1) {
    DeviceGuard guard;
    return init_device(*devs[0], staging, lazy, one_shot);
  }
  std::vector<int> rc(devs.size(), 0);
  std::vector<std::string> err(devs.size());
  fan_out(devs.size(), [&](size_t i) {
    rc[i] = init_device(*devs[i], staging, lazy, one_shot);
    if (rc[i]) err[i] = t_last_error;
  });
  for (size_t i = 0; i < devs.size(); ++i)
    if (rc[i]) return fail(rc[i], err[i]);
  return CIR_OK;
}

// Process-default context for cir_blake2b256 (BlockHash::hash_bytes has no
// context argument in the reference).
static std::once_flag g_default_once;
static cir_ctx* g_default = nullptr;
static int g_default_rc = 0;
static std::string g_default_err;

static int default_ctx(cir_ctx** out) {
  std::call_once(g_default_once, [] {
    g_default_rc = cir_init(&g_default, 1u, 16u << 20);
    if (g_default_rc) g_default_err = t_last_error;
  });
  if (g_default_rc) return fail(g_default_rc, g_default_err);
  *out = g_default;
  return CIR_OK;
}

}  // namespace cir

using namespace cir;

extern "C" {

int cir_device_count(void) try {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
} CIR_CATCH_BOUNDARY

uint32_t cir_devices_for_bytes(uint64_t work_bytes, uint64_t staging_bytes, uint32_t visible) {
  if (visible == 0) return 0;
  if (work_bytes == 0) return visible;
  const uint64_t slot =
      staging_bytes && staging_bytes != CIR_STAGING_LAZY ? staging_bytes : (256ull << 20);
  // a device is worth opening for at least two staging batches of the input
  const uint64_t per = slot > UINT64_MAX / 2 ? UINT64_MAX : 2 * slot;
  const uint64_t n = work_bytes / per + (work_bytes % per != 0);
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n, visible));
}

int cir_init(cir_ctx** out, uint32_t device_mask, uint64_t staging_bytes) try {
  return cir_init_n(out, device_mask, staging_bytes, 0, 0);
} CIR_CATCH_BOUNDARY

int cir_init_n(cir_ctx** out, uint32_t device_mask, uint64_t staging_bytes,
               uint32_t max_devices, uint32_t flags) try {
  if (!out) return fail(CIR_EINVAL, "cir_init: null ctx");
  *out = nullptr;
  if (flags & ~CIR_INIT_ONE_SHOT) return fail(CIR_EINVAL, "cir_init_n: unknown flags");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return fail(CIR_ENODEV, std::string("no HIP device: ") + hipGetErrorString(e));
  DeviceGuard guard;
  auto ctx = std::make_unique<cir_ctx>();
  const bool lazy = staging_bytes == CIR_STAGING_LAZY;
  ctx->staging = staging_bytes && !lazy ? staging_bytes : (256ull << 20);
  for (int i = 0; i < n && i < 32; ++i) {
    if (device_mask && !(device_mask & (1u << i))) continue;
    int rc = check_device(i);
    if (rc) return rc;
    auto d = std::make_unique<Device>();
    d->id = i;
    ctx->devs.push_back(std::move(d));
  }
  if (ctx->devs.empty()) return fail(CIR_ENODEV, "device_mask selects no visible device");
  // CIR_DEBUG_SPLIT=k (tests): every selected GPU appears k times, as k
  // independent device states (own streams, staging slots, scratch), so the
  // multi-device splits of the host paths run on a one-GPU box.
  if (const char* v = std::getenv("CIR_DEBUG_SPLIT")) {
    const int k = std::atoi(v);
    const size_t n0 = ctx->devs.size();
    for (int r = 1; r < k && r < 8; ++r)
      for (size_t i = 0; i < n0; ++i) {
        auto d = std::make_unique<Device>();
        d->id = ctx->devs[i]->id;
        ctx->devs.push_back(std::move(d));
      }
  }
  // the device-count hint: the first max_devices device states (distinct
  // GPUs first, CIR_DEBUG_SPLIT's extra states after them)
  if (max_devices && ctx->devs.size() > max_devices) ctx->devs.resize(max_devices);
  int rc = init_devices(ctx->devs, ctx->staging, lazy, (flags & CIR_INIT_ONE_SHOT) != 0);
  if (rc) return rc;
  if (const char* v = std::getenv("CIR_FOOTER"))
    ctx->footer = strcmp(v, "gpu") == 0 ? CIR_FOOTER_GPU : CIR_FOOTER_HOST;
  *out = ctx.release();
  return CIR_OK;
} CIR_CATCH_BOUNDARY

void cir_destroy(cir_ctx* ctx) { delete ctx; }

int cir_ctx_devices(const cir_ctx* ctx, int* ids, int max_ids) try {
  if (!ctx) return fail(CIR_EINVAL, "null ctx");
  int n = (int)ctx->devs.size();
  for (int i = 0; i < n && i < max_ids; ++i) ids[i] = ctx->devs[i]->id;
  return n;
} CIR_CATCH_BOUNDARY

const char* cir_strerror(int status) {
  switch (status) {
    case CIR_OK: return "ok";
    case CIR_EIO: return "i/o error";
    case CIR_EINVAL: return "invalid argument";
    case CIR_EHIP: return "HIP runtime error";
    case CIR_ENOMEM: return "out of memory";
    case CIR_EPARSE: return "error parsing index";
    case CIR_ENOTFOUND: return "not found";
    case CIR_EHASHSIZE: return "hash size is unsupported";
    case CIR_ENODEV: return "no usable gfx950 device";
    case CIR_EUNSUPPORTED: return "unsupported hash type";
    case CIR_EAGAIN: return "try again";
    default: return "unknown error";
  }
}

const char* cir_last_error(void) { return t_last_error.c_str(); }

void cir_free(void* p) { free(p); }

int cir_hash_chunks_dev(cir_ctx* ctx, const void* d_data, uint64_t nbytes, uint64_t block_size,
                        uint8_t* d_out, void* stream) try {
  if (block_size == 0) return fail(CIR_EINVAL, "block_size must be > 0");
  if (nbytes && (!d_data || !d_out)) return fail(CIR_EINVAL, "null device pointer");
  if (reinterpret_cast<uintptr_t>(d_out) & 15u)
    return fail(CIR_EINVAL, "d_out must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  // with a context, the ragged rest of a large file runs in quad mode on the
  // device's quad-part stream beside the uniform part (launch_chunks_split)
  Device* d = ctx ? stream_device(ctx, s) : nullptr;
  if (d && nbytes) {
    // (the part streams and the relay scratch exist since cir_init: nothing
    // here allocates or synchronises)
    std::lock_guard<std::mutex> lk(d->order_mu);
    DeviceGuard guard;
    CIR_HIP(hipSetDevice(d->id));
    CIR_HIP(dev::launch_chunks_split((const uint8_t*)d_data, nbytes, block_size, d_out, s,
                                     d->qstream, d->part_fork, d->q_join, &d->relay));
    return CIR_OK;
  }
  CIR_HIP(dev::launch_chunks((const uint8_t*)d_data, nbytes, block_size, d_out, s));
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_hash_blocks_dev_ht(cir_ctx* ctx, int hash_type, const void* d_arena,
                           const uint64_t* d_off, const uint32_t* d_len, size_t nblk,
                           uint8_t* d_out, void* stream) try {
  if (!valid_hash_type(hash_type)) return fail(CIR_EINVAL, "unknown hash type");
  if (nblk && (!d_arena || !d_off || !d_len || !d_out))
    return fail(CIR_EINVAL, "null device pointer");
  if (reinterpret_cast<uintptr_t>(d_out) & 15u)
    return fail(CIR_EINVAL, "d_out must be 16-byte aligned");
  // descriptor indices are 32-bit in the kernels and in the ordering's
  // permutation: one call takes at most 2^31-1 blocks
  if (nblk > (size_t)INT32_MAX) return fail(CIR_EINVAL, "more than 2^31-1 descriptors");
  hipStream_t s = (hipStream_t)stream;
  // Context-less calls hash in descriptor order, one lane per chain; with a
  // context the batch is ordered longest chain first on the device
  // (order.hip) and long BLAKE2b chains run in quad mode.
  if (ctx) {
    Device* d = stream_device(ctx, s);
    if (!d) return fail(CIR_EINVAL, "stream device is not part of the context");
    return hash_desc_ordered(*d, (const uint8_t*)d_arena, d_off, d_len, nblk, d_out, s, hash_type);
  }
  if (hash_type == CIR_HASH_SHA512_256)
    CIR_HIP(dev::launch_sha_desc((const uint8_t*)d_arena, d_off, d_len, nullptr, nblk, d_out, s));
  else
    CIR_HIP(dev::launch_general_desc((const uint8_t*)d_arena, d_off, d_len, nullptr, nblk, d_out, s));
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_hash_blocks_dev(cir_ctx* ctx, const void* d_arena, const uint64_t* d_off,
                        const uint32_t* d_len, size_t nblk, uint8_t* d_out, void* stream) try {
  return cir_hash_blocks_dev_ht(ctx, CIR_HASH_BLAKE2B_256, d_arena, d_off, d_len, nblk, d_out,
                                stream);
} CIR_CATCH_BOUNDARY

// Untrusted descriptors (cir_hash_blocks_dev_bounded, cir_verify_blocks_dev_
// bounded): the bounds pass (order.hip k_desc_bound) writes checked lengths
// and flags into scratch, the batch is hashed over the checked lengths as
// cir_hash_blocks_dev_ht would hash it, and then the flagged blocks' digests
// are zeroed (and failed in the compare when verifying: expected != NULL).
// Scratch: the device's bound scratch with a context, else a stream-ordered
// allocation freed behind the batch.  Nothing synchronises the stream.
static int bounded_run(cir_ctx* ctx, Device* d, int ht, const uint8_t* arena,
                       uint64_t arena_bytes, const uint64_t* off, const uint32_t* len, size_t n,
                       uint8_t* out, uint32_t* nrange, const uint8_t* expected, uint8_t* ok,
                       uint32_t* nbad, void* scratch, hipStream_t s) {
  uint32_t* slen = nullptr;
  uint8_t* flag = nullptr;
  CIR_HIP(dev::launch_desc_bound(off, len, n, arena_bytes, scratch, nrange, &slen, &flag, s));
  if (ctx) {
    int rc = hash_desc_ordered(*d, arena, off, slen, n, out, s, ht);
    if (rc) return rc;
  } else if (ht == CIR_HASH_SHA512_256) {
    CIR_HIP(dev::launch_sha_desc(arena, off, slen, nullptr, n, out, s));
  } else {
    CIR_HIP(dev::launch_general_desc(arena, off, slen, nullptr, n, out, s));
  }
  CIR_HIP(dev::launch_desc_zero(flag, n, out, s));
  if (expected) CIR_HIP(dev::launch_verify(out, expected, n, ok, nbad, s, flag));
  return CIR_OK;
}

static int hash_desc_bounded(cir_ctx* ctx, int ht, const void* d_arena, uint64_t arena_bytes,
                             const uint64_t* d_off, const uint32_t* d_len, size_t n,
                             uint8_t* d_out, uint32_t* d_nrange, const uint8_t* d_expected,
                             uint8_t* d_ok, uint32_t* d_nbad, hipStream_t s) {
  if (!valid_hash_type(ht)) return fail(CIR_EINVAL, "unknown hash type");
  if (n && (!d_off || !d_len || !d_out)) return fail(CIR_EINVAL, "null device pointer");
  // (d_arena may be NULL with arena_bytes == 0: every non-empty block is then
  // out of range, and a zero-length one at offset 0 hashes as the empty input)
  if (n && !d_arena && arena_bytes) return fail(CIR_EINVAL, "null arena with arena_bytes > 0");
  if (reinterpret_cast<uintptr_t>(d_out) & 15u)
    return fail(CIR_EINVAL, "digest arrays must be 16-byte aligned");
  if (n > (size_t)INT32_MAX) return fail(CIR_EINVAL, "more than 2^31-1 descriptors");
  Device* d = nullptr;
  if (ctx) {
    d = stream_device(ctx, s);
    if (!d) return fail(CIR_EINVAL, "stream device is not part of the context");
  }
  if (d_nbad) CIR_HIP(hipMemsetAsync(d_nbad, 0, 4, s));
  if (n == 0) {
    if (d_nrange) CIR_HIP(hipMemsetAsync(d_nrange, 0, 4, s));
    return CIR_OK;
  }
  const uint8_t* arena = static_cast<const uint8_t*>(d_arena);
  const size_t need = dev::bound_scratch_bytes(n);
  if (!d) {
    void* scratch = nullptr;
    CIR_HIP(hipMallocAsync(&scratch, need, s));
    const int rc = bounded_run(ctx, d, ht, arena, arena_bytes, d_off, d_len, n, d_out, d_nrange,
                               d_expected, d_ok, d_nbad, scratch, s);
    const hipError_t e = hipFreeAsync(scratch, s);
    if (rc) return rc;
    CIR_HIP(e);
    return CIR_OK;
  }
  std::lock_guard<std::mutex> lk(d->bound_mu);
  DeviceGuard guard;
  CIR_HIP(hipSetDevice(d->id));
  if (!d->bound_free) CIR_HIP(hipEventCreateWithFlags(&d->bound_free, hipEventDisableTiming));
  if (need > d->bound_cap) {
    // grows with the batch: a larger batch than any before waits for the
    // previous user of the scratch
    CIR_HIP(hipEventSynchronize(d->bound_free));
    (void)hipFree(d->bound_scratch);
    d->bound_scratch = nullptr;
    d->bound_cap = 0;
    CIR_HIP(hipMalloc(&d->bound_scratch, need));
    d->bound_cap = need;
  }
  CIR_HIP(hipStreamWaitEvent(s, d->bound_free, 0));
  const int rc = bounded_run(ctx, d, ht, arena, arena_bytes, d_off, d_len, n, d_out, d_nrange,
                             d_expected, d_ok, d_nbad, d->bound_scratch, s);
  // recorded on every path: whatever of the batch was queued is ordered
  // before the scratch's next user
  const hipError_t e = hipEventRecord(d->bound_free, s);
  if (rc) return rc;
  CIR_HIP(e);
  return CIR_OK;
}

int cir_hash_blocks_dev_bounded(cir_ctx* ctx, int hash_type, const void* d_arena,
                                uint64_t arena_bytes, const uint64_t* d_off, const uint32_t* d_len,
                                size_t nblk, uint8_t* d_out, uint32_t* d_nrange,
                                void* stream) try {
  return hash_desc_bounded(ctx, hash_type, d_arena, arena_bytes, d_off, d_len, nblk, d_out,
                           d_nrange, nullptr, nullptr, nullptr, (hipStream_t)stream);
} CIR_CATCH_BOUNDARY

int cir_verify_blocks_dev_bounded(cir_ctx* ctx, int hash_type, const void* d_arena,
                                  uint64_t arena_bytes, const uint64_t* d_off,
                                  const uint32_t* d_len, size_t nblk, const uint8_t* d_expected,
                                  uint8_t* d_digests, uint8_t* d_ok, uint32_t* d_nbad,
                                  void* stream) try {
  if (nblk && (!d_expected || !d_digests)) return fail(CIR_EINVAL, "null device pointer");
  if ((reinterpret_cast<uintptr_t>(d_expected) | reinterpret_cast<uintptr_t>(d_digests)) & 15u)
    return fail(CIR_EINVAL, "digest arrays must be 16-byte aligned");
  // (nblk == 0: *d_nbad = 0 and nothing else happens)
  return hash_desc_bounded(ctx, hash_type, d_arena, arena_bytes, d_off, d_len, nblk, d_digests,
                           nullptr, d_expected, d_ok, d_nbad, (hipStream_t)stream);
} CIR_CATCH_BOUNDARY

int cir_hash_blocks_ht(cir_ctx* ctx, int hash_type, const uint8_t* h_arena, const uint64_t* off,
                       const uint32_t* len, size_t nblk, uint8_t* h_out) try {
  if (!ctx) return fail(CIR_EINVAL, "null ctx");
  if (!valid_hash_type(hash_type)) return fail(CIR_EINVAL, "unknown hash type");
  if (nblk == 0) return CIR_OK;
  if (!h_arena || !off || !len || !h_out) return fail(CIR_EINVAL, "null pointer");
  // contiguous ranges balanced by bytes
  const size_t nd = std::min(ctx->devs.size(), nblk);
  uint64_t total = 0;
  for (size_t i = 0; i < nblk; ++i) total += (uint64_t)len[i] + 128;
  std::vector<size_t> cut(nd + 1, nblk);
  cut[0] = 0;
  uint64_t acc = 0;
  size_t p = 1;
  for (size_t i = 0; i < nblk && p < nd; ++i) {
    acc += (uint64_t)len[i] + 128;
    if (acc * nd >= total * p) cut[p++] = i + 1;
  }
  return for_each_device(ctx, [&](Device& d, size_t i) {
    if (i >= nd || cut[i] >= cut[i + 1]) return (int)CIR_OK;
    return run_blocks(ctx, d, h_arena, off, len, cut[i], cut[i + 1], h_out, hash_type);
  });
} CIR_CATCH_BOUNDARY

int cir_hash_blocks(cir_ctx* ctx, const uint8_t* h_arena, const uint64_t* off,
                    const uint32_t* len, size_t nblk, uint8_t* h_out) try {
  return cir_hash_blocks_ht(ctx, CIR_HASH_BLAKE2B_256, h_arena, off, len, nblk, h_out);
} CIR_CATCH_BOUNDARY

// Inputs up to this size take the one-launch path (k_single): the chain of
// a larger input runs for milliseconds, so the staged path's fixed cost no
// longer matters there.
constexpr size_t kSingleMax = 16ull << 20;
// Up to this size the kernel reads the pinned input itself (one launch).
constexpr size_t kSinglePull = 64ull << 10;

// The single-launch input buffers (pinned device-mapped host + device
// twin) with room for `need` bytes.  Caller holds d.single_mu with d current.
static int ensure_single_buffers(Device& d, size_t need) {
  // each resource is checked on its own, so a failure part-way leaves the
  // rest to be created by the next call (never a launch with a null output)
  if (!d.single) CIR_HIP(hipStreamCreateWithFlags(&d.single, hipStreamNonBlocking));
  if (!d.single_out)
    CIR_HIP(hipHostMalloc(&d.single_out, 64, hipHostMallocMapped | hipHostMallocCoherent));
  if (need > d.single_cap) {
    (void)hipHostFree(d.single_h);
    (void)hipFree(d.single_d);
    d.single_h = nullptr;
    d.single_d = nullptr;
    d.single_cap = 0;
    const size_t cap = std::max<size_t>(need, 64u << 10);
    CIR_HIP(hipHostMalloc(&d.single_h, cap, hipHostMallocMapped | hipHostMallocCoherent));
    const hipError_t e = hipMalloc(&d.single_d, cap);
    if (e != hipSuccess) {
      (void)hipHostFree(d.single_h);
      d.single_h = nullptr;
      return hip_fail(e, "hipMalloc(single_d)");
    }
    d.single_cap = cap;
  }
  return CIR_OK;
}

// BlockHash::hash_bytes in one kernel launch: copy into a pinned buffer the
// GPU reads over PCIe, launch, wait, read the digest the kernel wrote into
// mapped host memory.  Caller holds d.single_mu.
static int single_launch(Device& d, const uint8_t* p, size_t n, uint8_t* out) {
  DeviceGuard guard;
  CIR_HIP(hipSetDevice(d.id));
  const size_t need = (n + 15) & ~(size_t)15;
  int rc = ensure_single_buffers(d, need);
  if (rc) return rc;
  if (n) memcpy(d.single_h, p, n);
  // pinned host memory is device-accessible at its host address (unified
  // virtual addressing on ROCm).  Small inputs are pulled over PCIe by the
  // kernel itself (no copy launch); larger ones go up by one SDMA copy first.
  const uint8_t* src = d.single_h;
  if (n > kSinglePull) {
    CIR_HIP(hipMemcpyAsync(d.single_d, d.single_h, need, hipMemcpyHostToDevice, d.single));
    src = d.single_d;
  }
  CIR_HIP(dev::launch_single(src, (uint32_t)n, d.single_d, d.single_out, d.single));
  CIR_HIP(hipStreamSynchronize(d.single));
  memcpy(out, d.single_out, 32);
  return CIR_OK;
}

// Concurrent callers of cir_blake2b256 on one device, coalesced: one caller
// at a time leads -- takes every request queued so far and hashes them as one
// descriptor batch (a lone request goes through single_launch) -- while the
// others wait for their digest or for the lead.  One chain's latency then
// serves every caller that arrived meanwhile instead of one each.
struct SingleReq {
  const uint8_t* p;
  size_t n;
  uint8_t* out;
  int rc = CIR_OK;
  std::string err;
  bool done = false;
};

struct SingleQueue {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<SingleReq*> pending;
  bool leading = false;
};

// A batch of requests (total input <= kSingleBatchBytes) as descriptors on
// the single stream.  Caller holds d.single_mu.
static int single_batch(Device& d, const std::vector<SingleReq*>& reqs) {
  DeviceGuard guard;
  CIR_HIP(hipSetDevice(d.id));
  size_t need = 0;
  for (const SingleReq* r : reqs) need += (r->n + 15) & ~(size_t)15;
  int rc = ensure_single_buffers(d, std::max<size_t>(need, 16));
  if (rc) return rc;
  const size_t m = reqs.size();
  if (m > d.single_batch_cap) {
    (void)hipHostFree(d.single_desc_h);
    (void)hipFree(d.single_desc_d);
    d.single_desc_h = nullptr;
    d.single_desc_d = nullptr;
    d.single_batch_cap = 0;
    const size_t cap = std::max<size_t>(m, 256);
    CIR_HIP(hipHostMalloc(&d.single_desc_h, cap * 48, hipHostMallocDefault));
    const hipError_t e = hipMalloc(&d.single_desc_d, cap * 48);
    if (e != hipSuccess) {
      (void)hipHostFree(d.single_desc_h);
      d.single_desc_h = nullptr;
      return hip_fail(e, "hipMalloc(single_desc_d)");
    }
    d.single_batch_cap = cap;
  }
  // layout of both desc buffers: off[cap] (u64), len[cap] (u32), digests[cap]
  const size_t cap = d.single_batch_cap;
  uint64_t* h_off = (uint64_t*)d.single_desc_h;
  uint32_t* h_len = (uint32_t*)(d.single_desc_h + 8 * cap);
  uint8_t* h_out = d.single_desc_h + 16 * cap;
  uint64_t pos = 0;
  for (size_t i = 0; i < m; ++i) {
    h_off[i] = pos;
    h_len[i] = (uint32_t)reqs[i]->n;
    if (reqs[i]->n) memcpy(d.single_h + pos, reqs[i]->p, reqs[i]->n);
    pos += (reqs[i]->n + 15) & ~(size_t)15;
  }
  uint64_t* d_off = (uint64_t*)d.single_desc_d;
  uint32_t* d_len = (uint32_t*)(d.single_desc_d + 8 * cap);
  uint8_t* d_out = d.single_desc_d + 16 * cap;
  CIR_HIP(hipMemcpyAsync(d.single_d, d.single_h, std::max<uint64_t>(pos, 16),
                         hipMemcpyHostToDevice, d.single));
  CIR_HIP(hipMemcpyAsync(d_off, h_off, 8 * m, hipMemcpyHostToDevice, d.single));
  CIR_HIP(hipMemcpyAsync(d_len, h_len, 4 * m, hipMemcpyHostToDevice, d.single));
  rc = hash_desc_ordered(d, d.single_d, d_off, d_len, m, d_out, d.single, CIR_HASH_BLAKE2B_256);
  if (rc) return rc;
  CIR_HIP(hipMemcpyAsync(h_out, d_out, 32 * m, hipMemcpyDeviceToHost, d.single));
  CIR_HIP(hipStreamSynchronize(d.single));
  for (size_t i = 0; i < m; ++i) memcpy(reqs[i]->out, h_out + 32 * i, 32);
  return CIR_OK;
}

// Limits of one coalesced batch.
constexpr size_t kSingleBatchBytes = 64ull << 20;
constexpr size_t kSingleBatchMax = 4096;

static int single_coalesced(Device& d, SingleQueue& q, const uint8_t* p, size_t n, uint8_t* out) {
  SingleReq me;
  me.p = p;
  me.n = n;
  me.out = out;
  std::unique_lock<std::mutex> lk(q.mu);
  q.pending.push_back(&me);
  while (!me.done) {
    if (q.leading) {
      q.cv.wait(lk);
      continue;
    }
    // lead: take what is queued (first come first), up to the batch limits
    q.leading = true;
    std::vector<SingleReq*> batch;
    size_t bytes = 0, k = 0;
    for (; k < q.pending.size() && batch.size() < kSingleBatchMax; ++k) {
      SingleReq* r = q.pending[k];
      if (!batch.empty() && bytes + r->n > kSingleBatchBytes) break;
      bytes += r->n;
      batch.push_back(r);
    }
    q.pending.erase(q.pending.begin(), q.pending.begin() + (std::ptrdiff_t)k);
    lk.unlock();
    int rc;
    {
      std::lock_guard<std::mutex> sl(d.single_mu);
      rc = batch.size() == 1 ? single_launch(d, batch[0]->p, batch[0]->n, batch[0]->out)
                             : single_batch(d, batch);
    }
    const std::string err = rc ? t_last_error : std::string();
    lk.lock();
    for (SingleReq* r : batch) {
      r->rc = rc;
      r->err = err;
      r->done = true;
    }
    q.leading = false;
    q.cv.notify_all();
  }
  lk.unlock();
  if (me.rc) return fail(me.rc, me.err);
  return CIR_OK;
}

static int single_shot(int ht, const uint8_t* p, size_t n, uint8_t* out) {
  if (!out || (n && !p)) return fail(CIR_EINVAL, "null pointer");
  if (n > 0xffffffffull) return fail(CIR_EINVAL, "block longer than 4 GiB");
  cir_ctx* ctx = nullptr;
  int rc = default_ctx(&ctx);
  if (rc) return rc;
  if (ht == CIR_HASH_BLAKE2B_256 && n <= kSingleMax) {
    static SingleQueue q;  // the process-default context's first device
    return single_coalesced(*ctx->devs[0], q, p, n, out);
  }
  static const uint8_t empty = 0;
  const uint64_t off = 0;
  const uint32_t len = (uint32_t)n;
  return cir_hash_blocks_ht(ctx, ht, n ? p : &empty, &off, &len, 1, out);
}

int cir_blake2b256(const uint8_t* p, size_t n, uint8_t out[CIR_DIGEST_BYTES]) try {
  return single_shot(CIR_HASH_BLAKE2B_256, p, n, out);
} CIR_CATCH_BOUNDARY

int cir_sha512_256(const uint8_t* p, size_t n, uint8_t out[CIR_DIGEST_BYTES]) try {
  return single_shot(CIR_HASH_SHA512_256, p, n, out);
} CIR_CATCH_BOUNDARY

int cir_hash_file_ht(cir_ctx* ctx, int hash_type, int fd, uint64_t block_size,
                     uint64_t* size_out, uint8_t** hashes_out, size_t* nhash_out) try {
  if (!ctx || !size_out || !hashes_out || !nhash_out) return fail(CIR_EINVAL, "null pointer");
  if (block_size == 0 || block_size > 0xffffffffull)
    return fail(CIR_EINVAL, "block_size must be in 1 .. 2^32-1");
  if (!valid_hash_type(hash_type)) return fail(CIR_EINVAL, "unknown hash type");
  HashBuf h;
  const bool nt = stage_copy_nt();
  // Regular files: the bytes known to exist (st_size at the start) are read
  // with pread() by several threads per batch, then the read position moves
  // past them; beyond that (growth, pipes, sockets) plain read() to EOF,
  // as Hashes::hash_file's Read loop does.
  struct stat st;
  const off_t pos0 = ::lseek(fd, 0, SEEK_CUR);
  uint64_t known = 0, done = 0;
  const bool regular = pos0 >= 0 && ::fstat(fd, &st) == 0 && S_ISREG(st.st_mode);
  if (regular && st.st_size > pos0) known = (uint64_t)(st.st_size - pos0);
  // CIR_DEBUG_GROW=k (tests): take the file to be k bytes shorter than
  // fstat says, as if it grew by k between the fstat and the reads
  if (const char* v = std::getenv("CIR_DEBUG_GROW"))
    known -= std::min<uint64_t>(known, strtoull(v, nullptr, 10));
  if (known > 0 && ctx->devs.size() > 1 && known > block_size) {
    // several devices: split the known bytes, then make sure nothing follows
    // (a file growing meanwhile is re-hashed on one device, to its end)
    PosReader prd = [fd, pos0, nt](uint8_t* dst, uint64_t n, uint64_t off) -> int64_t {
      const int64_t e = parallel_pieces(n, [&](uint64_t o, uint64_t len) -> int64_t {
        uint64_t got = 0;
        while (got < len) {
          const ssize_t r = pread_staged(fd, dst + o + got, len - got,
                                         pos0 + (off_t)(off + o + got), nt);
          if (r < 0 && errno == EINTR) continue;
          if (r <= 0) return r < 0 ? -(int64_t)errno : (int64_t)got;
          got += (uint64_t)r;
        }
        return (int64_t)got;
      });
      return e < 0 ? e : (int64_t)n;
    };
    int rc = run_split(ctx, prd, known, block_size, h, hash_type);
    if (rc) return rc;
    uint8_t probe;
    ssize_t more;
    do more = ::pread(fd, &probe, 1, pos0 + (off_t)known);
    while (more < 0 && errno == EINTR);
    if (more == 0) {
      if (::lseek(fd, pos0 + (off_t)known, SEEK_SET) < 0)
        return fail(CIR_EIO, std::string("lseek: ") + strerror(errno));
      *size_out = known;
      return export_hashes(h, hashes_out, nhash_out);
    }
    known = 0;  // changed while hashed: fall through to the one-device read
  }
  Reader rd = [fd, pos0, nt, &known, &done](uint8_t* dst, uint64_t n) -> int64_t {
    if (done < known) {
      const uint64_t k = std::min(n, known - done);
      const uint64_t base = (uint64_t)pos0 + done;
      const int64_t e = parallel_pieces(k, [&](uint64_t off, uint64_t len) -> int64_t {
        uint64_t got = 0;
        while (got < len) {
          const ssize_t r = pread_staged(fd, dst + off + got, len - got,
                                         (off_t)(base + off + got), nt);
          if (r < 0 && errno == EINTR) continue;
          if (r < 0) return -(int64_t)errno;
          if (r == 0) break;  // truncated meanwhile
          got += (uint64_t)r;
        }
        return (int64_t)got;
      });
      if (e < 0 && e != -(int64_t)EIO) return e;
      if (e == 0) {
        done += k;
        if (::lseek(fd, (off_t)(base + k), SEEK_SET) < 0) return -(int64_t)errno;
        return (int64_t)k;
      }
      // shrank while hashing: fall back to sequential reads from here
      known = done;
      if (::lseek(fd, (off_t)base, SEEK_SET) < 0) return -(int64_t)errno;
    }
    for (;;) {
      ssize_t r = ::read(fd, dst, n);
      if (r < 0 && errno == EINTR) continue;
      return r < 0 ? -(int64_t)errno : (int64_t)r;
    }
  };
  // (a regular file's size at the fstat is a lower bound: an empty one
  // gets a 16-byte slot, not a block-sized one)
  int rc = run_file(ctx, rd, block_size, size_out, h, hash_type, regular ? known : kSizeUnknown);
  if (rc) return rc;
  return export_hashes(h, hashes_out, nhash_out);
} CIR_CATCH_BOUNDARY

int cir_hash_file(cir_ctx* ctx, int fd, uint64_t block_size, uint64_t* size_out,
                  uint8_t** hashes_out, size_t* nhash_out) try {
  return cir_hash_file_ht(ctx, CIR_HASH_BLAKE2B_256, fd, block_size, size_out, hashes_out,
                          nhash_out);
} CIR_CATCH_BOUNDARY

int cir_hash_memory_ht(cir_ctx* ctx, int hash_type, const uint8_t* data, uint64_t size,
                       uint64_t block_size, uint8_t** hashes_out, size_t* nhash_out) try {
  if (!ctx || !hashes_out || !nhash_out || (size && !data)) return fail(CIR_EINVAL, "null pointer");
  if (block_size == 0 || block_size > 0xffffffffull)
    return fail(CIR_EINVAL, "block_size must be in 1 .. 2^32-1");
  if (!valid_hash_type(hash_type)) return fail(CIR_EINVAL, "unknown hash type");
  const bool nt = stage_copy_nt();
  if (ctx->devs.size() > 1 && size > block_size) {
    PosReader prd = [data, nt](uint8_t* dst, uint64_t n, uint64_t off) -> int64_t {
      parallel_pieces(n, [&](uint64_t o, uint64_t len) -> int64_t {
        copy_staged(dst + o, data + off + o, len, nt);
        return (int64_t)len;
      });
      return (int64_t)n;
    };
    HashBuf h;
    int rc = run_split(ctx, prd, size, block_size, h, hash_type);
    if (rc) return rc;
    return export_hashes(h, hashes_out, nhash_out);
  }
  uint64_t pos = 0, got_size = 0;
  Reader rd = [&](uint8_t* dst, uint64_t n) -> int64_t {
    const uint64_t k = std::min(n, size - pos);
    const uint8_t* src = data + pos;
    parallel_pieces(k, [&](uint64_t off, uint64_t len) -> int64_t {
      copy_staged(dst + off, src + off, len, nt);
      return (int64_t)len;
    });
    pos += k;
    return (int64_t)k;
  };
  HashBuf h;
  int rc = run_file(ctx, rd, block_size, &got_size, h, hash_type, size, /*exact=*/true);
  if (rc) return rc;
  return export_hashes(h, hashes_out, nhash_out);
} CIR_CATCH_BOUNDARY

int cir_hash_memory(cir_ctx* ctx, const uint8_t* data, uint64_t size, uint64_t block_size,
                    uint8_t** hashes_out, size_t* nhash_out) try {
  return cir_hash_memory_ht(ctx, CIR_HASH_BLAKE2B_256, data, size, block_size, hashes_out,
                            nhash_out);
} CIR_CATCH_BOUNDARY

// ---- verification (row f2) ---------------------------------------------

int cir_verify_blocks_dev(cir_ctx* ctx, int hash_type, const void* d_arena, const uint64_t* d_off,
                          const uint32_t* d_len, size_t nblk, const uint8_t* d_expected,
                          uint8_t* d_digests, uint8_t* d_ok, uint32_t* d_nbad, void* stream) try {
  if (nblk && (!d_expected || !d_digests)) return fail(CIR_EINVAL, "null device pointer");
  if ((reinterpret_cast<uintptr_t>(d_expected) | reinterpret_cast<uintptr_t>(d_digests)) & 15u)
    return fail(CIR_EINVAL, "digest arrays must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  if (d_nbad) CIR_HIP(hipMemsetAsync(d_nbad, 0, 4, s));
  int rc = cir_hash_blocks_dev_ht(ctx, hash_type, d_arena, d_off, d_len, nblk, d_digests, stream);
  if (rc) return rc;
  CIR_HIP(dev::launch_verify(d_digests, d_expected, nblk, d_ok, d_nbad, s));
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_verify_blocks(cir_ctx* ctx, int hash_type, const uint8_t* h_arena, const uint64_t* off,
                      const uint32_t* len, size_t nblk, const uint8_t* expected, uint8_t* ok_out,
                      size_t* nbad_out) try {
  if (nblk && !expected) return fail(CIR_EINVAL, "null pointer");
  std::vector<uint8_t> got(nblk * 32);
  int rc = cir_hash_blocks_ht(ctx, hash_type, h_arena, off, len, nblk, got.data());
  if (rc) return rc;
  size_t nbad = 0;
  for (size_t b = 0; b < nblk; ++b) {
    const bool good = memcmp(got.data() + 32 * b, expected + 32 * b, 32) == 0;
    if (ok_out) ok_out[b] = good ? 1 : 0;
    nbad += !good;
  }
  if (nbad_out) *nbad_out = nbad;
  return CIR_OK;
} CIR_CATCH_BOUNDARY

// Host descriptors the caller cannot vouch for (the host twins of the
// *_dev_bounded calls): block b is out of range when off[b] + len[b] wraps
// or passes arena_bytes.  Such a block is never read (it is hashed as the
// empty input from the arena's start, then its digest is zeroed); the batch
// is otherwise the plain call's.  Returns the number flagged, with flag[b]
// set, or 0 with nothing copied when every block is in range.
static size_t host_bounds(const uint64_t* off, const uint32_t* len, size_t n,
                          uint64_t arena_bytes, std::vector<uint64_t>& off2,
                          std::vector<uint32_t>& len2, std::vector<uint8_t>& flag) {
  auto out_of_range = [&](size_t b) {
    const uint64_t end = off[b] + len[b];
    return end < off[b] || end > arena_bytes;
  };
  size_t nflag = 0;
  for (size_t b = 0; b < n; ++b) nflag += out_of_range(b);
  if (nflag == 0) return 0;
  off2.assign(off, off + n);
  len2.assign(len, len + n);
  flag.assign(n, 0);
  for (size_t b = 0; b < n; ++b)
    if (out_of_range(b)) {
      flag[b] = 1;
      off2[b] = 0;
      len2[b] = 0;
    }
  return nflag;
}

int cir_hash_blocks_bounded(cir_ctx* ctx, int hash_type, const uint8_t* h_arena,
                            uint64_t arena_bytes, const uint64_t* off, const uint32_t* len,
                            size_t nblk, uint8_t* h_out, size_t* nrange_out) try {
  if (nrange_out) *nrange_out = 0;
  if (nblk && (!off || !len || !h_out)) return fail(CIR_EINVAL, "null pointer");
  if (nblk && !h_arena && arena_bytes) return fail(CIR_EINVAL, "null arena with arena_bytes > 0");
  std::vector<uint64_t> off2;
  std::vector<uint32_t> len2;
  std::vector<uint8_t> flag;
  const size_t nflag = host_bounds(off, len, nblk, arena_bytes, off2, len2, flag);
  static const uint8_t kEmpty = 0;
  const uint8_t* arena = h_arena ? h_arena : &kEmpty;
  const int rc = nflag ? cir_hash_blocks_ht(ctx, hash_type, arena, off2.data(), len2.data(), nblk,
                                            h_out)
                       : cir_hash_blocks_ht(ctx, hash_type, arena, off, len, nblk, h_out);
  if (rc) return rc;
  for (size_t b = 0; nflag && b < nblk; ++b)
    if (flag[b]) memset(h_out + 32 * b, 0, 32);
  if (nrange_out) *nrange_out = nflag;
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_verify_blocks_bounded(cir_ctx* ctx, int hash_type, const uint8_t* h_arena,
                              uint64_t arena_bytes, const uint64_t* off, const uint32_t* len,
                              size_t nblk, const uint8_t* expected, uint8_t* ok_out,
                              size_t* nbad_out) try {
  if (nblk && !expected) return fail(CIR_EINVAL, "null pointer");
  std::vector<uint8_t> got(nblk * 32);
  size_t nrange = 0;
  int rc = cir_hash_blocks_bounded(ctx, hash_type, h_arena, arena_bytes, off, len, nblk,
                                   got.data(), &nrange);
  if (rc) return rc;
  // an out-of-range block is a mismatch whatever its expected digest (its
  // zeroed digest must not match an all-zero expected one)
  std::vector<uint64_t> off2;
  std::vector<uint32_t> len2;
  std::vector<uint8_t> flag;
  if (nrange) host_bounds(off, len, nblk, arena_bytes, off2, len2, flag);
  size_t nbad = 0;
  for (size_t b = 0; b < nblk; ++b) {
    const bool good =
        (!nrange || !flag[b]) && memcmp(got.data() + 32 * b, expected + 32 * b, 32) == 0;
    if (ok_out) ok_out[b] = good ? 1 : 0;
    nbad += !good;
  }
  if (nbad_out) *nbad_out = nbad;
  return CIR_OK;
} CIR_CATCH_BOUNDARY

}  // extern "C"

// ---- asynchronous verify (row f2, the daemon's per-block caller) --------
// The queue, its worker and its bounds are verify_queue.hpp; a context's
// queue hashes each batch as one host batch straight from the batch's arena
// (cir_hash_blocks_ht), created on the first verify call.
namespace cir {

static VerifyQueue* verify_queue(cir_ctx* ctx) {
  std::lock_guard<std::mutex> lk(ctx->av_mu);
  if (!ctx->av)
    ctx->av = std::make_unique<VerifyQueue>(
        [ctx](int ht, const uint8_t* arena, const uint64_t* off, const uint32_t* len, size_t n,
              uint8_t* out, std::string* err) {
          const int rc = cir_hash_blocks_ht(ctx, ht, arena, off, len, n, out);
          if (rc) *err = cir_last_error();
          return rc;
        });
  return ctx->av.get();
}

}  // namespace cir

extern "C" {

int cir_verify_submit(cir_ctx* ctx, int hash_type, const uint8_t* data, size_t n,
                      const uint8_t expected[CIR_DIGEST_BYTES], uint64_t* ticket) try {
  if (!ctx || !ticket || !expected || (n && !data)) return fail(CIR_EINVAL, "null pointer");
  if (!valid_hash_type(hash_type)) return fail(CIR_EINVAL, "unknown hash type");
  if (n > 0xffffffffull) return fail(CIR_EINVAL, "block longer than 4 GiB");
  std::string err;
  const int rc = verify_queue(ctx)->submit(hash_type, data, n, expected, ticket, &err);
  return rc ? fail(rc, err) : CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_verify_poll(cir_ctx* ctx, uint64_t ticket, int* state) try {
  if (!ctx || !state) return fail(CIR_EINVAL, "null pointer");
  std::string err;
  const int v = verify_queue(ctx)->poll(ticket, &err);
  if (v < 0) return fail(v, err);
  *state = v;
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_verify_wait(cir_ctx* ctx, uint64_t ticket, int* ok) try {
  if (!ctx || !ok) return fail(CIR_EINVAL, "null pointer");
  std::string err;
  const int v = verify_queue(ctx)->wait(ticket, &err);
  if (v < 0) return fail(v, err);
  *ok = v == 1;
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_verify_forget(cir_ctx* ctx, uint64_t ticket) try {
  if (!ctx) return fail(CIR_EINVAL, "null ctx");
  std::string err;
  const int rc = verify_queue(ctx)->forget(ticket, &err);
  return rc ? fail(rc, err) : CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_verify_window(cir_ctx* ctx, uint32_t window_us, uint32_t max_batch) try {
  if (!ctx || max_batch == 0) return fail(CIR_EINVAL, "bad argument");
  verify_queue(ctx)->window(window_us, max_batch);
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_verify_limits(cir_ctx* ctx, uint64_t max_bytes, uint64_t max_results, int flags) try {
  if (!ctx) return fail(CIR_EINVAL, "null ctx");
  if (flags & ~CIR_VERIFY_NONBLOCK) return fail(CIR_EINVAL, "unknown flags");
  verify_queue(ctx)->limits(max_bytes, max_results, (flags & CIR_VERIFY_NONBLOCK) != 0);
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_verify_stats(cir_ctx* ctx, uint64_t out[CIR_VERIFY_STATS_FIELDS]) try {
  if (!ctx || !out) return fail(CIR_EINVAL, "null pointer");
  verify_queue(ctx)->stats(out);
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_check_file(cir_ctx* ctx, int hash_type, int fd, uint64_t block_size,
                   const uint8_t* expected, size_t nhash, int* ok_out) try {
  if (!ctx || !ok_out || (nhash && !expected)) return fail(CIR_EINVAL, "null pointer");
  uint8_t* h = nullptr;
  size_t n = 0;
  uint64_t size = 0;
  int rc = cir_hash_file_ht(ctx, hash_type, fd, block_size, &size, &h, &n);
  if (rc) return rc;
  *ok_out = n == nhash && (n == 0 || memcmp(h, expected, 32 * n) == 0);
  free(h);
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_debug_hash_uniform_dev(int loader, const void* d_data, uint64_t block_size, uint64_t nblk,
                               uint8_t* d_out, void* stream) try {
  if (block_size == 0 || block_size % 128 || nblk % dev::kThreads || (loader != 0 && loader != 1) ||
      (reinterpret_cast<uintptr_t>(d_data) & 15u))
    return fail(CIR_EINVAL, "uniform kernel needs bs % 128 == 0, nblk % 256 == 0, 16-B alignment");
  CIR_HIP(dev::launch_uniform(loader == 0 ? dev::Loader::kGlds : dev::Loader::kDirect,
                              (const uint8_t*)d_data, block_size, nblk, d_out, (hipStream_t)stream));
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_debug_compress_only_dev(uint64_t nlanes, uint32_t lines, uint8_t* d_out, void* stream) try {
  if (nlanes % dev::kThreads || lines == 0 || !d_out)
    return fail(CIR_EINVAL, "compress-only kernel needs nlanes % 256 == 0, lines > 0, an output");
  CIR_HIP(dev::launch_compress_only(nlanes, lines, d_out, (hipStream_t)stream));
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_debug_desc_timing(cir_ctx* ctx, int enable) try {
  if (!ctx || ctx->devs.empty()) return fail(CIR_EINVAL, "null ctx");
  Device& d = *ctx->devs[0];
  std::lock_guard<std::mutex> lk(d.order_mu);
  d.timing = enable != 0;
  d.tev_used = 0;
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_debug_desc_times(cir_ctx* ctx, double out[5]) try {
  if (!ctx || ctx->devs.empty() || !out) return fail(CIR_EINVAL, "null pointer");
  Device& d = *ctx->devs[0];
  std::lock_guard<std::mutex> lk(d.order_mu);
  DeviceGuard guard;
  CIR_HIP(hipSetDevice(d.id));
  for (int k = 0; k < 5; ++k) out[k] = 0.0;
  for (size_t b = 0; b < d.tev_used; ++b) {
    const auto& e = d.tev[b];
    for (hipEvent_t x : e) CIR_HIP(hipEventSynchronize(x));
    float order = 0, quad = 0, lane = 0, to_q = 0, to_l = 0;
    CIR_HIP(hipEventElapsedTime(&order, e[0], e[1]));
    CIR_HIP(hipEventElapsedTime(&quad, e[2], e[3]));
    CIR_HIP(hipEventElapsedTime(&lane, e[4], e[5]));
    CIR_HIP(hipEventElapsedTime(&to_q, e[0], e[3]));
    CIR_HIP(hipEventElapsedTime(&to_l, e[0], e[5]));
    out[0] += 1.0;
    out[1] += order;
    out[2] += quad;
    out[3] += lane;
    out[4] += std::max(to_q, to_l);
  }
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_debug_device_identity(int device, char* pci_bus_id, size_t len, uint8_t uuid[16],
                              uint64_t clocks[5]) try {
  if (!pci_bus_id || len < 13 || !uuid || !clocks) return fail(CIR_EINVAL, "null pointer");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
    return fail(CIR_ENODEV, "no such HIP device");
  DeviceGuard guard;
  CIR_HIP(hipSetDevice(device));
  CIR_HIP(hipDeviceGetPCIBusId(pci_bus_id, (int)std::min<size_t>(len, 256), device));
  hipUUID u;
  CIR_HIP(hipDeviceGetUuid(&u, device));
  memcpy(uuid, u.bytes, 16);
  int rate_khz = 0;
  CIR_HIP(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, device));
  uint64_t* d = nullptr;
  CIR_HIP(hipMalloc(&d, 4 * sizeof(uint64_t)));
  // ~100 us of wall-clock ticks between the two reads
  const uint64_t spin = std::max<uint64_t>(1, (uint64_t)rate_khz / 10);
  hipError_t e = dev::launch_clock_probe(d, spin, nullptr);
  if (e == hipSuccess) e = hipMemcpy(clocks, d, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(e, "clock probe");
  clocks[4] = (uint64_t)rate_khz;
  return CIR_OK;
} CIR_CATCH_BOUNDARY

uint64_t cir_debug_relay_blocks(uint64_t nfull, uint64_t block_size) {
  return dev::relay_blocks(nfull, block_size);
}

int cir_fill_splitmix64_dev(void* d_ptr, uint64_t nbytes, uint64_t seed, uint64_t block_bytes,
                            uint64_t first_block, void* stream) try {
  if (nbytes % 8 || block_bytes % 8) return fail(CIR_EINVAL, "sizes must be multiples of 8");
  if (nbytes && !d_ptr) return fail(CIR_EINVAL, "null device pointer");
  CIR_HIP(dev::launch_fill_splitmix64((uint64_t*)d_ptr, nbytes / 8, seed, block_bytes / 8,
                                      first_block, (hipStream_t)stream));
  return CIR_OK;
} CIR_CATCH_BOUNDARY

}  // extern "C"
