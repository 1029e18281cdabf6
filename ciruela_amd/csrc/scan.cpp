// cir_scan_v1: dir_signature::v1::scan on the GPU path, and index helpers.
//
// Reference: the scan call of `ciruela sync` (src/client/sync/uploads.rs:
// 49-59: ScannerConfig::new, threads(gopt.threads), hash(blake2b_256()),
// add_dir(dir, "/"), v1::scan(&cfg, &mut index_buf)) and of
// examples/custom_uploader.rs:59-65.  The crate walks the tree, splits every
// regular file into block_size blocks and hashes each block on a CPU pool;
// here host reader threads only stage file bytes into pinned buffers and
// every block (and the footer) is hashed by the gfx950 kernels.
//
// Order of the emitted index (restated from the reference's own re-emitter,
// MutableIndex::to_raw_data / _emit_dir, src/cluster/download.rs:287-319):
// a directory line, its files and symlinks sorted by name (bytewise), then
// its subdirectories recursively in name order.
#include <dirent.h>
#include <stdio.h>
#include <errno.h>
#include <fcntl.h>
#include <limits.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <map>
#include <memory>
#include <functional>
#include <thread>

#include "blake2b_host.hpp"
#include "dirsig.hpp"
#include "sha512_host.hpp"
#include "stripes.hpp"
#include "runtime.hpp"

namespace cir {

struct ScanFile {
  std::string real;
  uint64_t size = 0;
  uint64_t first_blk = 0;  // global block index of block 0
};

struct PlanItem {
  dirsig::EntryKind kind;
  std::string name;  // kDir: virtual path; else entry name
  bool exe = false;
  size_t file = 0;     // kFile: index into files
  std::string target;  // kLink
};

// open(2) for a path of any length.  Below PATH_MAX the path opens as it
// is; a longer one is opened piecewise -- each piece shorter than PATH_MAX
// and ending at a '/' -- relative to the directory the previous piece opened
// (openat), so the files of a tree nested past PATH_MAX still open.
static int open_long(const std::string& path, int flags) {
  flags |= O_CLOEXEC;
  if (path.size() < PATH_MAX) return ::open(path.c_str(), flags);
  int dfd = AT_FDCWD;
  size_t pos = 0;
  auto drop = [&dfd] {
    if (dfd != AT_FDCWD) {
      const int e = errno;
      ::close(dfd);
      errno = e;
    }
  };
  while (path.size() - pos >= PATH_MAX) {
    const size_t cut = path.rfind('/', pos + PATH_MAX - 2);
    if (cut == std::string::npos || cut < pos) {  // one component longer than PATH_MAX
      drop();
      errno = ENAMETOOLONG;
      return -1;
    }
    const std::string piece = cut > pos ? path.substr(pos, cut - pos) : pos == 0 ? "/" : ".";
    const int nfd = ::openat(dfd, piece.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
    drop();
    if (nfd < 0) return -1;
    dfd = nfd;
    pos = cut + 1;
  }
  const int fd = ::openat(dfd, path.c_str() + pos, flags);
  drop();
  return fd;
}

// The tree walk.  Directories are read in parallel -- each one's entries
// listed, sorted and lstat'ed by whichever walker thread takes it, its
// subdirectories queued for the others (a tree of many small files is
// metadata-bound: 200,000 files took 265 ms on one thread,
// tools/manyfiles_probe.py) -- and the plan is then put together on the
// calling thread in the serial walk's order: a directory's line, its files
// and symlinks in name order, then its subdirectories in name order, depth
// first.  A failure is reported as the serial walk would meet it first: a
// directory's own error (opening or listing it, an lstat, a readlink) before
// anything below it.
//
// Every directory is opened relative to its parent's fd (openat with
// O_NOFOLLOW: the entry lstat'ed as a directory is the one read) and listed,
// lstat'ed and read-linked through its own fd (fdopendir, fstatat
// AT_SYMLINK_NOFOLLOW, readlinkat), as dir-signature 0.2.9 walks with openat
// (Cargo.lock:323): no call takes the full path, so a tree nested past
// PATH_MAX indexes like any other.  A directory's fd stays open until it has
// been listed and every subdirectory has opened its own from it (a count of
// holders); subdirectories are taken last-queued first, so the fds open at
// once stay near the walkers' depth, not the tree's width.
struct DirNode {
  struct Ent {
    std::string name;
    mode_t mode = 0;
    uint64_t size = 0;
    std::string target;  // symlinks
  };
  std::string real, vpath, name;  // name: the entry in the parent
  DirNode* parent = nullptr;
  int fd = -1;
  std::atomic<size_t> holders{1};  // itself while it is read, then each unopened subdir
  std::vector<Ent> ents;  // files and symlinks, name order
  std::vector<std::unique_ptr<DirNode>> subdirs;  // name order
  int rc = CIR_OK;
  std::string err;  // the first failure met in this directory
};

static void release_fd(DirNode& n) {
  if (n.holders.fetch_sub(1) == 1 && n.fd >= 0) {
    ::close(n.fd);
    n.fd = -1;
  }
}

static void read_dir(DirNode& n) {
  // this directory's fd: the root by its path, the rest relative to the
  // parent's (which stays open for it), never through a symlink
  n.fd = n.parent
             ? ::openat(n.parent->fd, n.name.c_str(),
                        O_RDONLY | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC)
             : open_long(n.real, O_RDONLY | O_DIRECTORY);
  const int open_errno = errno;
  if (n.parent) release_fd(*n.parent);
  if (n.fd < 0) {
    n.rc = CIR_EIO;
    n.err = "error indexing dir " + n.real + ": " + strerror(open_errno);
    return;
  }
  // (fdopendir owns the fd it is given: a duplicate, so n.fd stays ours)
  const int lfd = ::fcntl(n.fd, F_DUPFD_CLOEXEC, 0);
  DIR* d = lfd >= 0 ? ::fdopendir(lfd) : nullptr;
  if (!d) {
    const int e = errno;
    if (lfd >= 0) ::close(lfd);
    n.rc = CIR_EIO;
    n.err = "error indexing dir " + n.real + ": " + strerror(e);
    return;
  }
  std::vector<std::string> names;
  for (;;) {
    errno = 0;
    struct dirent* de = ::readdir(d);
    if (!de) {
      // NULL is the end of the directory only when errno is untouched
      if (errno != 0) {
        const int e = errno;
        ::closedir(d);
        n.rc = CIR_EIO;
        n.err = "error reading dir " + n.real + ": " + strerror(e);
        return;
      }
      break;
    }
    if (!strcmp(de->d_name, ".") || !strcmp(de->d_name, "..")) continue;
    names.emplace_back(de->d_name);
  }
  ::closedir(d);
  std::sort(names.begin(), names.end());
  for (std::string& nm : names) {
    struct stat st;
    if (::fstatat(n.fd, nm.c_str(), &st, AT_SYMLINK_NOFOLLOW) != 0) {
      n.rc = CIR_EIO;
      n.err = "error indexing dir " + n.real + "/" + nm + ": " + strerror(errno);
      return;
    }
    if (S_ISDIR(st.st_mode)) {
      auto c = std::make_unique<DirNode>();
      c->real = n.real + "/" + nm;
      c->vpath = n.vpath == "/" ? "/" + nm : n.vpath + "/" + nm;
      c->name = std::move(nm);
      c->parent = &n;
      n.subdirs.push_back(std::move(c));
    } else if (S_ISREG(st.st_mode)) {
      DirNode::Ent e;
      e.name = std::move(nm);
      e.mode = st.st_mode;
      e.size = (uint64_t)st.st_size;
      n.ents.push_back(std::move(e));
    } else if (S_ISLNK(st.st_mode)) {
      std::string tgt(4096, '\0');
      const ssize_t r = ::readlinkat(n.fd, nm.c_str(), &tgt[0], tgt.size());
      if (r < 0) {
        n.rc = CIR_EIO;
        n.err = "error reading link " + n.real + "/" + nm + ": " + strerror(errno);
        return;
      }
      tgt.resize((size_t)r);
      DirNode::Ent e;
      e.name = std::move(nm);
      e.mode = st.st_mode;
      e.target = std::move(tgt);
      n.ents.push_back(std::move(e));
    }
    // sockets, fifos and devices are not part of an image
  }
}

static int emit_plan(DirNode& n, std::vector<PlanItem>& plan, std::vector<ScanFile>& files) {
  if (n.rc) return fail(n.rc, n.err);
  PlanItem di;
  di.kind = dirsig::EntryKind::kDir;
  di.name = n.vpath;
  plan.push_back(std::move(di));
  for (DirNode::Ent& e : n.ents) {
    PlanItem it;
    it.name = e.name;
    if (S_ISLNK(e.mode)) {
      it.kind = dirsig::EntryKind::kLink;
      it.target = std::move(e.target);
    } else {
      it.kind = dirsig::EntryKind::kFile;
      it.exe = (e.mode & 0111) != 0;
      it.file = files.size();
      ScanFile f;
      f.real = n.real + "/" + e.name;
      f.size = e.size;
      files.push_back(std::move(f));
    }
    plan.push_back(std::move(it));
  }
  for (auto& c : n.subdirs) {
    const int rc = emit_plan(*c, plan, files);
    if (rc) return rc;
  }
  return CIR_OK;
}

static void close_all(DirNode& n) {
  if (n.fd >= 0) ::close(n.fd);
  n.fd = -1;
  for (auto& c : n.subdirs) close_all(*c);
}

static int walk(const std::string& real, const std::string& vpath, unsigned threads,
                std::vector<PlanItem>& plan, std::vector<ScanFile>& files) {
  DirNode root;
  root.real = real;
  root.vpath = vpath;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<DirNode*> stack{&root};  // last queued first (see above)
  size_t busy = 0;
  parallel_run(std::max(1u, threads), [&] {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return !stack.empty() || busy == 0; });
      if (stack.empty()) return;  // nothing queued, nobody reading: done
      DirNode* n = stack.back();
      stack.pop_back();
      ++busy;
      lk.unlock();
      try {
        read_dir(*n);
      } catch (...) {  // (no exception may leave a walker: the others wait on busy)
        n->rc = CIR_ENOMEM;
        n->err = "walking " + n->real + ": out of memory";
        n->subdirs.clear();
      }
      if (n->rc != CIR_OK) n->subdirs.clear();  // none of them will be read
      // each subdirectory holds this fd until it has opened its own; the
      // read itself lets go of it now
      n->holders.fetch_add(n->subdirs.size());
      release_fd(*n);
      lk.lock();
      --busy;
      if (n->rc == CIR_OK) {
        try {
          // pushed in reverse name order: the first subdirectory is read first
          for (auto it = n->subdirs.rbegin(); it != n->subdirs.rend(); ++it)
            stack.push_back(it->get());
        } catch (...) {  // (the others must still be woken below)
          n->rc = CIR_ENOMEM;
          n->err = "walking " + n->real + ": out of memory";
          // the subdirectories not queued still hold this fd: close_all
        }
      }
      cv.notify_all();
    }
  });
  close_all(root);  // (only an out-of-memory walk leaves an fd open)
  return emit_plan(root, plan, files);
}

// Read jobs are cut into pieces of at most this size so that `threads`
// readers stay busy on trees of large files.
constexpr uint64_t kReadPiece = 4ull << 20;

static bool trace_on() { return trace_enabled(); }

static double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct ReadJob {
  size_t file;
  uint64_t file_off;
  uint64_t len;
  uint8_t* dst;
};

static int run_reads(const std::vector<ReadJob>& jobs, const std::vector<ScanFile>& files,
                     unsigned threads) {
  std::atomic<size_t> next{0};
  std::atomic<int> rc{0};
  std::string err;
  std::mutex err_mu;
  const bool nt = stage_copy_nt();
  auto worker = [&] {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= jobs.size() || rc.load()) return;
      const ReadJob& j = jobs[i];
      const std::string& path = files[j.file].real;
      const int fd = open_long(path, O_RDONLY);
      bool ok = fd >= 0;
      uint64_t got = 0;
      while (ok && got < j.len) {
        // into the pinned slot (streaming stores through a bounce buffer by
        // default: runtime.cpp pread_staged)
        const ssize_t r =
            pread_staged(fd, j.dst + got, j.len - got, (off_t)(j.file_off + got), nt);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) {
          ok = false;
          if (r == 0) errno = ENODATA;  // file shrank during the scan
          break;
        }
        got += (uint64_t)r;
      }
      const int e = errno;
      if (fd >= 0) ::close(fd);
      if (!ok) {
        std::lock_guard<std::mutex> lk(err_mu);
        if (!rc.load()) err = "error reading " + path + ": " + strerror(e);
        rc.store(CIR_EIO);
        return;
      }
    }
  };
  parallel_run(std::max(1u, std::min<unsigned>(threads, (unsigned)jobs.size())), worker);
  if (rc.load()) return fail(rc.load(), err);
  return CIR_OK;
}

// The scan's digests, 32 bytes per block in the global block order.
struct DigestBuf {
  std::unique_ptr<uint8_t[]> p;
  uint8_t* data() { return p.get(); }
};

// Hash every block of every file; digests[32*g] for global block g.
// Batches are packed into the two staging slots of device 0 (file segments
// 16-byte aligned, one descriptor per block) by `threads` reader threads
// while the previous batch uploads and hashes.
using Progress = std::function<int(uint64_t done_blk)>;

// The block ranges `ranges` (each [b0, b1) of the global block order, in
// increasing order; a range may start or end inside a file) on device d, one
// pipeline across all of them (a batch never spans two ranges).  done(r, n)
// is called after each batch with the range's index and the number of its
// blocks finished so far (a prefix of the range: the slots retire in
// submission order).
// With `scan_t0` >= 0 (cir_debug_scan_timing on) every batch is timed and
// appended to ctx->stats as a row (include/ciruela_blockhash.h), times in ms
// since scan_t0 on the host clock; the device's copy stream gets a reference
// event at the start that maps its HIP event times onto that clock.
using BlockRanges = std::vector<std::pair<uint64_t, uint64_t>>;
static int hash_range(cir_ctx* ctx, Device& d, size_t di, const std::vector<ScanFile>& files,
                      uint64_t bs, unsigned threads, int ht, DigestBuf& digests,
                      const BlockRanges& ranges,
                      const std::function<int(size_t, uint64_t)>& done, double scan_t0) {
  if (ranges.empty()) return CIR_OK;
  std::lock_guard<std::mutex> lk(d.mu);
  DeviceGuard guard;
  CIR_HIP(hipSetDevice(d.id));
  SlotDrain drain{d};  // an early return leaves no slot busy
  const bool stats = scan_t0 >= 0;
  struct RecordTimes {  // the device's slots are timed for this range only
    Device& d;
    ~RecordTimes() { d.record_times = false; }
  } record_times{d};
  d.record_times = stats;
  double ref_ms = 0;  // host time of the copy stream's reference event
  if (stats) {
    if (!d.t_ref) CIR_HIP(hipEventCreate(&d.t_ref));
    CIR_HIP(hipEventRecord(d.t_ref, d.copy));
    ref_ms = now_ms() - scan_t0;
  }
  std::vector<std::array<double, kScanBatchFields>> rows;
  // A slot holds at least one block; a block is never longer than the
  // largest file, so a huge block size over small files does not grow the
  // slots to the block size.  (A multiple of 16: segments start 16-byte
  // aligned.)
  uint64_t seg = 0;
  for (const ScanFile& f : files) seg = std::max(seg, std::min<uint64_t>(f.size, bs));
  const uint64_t cap = (std::max<uint64_t>(ctx->staging, seg + 16) + 15) & ~15ull;
  const uint64_t cap_blk = std::max<uint64_t>(cap / 512, 4096);
  // the first batches ramp up (1/8, 1/4, 1/2 of a slot, then whole slots):
  // the first upload starts after a short read instead of a whole slot's,
  // and each read still finishes within the previous upload
  uint64_t fill = scan_ramp() ? std::max<uint64_t>(seg + 16, cap >> 3) : cap;
  size_t ri = 0;  // the range being packed
  uint64_t b0 = 0, b1 = 0;
  size_t fi = 0;
  uint64_t fblk = 0;  // next block within files[fi]
  auto start_range = [&](size_t r) {
    ri = r;
    b0 = ranges[r].first;
    b1 = ranges[r].second;
    // the last file whose first block is <= b0 (empty files share first_blk)
    fi = std::upper_bound(files.begin(), files.end(), b0,
                          [](uint64_t b, const ScanFile& f) { return b < f.first_blk; }) -
         files.begin();
    fi = fi ? fi - 1 : 0;
    fblk = b0 > files[fi].first_blk ? b0 - files[fi].first_blk : 0;
  };
  start_range(0);
  constexpr int kS = Device::kSlots;
  uint64_t pending_first[kS] = {}, pending_n[kS] = {};
  size_t pending_range[kS] = {};
  double pending_row[kS][6] = {};  // bytes, blocks, wait, read start, read end
  int k = 0;
  auto busy = [&] {
    for (const Slot& s : d.slot)
      if (s.busy) return true;
    return false;
  };
  // blocks left in the current range
  auto more_here = [&] {
    while (fi < files.size() && fblk * bs >= files[fi].size) {
      ++fi;
      fblk = 0;
    }
    return fi < files.size() && files[fi].first_blk + fblk < b1;
  };
  // blocks left in this or a later range (moves on to the next range)
  auto more = [&] {
    while (!more_here()) {
      if (ri + 1 >= ranges.size()) return false;
      start_range(ri + 1);
    }
    return true;
  };
  while (more() || busy()) {
    Slot& s = d.slot[k];
    const double t_wait0 = (trace_on() || stats) ? now_ms() : 0;
    if (s.busy) {
      const bool timed = s.timed;
      int rc = slot_wait(d, s);
      if (rc) return rc;
      if (timed && trace_on()) {
        float copy_ms = 0, hash_ms = 0, gap_ms = 0;
        (void)hipEventElapsedTime(&copy_ms, s.t_copy0, s.t_copy1);
        (void)hipEventElapsedTime(&gap_ms, s.t_copy1, s.t_hash0);
        (void)hipEventElapsedTime(&hash_ms, s.t_hash0, s.t_done);
        fprintf(stderr, "cir_scan dev %d slot %d: h2d %.2f ms, h2d->hash %.2f ms, hash+d2h %.2f ms\n",
                d.id, k, copy_ms, gap_ms, hash_ms);
      }
      if (timed && stats) {
        float e[4] = {0, 0, 0, 0};
        const hipEvent_t ev[4] = {s.t_copy0, s.t_copy1, s.t_hash0, s.t_done};
        for (int j = 0; j < 4; ++j) CIR_HIP(hipEventElapsedTime(&e[j], d.t_ref, ev[j]));
        rows.push_back({(double)di, pending_row[k][0], pending_row[k][1], pending_row[k][2],
                        pending_row[k][3], pending_row[k][4], ref_ms + e[0], ref_ms + e[1],
                        ref_ms + e[2], ref_ms + e[3]});
      }
      memcpy(digests.data() + 32 * pending_first[k], s.h_out, 32 * pending_n[k]);
      const size_t pr = pending_range[k];
      rc = done(pr, pending_first[k] + pending_n[k] - ranges[pr].first);
      if (rc) return rc;
    }
    const bool clock = trace_on() || stats;
    const double t_wait1 = clock ? now_ms() : 0;
    if (more()) {
      int rc = d.ensure_slot(s, cap, cap_blk);
      if (rc) return rc;
      std::vector<ReadJob> jobs;
      uint64_t pos = 0, n = 0;
      uint64_t used = 0;  // end of the last segment packed (pos may be aligned past it)
      const uint64_t first = files[fi].first_blk + fblk;
      while (more_here() && n < cap_blk) {
        const ScanFile& f = files[fi];
        const uint64_t left_blk = std::min<uint64_t>((f.size + bs - 1) / bs - fblk,
                                                     b1 - (f.first_blk + fblk));
        pos = (pos + 15) & ~15ull;
        if (pos + std::min<uint64_t>(bs, f.size - fblk * bs) > fill) break;
        // as many whole blocks of this file as fit
        uint64_t take = std::min<uint64_t>(left_blk, cap_blk - n);
        take = std::min<uint64_t>(take, std::max<uint64_t>((fill - pos) / bs, 1));
        const uint64_t off0 = fblk * bs;
        const uint64_t bytes = std::min<uint64_t>(take * bs, f.size - off0);
        if (pos + bytes > fill) break;
        for (uint64_t j = 0; j < take; ++j) {
          s.h_off[n + j] = pos + j * bs;
          s.h_len[n + j] = (uint32_t)std::min<uint64_t>(bs, f.size - off0 - j * bs);
        }
        for (uint64_t piece = 0; piece < bytes; piece += kReadPiece)
          jobs.push_back({fi, off0 + piece, std::min<uint64_t>(kReadPiece, bytes - piece),
                          s.h_data + pos + piece});
        pos += bytes;
        used = pos;
        n += take;
        fblk += take;
      }
      fill = std::min(cap, fill * 2);
      const double t_read0 = clock ? now_ms() : 0;
      rc = run_reads(jobs, files, threads);
      if (rc) return rc;
      const double t_read1 = clock ? now_ms() : 0;
      // the packed bytes only: a break after aligning `pos` for the next
      // segment must not send the slot's end (round 4 sent up to 15 bytes
      // past a slot whose size was not a multiple of 16: a block size above
      // the staging size failed the upload)
      rc = slot_submit(d, s, std::max<uint64_t>(used, 16), n, ht);
      if (rc) return rc;
      if (trace_on())
        fprintf(stderr, "cir_scan dev %d batch: %.1f MiB, %zu jobs, wait %.2f ms, read %.2f ms (%.1f GB/s)\n",
                d.id, used / 1048576.0, jobs.size(), t_wait1 - t_wait0, t_read1 - t_read0,
                used / 1e6 / std::max(t_read1 - t_read0, 1e-3));
      pending_first[k] = first;
      pending_n[k] = n;
      pending_range[k] = ri;
      if (stats) {
        pending_row[k][0] = (double)used;
        pending_row[k][1] = (double)n;
        pending_row[k][2] = t_wait1 - t_wait0;
        pending_row[k][3] = t_read0 - scan_t0;
        pending_row[k][4] = t_read1 - scan_t0;
      }
    }
    k = (k + 1) % kS;
  }
  if (stats) {
    std::lock_guard<std::mutex> sl(ctx->stats.mu);
    ctx->stats.batches.insert(ctx->stats.batches.end(), rows.begin(), rows.end());
  }
  return CIR_OK;
}

// Hash every block of every file; digests[32*g] for global block g.
// Batches are packed into the staging slots of a device (file segments
// 16-byte aligned, one descriptor per block) by `threads` reader threads
// while the previous batches upload and hash.  With several devices in the
// context the global block order is cut into stripes of one staging batch's
// worth of whole blocks, dealt round-robin to the devices (SURVEY.md 8e's
// range split, interleaved), each device driven by its own thread with
// threads / ndev readers; progress(n) reports the prefix of the global order
// that is complete -- with interleaved stripes it advances steadily while the
// devices work, so the emitter and the footer keep streaming (one contiguous
// range per device held the whole index back until device 0's range had
// finished, and hashed most of the footer after the last batch) -- called
// under a lock with device 0 current.
static int hash_files(cir_ctx* ctx, std::vector<ScanFile>& files, uint64_t bs, unsigned threads,
                      int ht, DigestBuf& digests, const Progress& progress,
                      double scan_t0) {
  uint64_t nblk_total = 0;
  for (ScanFile& f : files) {
    f.first_blk = nblk_total;
    nblk_total += (f.size + bs - 1) / bs;
  }
  // not zero-filled: every digest is written before its file is emitted,
  // and the pages are touched by those copies as the batches come back
  // instead of up front (52 MB for config 5: ~5-8 ms before the first read)
  digests.p.reset(new uint8_t[32 * nblk_total]);
  if (nblk_total == 0) return CIR_OK;
  const size_t nd = std::min<size_t>(ctx->devs.size(), nblk_total);
  if (nd <= 1)
    return hash_range(ctx, *ctx->devs[0], 0, files, bs, threads, ht, digests,
                      {{0, nblk_total}},
                      [&](size_t, uint64_t n) { return progress(n); }, scan_t0);
  uint64_t stripe = std::max<uint64_t>(1, ctx->staging / bs);
  if (const char* e = getenv("CIR_DEBUG_STRIPE_BLOCKS"))  // tests: stripes of a few blocks
    if (atoll(e) > 0) stripe = (uint64_t)atoll(e);
  StripePrefix order(nblk_total, stripe);
  const size_t nstripes = order.stripes();
  std::vector<BlockRanges> dev_ranges(nd);
  std::vector<std::vector<size_t>> global_index(nd);  // (device, range) -> stripe
  for (size_t st = 0; st < nstripes; ++st) {
    const size_t i = st % nd;
    dev_ranges[i].push_back({st * stripe, std::min<uint64_t>((st + 1) * stripe, nblk_total)});
    global_index[i].push_back(st);
  }
  std::mutex mu;
  const int dev0 = ctx->devs[0]->id;
  auto done = [&](size_t i, size_t r, uint64_t n) -> int {
    std::lock_guard<std::mutex> lk(mu);
    uint64_t prefix = 0;
    // (a batch inside the first open stripe extends the prefix too, and so
    // does the last stripe's completion)
    if (!order.update(global_index[i][r], n, &prefix)) return CIR_OK;
    int cur = 0;
    CIR_HIP(hipGetDevice(&cur));
    CIR_HIP(hipSetDevice(dev0));
    const int rc = progress(prefix);
    CIR_HIP(hipSetDevice(cur));
    return rc;
  };
  const unsigned per = std::max(1u, threads / (unsigned)nd);
  std::vector<int> rc(nd, 0);
  std::vector<std::string> err(nd);
  fan_out(nd, [&](size_t i) {
    rc[i] = hash_range(ctx, *ctx->devs[i], i, files, bs, per, ht, digests, dev_ranges[i],
                       [&, i](size_t r, uint64_t n) { return done(i, r, n); }, scan_t0);
    if (rc[i]) err[i] = cir_last_error();
  });
  for (size_t i = 0; i < nd; ++i)
    if (rc[i]) return fail(rc[i], err[i]);
  CIR_HIP(hipSetDevice(dev0));
  return CIR_OK;
}

// ---- incremental footer ---------------------------------------------------
// The footer is H(index body): one sequential chain over the whole body.  The
// body is emitted as the files' digests come back, and every completed
// stretch of it (whole 128-B lines, at least one byte held back for the
// final block) is fed to a resumable single-chain kernel on the device's
// `chain` stream, so the chain advances while later batches are still read
// and hashed.
struct FooterChain {
  Device& d;
  size_t fed = 0;
  int k = 0;
  size_t feeds = 0;
  // with `timed`, a pair of HIP events around every chain-step launch (the
  // kernel only, not its text upload): busy_ms() sums them
  bool timed = false;
  std::vector<hipEvent_t> tev;
  explicit FooterChain(Device& dev, bool t) : d(dev), timed(t) {}
  ~FooterChain() {
    if (!tev.empty()) (void)hipStreamSynchronize(d.chain);
    for (hipEvent_t e : tev) (void)hipEventDestroy(e);
  }
  double busy_ms() {
    double ms = 0;
    for (size_t i = 0; i + 1 < tev.size(); i += 2) {
      float x = 0;
      if (hipEventElapsedTime(&x, tev[i], tev[i + 1]) == hipSuccess) ms += x;
    }
    return ms;
  }

  // (caller holds d.chain_mu.)  A one-shot context's device has the chain
  // state and events from cir_init but no chain stream: each piece missing
  // is created here, and only those.
  int start() {
    if (!d.chain) CIR_HIP(hipStreamCreateWithFlags(&d.chain, hipStreamNonBlocking));
    if (!d.chain_state) CIR_HIP(hipMalloc(&d.chain_state, 16 * 8));
    for (int b = 0; b < 2; ++b)
      if (!d.chain_done[b])
        CIR_HIP(hipEventCreateWithFlags(&d.chain_done[b], hipEventDisableTiming));
    CIR_HIP(hipMemsetAsync(d.chain_state, 0, 16 * 8, d.chain));
    fed = 0;
    return CIR_OK;
  }

  // feed body[fed, fed + n) (n whole lines unless final)
  int push(const dirsig::Emitter& em, size_t n, bool final) {
    while (n > 0 || final) {
      const size_t piece = std::min<size_t>(n, final ? n : (size_t)256 << 20);
      const bool last = final && piece == n;
      CIR_HIP(hipEventSynchronize(d.chain_done[k]));  // buffer k free again
      if (piece > d.chain_cap[k]) {
        const double ta = trace_on() ? now_ms() : 0;
        (void)hipHostFree(d.chain_h[k]);
        (void)hipFree(d.chain_d[k]);
        d.chain_h[k] = nullptr;
        d.chain_d[k] = nullptr;
        d.chain_cap[k] = 0;
        const size_t cap = std::max<size_t>(piece, (size_t)4 << 20);
        CIR_HIP(hipHostMalloc(&d.chain_h[k], cap, hipHostMallocDefault));
        CIR_HIP(hipMalloc(&d.chain_d[k], cap));
        d.chain_cap[k] = cap;
        if (trace_on())
          fprintf(stderr, "cir_scan footer buffer %d: %.1f MiB in %.2f ms\n", k,
                  cap / 1048576.0, now_ms() - ta);
      }
      if (piece) {
        memcpy(d.chain_h[k], em.body_at(fed), piece);
        CIR_HIP(hipMemcpyAsync(d.chain_d[k], d.chain_h[k], piece, hipMemcpyHostToDevice, d.chain));
      }
      hipEvent_t e0 = nullptr, e1 = nullptr;
      if (timed) {
        CIR_HIP(hipEventCreate(&e0));
        tev.push_back(e0);
        CIR_HIP(hipEventCreate(&e1));
        tev.push_back(e1);
        CIR_HIP(hipEventRecord(e0, d.chain));
      }
      CIR_HIP(dev::launch_chain_step(d.chain_state, d.chain_d[k], (uint32_t)piece, last, d.chain));
      if (timed) CIR_HIP(hipEventRecord(e1, d.chain));
      CIR_HIP(hipEventRecord(d.chain_done[k], d.chain));
      ++feeds;
      k ^= 1;
      fed += piece;
      n -= piece;
      if (last) break;
    }
    return CIR_OK;
  }

  // feed what is complete, keeping >= 1 byte back; skip tiny feeds
  int advance(const dirsig::Emitter& em, size_t min_feed) {
    const size_t avail = em.body_size() - fed;
    const size_t n = avail > 0 ? (avail - 1) / 128 * 128 : 0;
    if (n < min_feed) return CIR_OK;
    return push(em, n, false);
  }

  int finish(const dirsig::Emitter& em, uint8_t out[32]) {
    int rc = push(em, em.body_size() - fed, true);
    if (rc) return rc;
    CIR_HIP(hipMemcpyAsync(out, d.chain_state, 32, hipMemcpyDeviceToHost, d.chain));
    CIR_HIP(hipStreamSynchronize(d.chain));
    return CIR_OK;
  }
};

// The same footer on one host thread (CIR_FOOTER_HOST, the default): every
// completed stretch of the body is copied out (the emitter's string may grow
// and move) and queued to a thread that feeds it to a streaming BLAKE2b-256
// (blake2b_host.cpp), so hashing the ~106 MB of text of config 5 overlaps the
// scan and the scan's tail after its last batch is the last stretch only.
// Round 4, config 5 on one box (profiles/r04/footer/): see DESIGN.md 5.
class HostFooter {
 public:
  explicit HostFooter(int ht)
      : sha_(ht == CIR_HASH_SHA512_256 ? new host::Sha512_256 : nullptr), th_([this] { run(); }) {}
  ~HostFooter() { close(); }
  size_t fed() const { return fed_; }
  size_t feeds() const { return feeds_; }
  double busy_ms() const { return busy_ms_; }  // valid after finish()

  void advance(const dirsig::Emitter& em, size_t min_feed) {
    const size_t n = em.body_size() - fed_;
    if (n == 0 || n < min_feed) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.emplace_back(em.body_at(fed_), n);
    }
    cv_.notify_one();
    fed_ += n;
    ++feeds_;
  }

  void finish(const dirsig::Emitter& em, uint8_t out[32]) {
    advance(em, 0);
    close();
    if (sha_)
      sha_->final(out);
    else
      st_.final(out);
  }

 private:
  void close() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      closed_ = true;
    }
    cv_.notify_one();
    if (th_.joinable()) th_.join();
  }
  void run() {
    for (;;) {
      std::vector<std::string> take;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return closed_ || !q_.empty(); });
        if (q_.empty()) return;  // closed and drained
        take.swap(q_);
      }
      const double t0 = now_ms();
      for (const std::string& c : take) {
        if (sha_)
          sha_->update((const uint8_t*)c.data(), c.size());
        else
          st_.update((const uint8_t*)c.data(), c.size());
      }
      busy_ms_ += now_ms() - t0;
    }
  }
  host::Blake2b256 st_;
  std::unique_ptr<host::Sha512_256> sha_;  // a sha512/256 index's footer
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::string> q_;
  bool closed_ = false;
  size_t fed_ = 0, feeds_ = 0;
  double busy_ms_ = 0;
  std::thread th_;  // last: started once every other member exists
};

// ---- RawIndex::into_mut + MutableIndex::to_raw_data ---------------------
// (src/cluster/download.rs:171-188 fill_dirs :108-168, emit :266-319)
struct TreeItem;
using Tree = std::map<std::string, TreeItem>;  // BTreeMap<OsString, Item>, bytewise order
struct TreeItem {
  dirsig::EntryKind kind = dirsig::EntryKind::kDir;
  std::unique_ptr<Tree> dir;
  bool exe = false;
  uint64_t size = 0;
  std::vector<uint8_t> hashes;
  std::string target;
};

static void split_path(const std::string& p, std::vector<std::string>* parts) {
  parts->clear();
  size_t i = 0;
  while (i < p.size()) {
    while (i < p.size() && p[i] == '/') ++i;
    size_t j = i;
    while (j < p.size() && p[j] != '/') ++j;
    if (j > i) parts->push_back(p.substr(i, j - i));
    i = j;
  }
}

static void emit_tree(dirsig::Emitter& em, const std::string& path, const Tree& t) {
  if (t.empty()) return;  // the reference skips empty directories (:292-294)
  em.start_dir(path);
  for (const auto& kv : t) {
    const TreeItem& it = kv.second;
    if (it.kind == dirsig::EntryKind::kFile)
      em.add_file(kv.first, it.exe, it.size, it.hashes.data(), it.hashes.size() / 32);
    else if (it.kind == dirsig::EntryKind::kLink)
      em.add_symlink(kv.first, it.target);
  }
  for (const auto& kv : t)
    if (kv.second.kind == dirsig::EntryKind::kDir)
      emit_tree(em, path == "/" ? "/" + kv.first : path + "/" + kv.first, *kv.second.dir);
}

}  // namespace cir

using namespace cir;

// cir_scan_v1 (the index in one malloc'd buffer) and cir_scan_v1_write (the
// index written out to `write` as it is emitted: header first, then each
// stretch of the body after every batch that completes files, the footer
// line last; the emitter keeps only the unwritten tail).
namespace {
struct IndexSink {
  cir_write_fn write;
  void* user;
};
}  // namespace

static int scan_impl(cir_ctx* ctx, const char* const* dirs, const char* const* prefixes,
                     size_t ndirs, uint64_t block_size, int hash_type, uint32_t threads,
                     const IndexSink* sink, uint8_t** index_out, size_t* len_out) {
  if (!ctx || (!sink && (!index_out || !len_out)) || (ndirs && !dirs))
    return fail(CIR_EINVAL, "null pointer");
  if (sink && !sink->write) return fail(CIR_EINVAL, "null index writer");
  if (block_size == 0 || block_size > 0xffffffffull)
    return fail(CIR_EINVAL, "block_size must be in 1 .. 2^32-1");
  dirsig::Header hdr;
  hdr.block_size = block_size;
  if (hash_type == CIR_HASH_BLAKE2B_256)
    hdr.hash = dirsig::HashType::kBlake2b256;
  else if (hash_type == CIR_HASH_SHA512_256)
    hdr.hash = dirsig::HashType::kSha512_256;
  else
    return fail(CIR_EINVAL, "unknown hash type");
  // The footer is hashed incrementally while the scan runs: on a host
  // thread (CIR_FOOTER_HOST, either hash type) or, for blake2b/256, by the
  // GPU chain kernel (CIR_FOOTER_GPU, quad mode); a sha512/256 footer under
  // CIR_FOOTER_GPU is hashed once at the end (one lane).
  const bool host_footer = ctx->footer == CIR_FOOTER_HOST;
  const bool gpu_chain = !host_footer && hash_type == CIR_HASH_BLAKE2B_256;
  if (threads == 0) threads = host_copy_threads(ctx->devs.size());  // auto_threads
  bool stats;
  size_t rows0;  // this scan's batches are the rows recorded from here on
  {
    std::lock_guard<std::mutex> sl(ctx->stats.mu);
    stats = ctx->stats.on;
    rows0 = ctx->stats.batches.size();
  }

  const double t0 = now_ms();
  std::vector<PlanItem> plan;
  std::vector<ScanFile> files;
  for (size_t i = 0; i < ndirs; ++i) {
    std::string pre = prefixes && prefixes[i] ? prefixes[i] : "/";
    if (pre.empty() || pre[0] != '/') pre = "/" + pre;
    while (pre.size() > 1 && pre.back() == '/') pre.pop_back();
    int rc = walk(dirs[i], pre, threads, plan, files);
    if (rc) return rc;
  }
  dirsig::Emitter em(hdr);
  {
    // the body's size, near enough to grow the buffer once: 65 bytes per
    // digest plus each line's name and size (escaping may add a little)
    size_t est = 4096;
    for (const PlanItem& it : plan) {
      est += it.name.size() + it.target.size() + 32;
      if (it.kind == dirsig::EntryKind::kFile)
        est += 65 * ((files[it.file].size + block_size - 1) / block_size);
    }
    // (streamed out: the buffer holds one batch's text at a time)
    if (sink) est = std::min<size_t>(est, (size_t)4 << 20);
    if (!em.reserve_body(est + est / 64)) return fail(CIR_ENOMEM, "index buffer");
  }
  Device& dv = *ctx->devs[0];
  std::unique_lock<std::mutex> chain_lock(dv.chain_mu, std::defer_lock);
  if (gpu_chain) chain_lock.lock();
  DeviceGuard guard;  // the caller's current device is restored on return
  CIR_HIP(hipSetDevice(dv.id));
  FooterChain chain(dv, stats);
  std::unique_ptr<HostFooter> hfoot;
  if (host_footer) hfoot = std::make_unique<HostFooter>(hash_type);
  int rc = gpu_chain ? chain.start() : CIR_OK;
  if (rc) return rc;
  DigestBuf digests;
  size_t plan_pos = 0;
  size_t sunk = 0;  // index bytes handed to the sink
  size_t writes = 0;
  // hand the new index bytes to the sink, then drop from the emitter what
  // both the sink and the footer are done with (the footer feeds hold body
  // offsets: a GPU-chain feed keeps a partial line back)
  auto flush = [&]() -> int {
    if (!sink) return CIR_OK;
    if (em.failed()) return fail(CIR_ENOMEM, "index buffer");
    const size_t end = em.index_size();
    if (end > sunk) {
      if (sink->write(sink->user, em.index_at(sunk), end - sunk) != 0)
        return fail(CIR_EIO, "index writer failed");
      sunk = end;
      ++writes;
    }
    const size_t footer_fed = hfoot ? hfoot->fed() : gpu_chain ? chain.fed : 0;
    em.consume(std::min(sunk, em.header_size() + footer_fed));
    return CIR_OK;
  };
  // emit every plan item whose file blocks are all hashed (files complete in
  // plan order), then feed the finished stretch of the body to the footer
  auto emit_ready = [&](uint64_t done_blk) -> int {
    for (; plan_pos < plan.size(); ++plan_pos) {
      const PlanItem& it = plan[plan_pos];
      if (it.kind == dirsig::EntryKind::kDir) {
        em.start_dir(it.name);
      } else if (it.kind == dirsig::EntryKind::kLink) {
        em.add_symlink(it.name, it.target);
      } else {
        const ScanFile& f = files[it.file];
        const uint64_t nb = (f.size + block_size - 1) / block_size;
        if (f.first_blk + nb > done_blk) break;
        em.add_file(it.name, it.exe, f.size, digests.data() + 32 * f.first_blk, nb);
      }
    }
    if (hfoot) hfoot->advance(em, (size_t)256 << 10);
    const int rc = gpu_chain ? chain.advance(em, (size_t)256 << 10) : (int)CIR_OK;
    return rc ? rc : flush();
  };
  const double t1 = now_ms();
  rc = hash_files(ctx, files, block_size, threads, hash_type, digests, emit_ready,
                  stats ? t0 : -1.0);
  if (rc) return rc;
  const double t2 = now_ms();
  rc = emit_ready(~0ull);
  if (rc) return rc;
  const double t3 = now_ms();
  // Footer = H(every byte after the header line).
  uint8_t footer[32];
  if (hfoot) {
    hfoot->finish(em, footer);
  } else if (gpu_chain) {
    if (em.body_size() - chain.fed > 0xffffffffull)
      return fail(CIR_EINVAL, "index tail above 4 GiB");
    rc = chain.finish(em, footer);
  } else {
    if (em.body_size() > 0xffffffffull) return fail(CIR_EINVAL, "index body longer than 4 GiB");
    const uint64_t off = 0;
    const uint32_t blen = (uint32_t)em.body_size();
    static const uint8_t empty = 0;
    // (nothing of the body was consumed: no footer feed held it)
    rc = cir_hash_blocks_ht(ctx, hash_type,
                            blen ? (const uint8_t*)em.body_at(0) : &empty, &off, &blen, 1, footer);
  }
  if (rc) return rc;
  const double t4 = now_ms();
  size_t total = 0;
  if (sink) {
    if (!em.finish_footer(footer, 32)) return fail(CIR_ENOMEM, "index buffer");
    rc = flush();
    if (rc) return rc;
    total = sunk;
    if (len_out) *len_out = total;
  } else {
    *index_out = em.finish_malloc(footer, 32, &total);
    if (!*index_out) return fail(CIR_ENOMEM, "malloc");
    *len_out = total;
  }
  const double t5 = now_ms();
  if (stats) {
    std::lock_guard<std::mutex> sl(ctx->stats.mu);
    ctx->stats.phases = {t1 - t0,
                         t2 - t1,
                         t3 - t2,
                         t4 - t2,
                         t5 - t4,
                         hfoot ? hfoot->busy_ms() : gpu_chain ? chain.busy_ms() : 0.0,
                         (double)(hfoot ? CIR_FOOTER_HOST : CIR_FOOTER_GPU),
                         (double)(ctx->stats.batches.size() - rows0),
                         (double)total,
                         (double)(hfoot ? hfoot->feeds() : chain.feeds)};
    ++ctx->stats.scans;
  }
  if (trace_on())
    fprintf(stderr,
            "cir_scan phases: walk %.1f ms, hash loop %.1f ms, last emit %.1f ms, footer %.1f ms, "
            "output %.1f ms; %zu files, index %.1f MiB%s\n",
            t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, files.size(), total / 1048576.0,
            sink ? (", written in " + std::to_string(writes) + " pieces").c_str() : "");
  return CIR_OK;
}

extern "C" {

int cir_scan_v1(cir_ctx* ctx, const char* const* dirs, const char* const* prefixes, size_t ndirs,
                uint64_t block_size, int hash_type, uint32_t threads, uint8_t** index_out,
                size_t* len_out) try {
  return scan_impl(ctx, dirs, prefixes, ndirs, block_size, hash_type, threads, nullptr, index_out,
                   len_out);
} CIR_CATCH_BOUNDARY

int cir_scan_v1_write(cir_ctx* ctx, const char* const* dirs, const char* const* prefixes,
                      size_t ndirs, uint64_t block_size, int hash_type, uint32_t threads,
                      cir_write_fn write, void* user, size_t* len_out) try {
  const IndexSink sink{write, user};
  return scan_impl(ctx, dirs, prefixes, ndirs, block_size, hash_type, threads, &sink, nullptr,
                   len_out);
} CIR_CATCH_BOUNDARY

// RawIndex::into_mut + MutableIndex::to_raw_data: parse, rebuild the tree and
// re-emit it in the reference's order with a freshly computed footer.
int cir_index_rewrite(cir_ctx* ctx, const uint8_t* in, size_t len, uint8_t** out, size_t* out_len) try {
  if (!in || !out || !out_len) return fail(CIR_EINVAL, "null pointer");
  dirsig::Index idx;
  std::string err;
  // parsed before the context is needed: a malformed index is a ParseError
  // whatever the device state (RawIndex::into_mut, src/cluster/download.rs:175-181)
  if (!dirsig::parse(in, len, &idx, &err)) return fail(CIR_EPARSE, "ParseError: " + err);
  // fill_dirs (src/cluster/download.rs:108-167) on the host, also before the
  // context is needed: a file and a directory of one name is a PathConflict
  // (:138-140), whatever the device state
  Tree root;
  Tree* cur = &root;
  std::vector<std::string> parts;
  for (dirsig::Entry& e : idx.entries) {
    split_path(e.path, &parts);
    if (e.kind == dirsig::EntryKind::kDir) {
      cur = &root;
      for (const std::string& c : parts) {
        TreeItem& it = (*cur)[c];
        if (!it.dir) {
          if (it.kind != dirsig::EntryKind::kDir)
            return fail(CIR_EPARSE, "The following path conflicts with others: " + e.path);
          it.dir = std::make_unique<Tree>();
        }
        cur = it.dir.get();
      }
      continue;
    }
    if (parts.empty()) return fail(CIR_EPARSE, "Invalid path in index: " + e.path);
    TreeItem it;
    it.kind = e.kind;
    it.exe = e.exe;
    it.size = e.size;
    it.hashes = std::move(e.hashes);
    it.target = std::move(e.target);
    (*cur)[parts.back()] = std::move(it);
  }
  if (!ctx) return fail(CIR_EINVAL, "null ctx");
  dirsig::Emitter em(idx.header);
  emit_tree(em, "/", root);
  if (em.body_size() > 0xffffffffull) return fail(CIR_EINVAL, "index body longer than 4 GiB");
  uint8_t footer[32];
  const uint64_t off = 0;
  const uint32_t blen = (uint32_t)em.body_size();
  static const uint8_t empty = 0;
  const int ht = idx.header.hash == dirsig::HashType::kSha512_256 ? CIR_HASH_SHA512_256
                                                                   : CIR_HASH_BLAKE2B_256;
  int rc = CIR_OK;
  if (ctx->footer == CIR_FOOTER_HOST) {
    // the footer is one serial chain: on the host, as cir_scan_v1 does
    if (ht == CIR_HASH_SHA512_256) {
      host::Sha512_256 h;
      h.update((const uint8_t*)em.body_data(), em.body_size());
      h.final(footer);
    } else {
      host::Blake2b256 h;
      h.update((const uint8_t*)em.body_data(), em.body_size());
      h.final(footer);
    }
  } else {
    rc = cir_hash_blocks_ht(ctx, ht, blen ? (const uint8_t*)em.body_data() : &empty, &off, &blen,
                            1, footer);
  }
  if (rc) return rc;
  *out = em.finish_malloc(footer, 32, out_len);
  if (!*out) return fail(CIR_ENOMEM, "malloc");
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_set_footer_mode(cir_ctx* ctx, int mode) try {
  if (!ctx) return fail(CIR_EINVAL, "null ctx");
  if (mode != CIR_FOOTER_HOST && mode != CIR_FOOTER_GPU) return fail(CIR_EINVAL, "unknown footer mode");
  ctx->footer = mode;
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_debug_scan_timing(cir_ctx* ctx, int enable) try {
  if (!ctx) return fail(CIR_EINVAL, "null ctx");
  std::lock_guard<std::mutex> sl(ctx->stats.mu);
  ctx->stats.on = enable != 0;
  if (enable) {
    ctx->stats.batches.clear();
    ctx->stats.phases.fill(0.0);
    ctx->stats.scans = 0;
  }
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_debug_scan_batches(cir_ctx* ctx, double* rows, size_t max_rows, size_t* nrows) try {
  if (!ctx || !nrows || (max_rows && !rows)) return fail(CIR_EINVAL, "null pointer");
  std::lock_guard<std::mutex> sl(ctx->stats.mu);
  const auto& b = ctx->stats.batches;
  for (size_t i = 0; i < b.size() && i < max_rows; ++i)
    memcpy(rows + i * kScanBatchFields, b[i].data(), sizeof(double) * kScanBatchFields);
  *nrows = b.size();
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_debug_scan_phases(cir_ctx* ctx, double out[CIR_SCAN_PHASE_FIELDS]) try {
  if (!ctx || !out) return fail(CIR_EINVAL, "null pointer");
  std::lock_guard<std::mutex> sl(ctx->stats.mu);
  memcpy(out, ctx->stats.phases.data(), sizeof(double) * kScanPhaseFields);
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_debug_host_blake2b256(const uint8_t* p, size_t n, size_t piece, uint8_t out[32]) try {
  if (!out || (n && !p)) return fail(CIR_EINVAL, "null pointer");
  host::Blake2b256 h;
  if (piece == 0) piece = n;
  for (size_t off = 0; off < n; off += piece) h.update(p + off, std::min(piece, n - off));
  h.final(out);
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_debug_host_sha512_256(const uint8_t* p, size_t n, size_t piece, uint8_t out[32]) try {
  if (!out || (n && !p)) return fail(CIR_EINVAL, "null pointer");
  host::Sha512_256 h;
  if (piece == 0) piece = n;
  for (size_t off = 0; off < n; off += piece) h.update(p + off, std::min(piece, n - off));
  h.final(out);
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_index_get_hash(const uint8_t* index, size_t len, uint8_t* id_out, size_t* id_len) try {
  if (!index || !id_out || !id_len) return fail(CIR_EINVAL, "null pointer");
  std::vector<uint8_t> id;
  std::string err;
  if (!dirsig::get_hash(index, len, &id, &err)) return fail(CIR_EPARSE, err);
  if (id.size() > 64) return fail(CIR_EPARSE, "footer longer than 64 bytes");
  memcpy(id_out, id.data(), id.size());
  *id_len = id.size();
  return CIR_OK;
} CIR_CATCH_BOUNDARY

}  // extern "C"
