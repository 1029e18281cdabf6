// ciruela-index: the indexing half of `ciruela sync`, on the GPU path.
//
// Reference: `ciruela sync` (src/client/main.rs:94-99 -> src/client/sync/
// mod.rs:168-220 -> uploads::prepare, src/client/sync/uploads.rs:61-105).
// For every --append / --append-weak / --replace SRC:DEST it runs the scan
// (uploads.rs:49-59, threads = --disk-threads), registers the
// index (InMemoryIndexes::register_index -> ImageId) and prints
//   <image id> <kind> <dest> <src>
// Signing and the upload itself (networking, src/client/sync/network.rs) are
// out of scope; --index-dir writes each index as
// <dir>/<image id>.ds1 so a separate uploader can pick it up.
//
//   ciruela-index sync [--disk-threads N] [--block-size N] [--index-dir D]
//                      --append SRC:/DEST [--append-weak SRC:/DEST]
//                      [--replace SRC:/DEST[:OLD_IMAGE_ID]] ...
//   ciruela-index hash [--block-size N] FILE...   (per-block BlockHash list)
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "ciruela_blockhash.h"

static void usage() {
  fprintf(stderr,
          "usage: ciruela-index sync [--disk-threads N] [--block-size N] [--index-dir D]\n"
          "                          (--append|--append-weak|--replace) SRC:/DEST ...\n"
          "       ciruela-index hash [--block-size N] FILE...\n");
}

static std::string hex(const uint8_t* p, size_t n) {
  static const char k[] = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; ++i) {
    s += k[p[i] >> 4];
    s += k[p[i] & 15];
  }
  return s;
}

static int die(int rc, const char* what) {
  fprintf(stderr, "%s: %s: %s\n", what, cir_strerror(rc), cir_last_error());
  return rc == CIR_EIO ? 1 : 2;
}

// Bytes of the regular files under path, counted only until they reach cap.
// The top-level argument is followed as the scan and the hash path follow it
// (open): a symlinked SRC or FILE counts its target; entries inside
// directories are not followed (fstatat AT_SYMLINK_NOFOLLOW), as the scan's
// walk does, and each directory is read through its own fd opened from its
// parent's (openat), so a tree nested past PATH_MAX is counted too.  A
// top-level argument that is neither a regular file nor a directory (a pipe,
// /dev/stdin) has no size to count and gets the default staging (returns cap).
static uint64_t dir_bytes(int dfd, uint64_t cap, uint64_t acc) {
  const int lfd = fcntl(dfd, F_DUPFD_CLOEXEC, 0);
  DIR* d = lfd >= 0 ? fdopendir(lfd) : nullptr;
  if (!d) {
    if (lfd >= 0) close(lfd);
    return acc;
  }
  while (struct dirent* e = readdir(d)) {
    if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
    struct stat st;
    if (fstatat(dfd, e->d_name, &st, AT_SYMLINK_NOFOLLOW) != 0) continue;
    if (S_ISREG(st.st_mode)) {
      acc += (uint64_t)st.st_size;
    } else if (S_ISDIR(st.st_mode)) {
      const int cfd = openat(dfd, e->d_name, O_RDONLY | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC);
      if (cfd >= 0) {
        acc = dir_bytes(cfd, cap, acc);
        close(cfd);
      }
    }
    if (acc >= cap) break;
  }
  closedir(d);
  return acc;
}

static uint64_t tree_bytes(const std::string& path, uint64_t cap, uint64_t acc) {
  struct stat st;
  if (acc >= cap) return acc;
  if (stat(path.c_str(), &st) != 0) return cap;
  if (S_ISREG(st.st_mode)) return acc + (uint64_t)st.st_size;
  if (!S_ISDIR(st.st_mode)) return cap;
  const int fd = open(path.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  if (fd < 0) return acc;
  acc = dir_bytes(fd, cap, acc);
  close(fd);
  return acc;
}

// Bytes of every input, counted up to what decides the device count: two
// default staging slots per device for 32 devices (cir_devices_for_bytes).
static uint64_t input_bytes(const std::vector<std::string>& paths) {
  constexpr uint64_t kCap = 32 * 2 * (256ull << 20);
  uint64_t total = 0;
  for (const std::string& p : paths) total = tree_bytes(p, kCap, total);
  return total;
}

// Staging per slot: the library default (256 MiB) for large inputs; a small
// input gets slots just big enough to hold it, so a one-shot `sync` of a few
// MiB does not pin 3 x 256 MiB of host memory it never fills (cir_init
// allocates the slots up front).
static uint64_t staging_for(uint64_t total) {
  constexpr uint64_t kMax = 256ull << 20, kMin = 1ull << 20;
  if (total >= kMax) return 0;
  return std::max<uint64_t>(kMin, (total + kMin - 1) / kMin * kMin);
}

// A profiling tool library loaded into this process (rocprofv3's
// environment), which writes its output from the exit handlers.
static bool profiled() {
  extern char** environ;
  for (char** e = environ; e && *e; ++e)
    if (!strncmp(*e, "ROCP_TOOL_LIBRARIES=", 20) || !strncmp(*e, "ROCPROF", 7)) return true;
  return false;
}

struct Job {
  std::string kind, src, dest;
};

// split "source:/dir/dest" (src/client/sync/uploads.rs:25-33)
static bool split(const std::string& cli, std::string* src, std::string* dest) {
  const size_t c = cli.find(':');
  if (c == std::string::npos) return false;
  *src = cli.substr(0, c);
  std::string rest = cli.substr(c + 1);
  const size_t c2 = rest.find(':');
  *dest = c2 == std::string::npos ? rest : rest.substr(0, c2);
  return !dest->empty() && (*dest)[0] == '/';
}

int main(int argc, char** argv) {
  if (argc < 2) {
    usage();
    return 2;
  }
  const std::string cmd = argv[1];
  // --disk-threads N is GlobalOptions.threads (src/client/global_options.rs:13,
  // default 4), the reference's CPU hashing pool.  Here the host threads
  // only read files into the staging buffers, and 4 readers hold a large
  // tree to ~22 GiB/s, so without the flag the library picks
  // its reader count (0: min(12, 3/4 of the CPU share)); given, N is used.
  uint32_t threads = 0;
  uint64_t bs = CIR_DEFAULT_BLOCK_SIZE;
  std::string index_dir;
  std::vector<Job> jobs;
  std::vector<std::string> files;
  for (int i = 2; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) {
        usage();
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--disk-threads" || a == "--block-size") {
      // a decimal count (clap's usize parse in the reference): anything else
      // is a usage error, not an exception out of main
      const std::string v = val();
      char* end = nullptr;
      errno = 0;
      const unsigned long long n = strtoull(v.c_str(), &end, 10);
      if (v.empty() || v[0] == '-' || *end || errno ||
          (a == "--disk-threads" && n > 0xffffffffull)) {
        fprintf(stderr, "invalid value for %s: %s\n", a.c_str(), v.c_str());
        return 2;
      }
      if (a == "--disk-threads")
        threads = (uint32_t)n;
      else
        bs = n;
    }
    else if (a == "--index-dir") index_dir = val();
    else if (a == "--append" || a == "--append-weak" || a == "--replace") {
      Job j;
      j.kind = a.substr(2);
      if (!split(val(), &j.src, &j.dest)) {
        fprintf(stderr, "Destination directory is invalid, must be `source:/dir/dest`\n");
        return 2;
      }
      jobs.push_back(j);
    } else if (cmd == "hash" && a.size() && a[0] != '-') {
      files.push_back(a);
    } else {
      usage();
      return 2;
    }
  }
  std::vector<std::string> inputs = files;
  for (const Job& j : jobs) inputs.push_back(j.src);
  cir_ctx* ctx = nullptr;
  const uint64_t total = input_bytes(inputs);
  const uint64_t staging = staging_for(total);
  const char* tv = getenv("CIR_TRACE");
  const bool trace = tv && *tv && strcmp(tv, "0") != 0;
  // An input below one staging slot is one small batch: its copies go
  // through the runtime's blit kernels instead of the SDMA engines, whose
  // first use in a process costs ~16-17 ms (cir_init's first uploads) -- a
  // tenth of a one-shot `sync` of config 1's 10 MiB tree
  // (profiles/r05/cli_sdma_ab.log).  Large inputs keep SDMA (the link's full
  // rate); a caller's own HSA_ENABLE_SDMA wins.  Set before the first HIP
  // call, when the runtime reads it.
  const bool small = staging != 0;
  if (small && !getenv("HSA_ENABLE_SDMA")) setenv("HSA_ENABLE_SDMA", "0", 0);
  auto ms_since = [](std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
  };
  if (trace) {
    fprintf(stderr, "ciruela-index: staging %llu bytes per slot (0 = library default), %s copies\n",
            (unsigned long long)staging,
            strcmp(getenv("HSA_ENABLE_SDMA") ? getenv("HSA_ENABLE_SDMA") : "1", "0") == 0
                ? "blit" : "SDMA");
    // the HIP runtime's own start-up (device discovery), apart from cir_init
    const auto t0 = std::chrono::steady_clock::now();
    const int n = cir_device_count();
    fprintf(stderr, "ciruela-index: HIP runtime start %.1f ms (%d devices)\n", ms_since(t0), n);
  }
  // open only the GPUs the input can use: one per two staging batches of it
  // (cir_devices_for_bytes), the lowest-numbered first -- a tree below one
  // slot (256 MiB) is one batch on one GPU -- instead of every GPU of the
  // node (each costs its device context, streams and 834 MiB of pinned
  // staging at start-up, include/ciruela_blockhash.h)
  // (an empty input -- empty files, an empty tree -- is measured, not
  // unknown: one device, not cir_devices_for_bytes' "0 = every device")
  const uint32_t ndev = cir_devices_for_bytes(std::max<uint64_t>(total, 1), staging, 32);
  const auto t_init = std::chrono::steady_clock::now();
  // and a small input is one short job: one stream and one slot per device
  // (CIR_INIT_ONE_SHOT; the other streams' hardware queues were ~25 ms of
  // cir_init, profiles/r05/start_env.log)
  int rc = cir_init_n(&ctx, 0, staging, ndev, small ? CIR_INIT_ONE_SHOT : 0u);
  if (rc) return die(rc, "cir_init");
  if (trace) {
    int ids[64];
    const int opened = cir_ctx_devices(ctx, ids, 64);
    fprintf(stderr, "ciruela-index: cir_init %.1f ms, %d device(s) for %llu input bytes\n",
            ms_since(t_init), opened, (unsigned long long)total);
  }
  if (cmd == "hash") {
    for (const std::string& f : files) {
      const int fd = open(f.c_str(), O_RDONLY);
      if (fd < 0) {
        perror(f.c_str());
        return 1;
      }
      uint64_t size = 0;
      uint8_t* h = nullptr;
      size_t n = 0;
      rc = cir_hash_file(ctx, fd, bs, &size, &h, &n);
      close(fd);
      if (rc) return die(rc, f.c_str());
      printf("%s %llu", f.c_str(), (unsigned long long)size);
      for (size_t k = 0; k < n; ++k) printf(" %s", hex(h + 32 * k, 32).c_str());
      printf("\n");
      cir_free(h);
    }
  } else if (cmd == "sync") {
    if (jobs.empty()) {
      usage();
      return 2;
    }
    cir_indexes* idx = cir_indexes_new();
    cir_blocks* blocks = cir_blocks_new();
    for (const Job& j : jobs) {
      const auto t0 = std::chrono::steady_clock::now();
      const char* dirs[1] = {j.src.c_str()};
      const char* pre[1] = {"/"};
      uint8_t* index = nullptr;
      size_t len = 0;
      rc = cir_scan_v1(ctx, dirs, pre, 1, bs, CIR_HASH_BLAKE2B_256, threads, &index, &len);
      if (rc) return die(rc, ("error indexing dir " + j.src).c_str());
      uint8_t id[64];
      size_t idl = 0;
      rc = cir_indexes_register(idx, index, len, id, &idl);
      if (rc) return die(rc, "register_index");
      rc = cir_blocks_register_dir(blocks, j.src.c_str(), index, len);
      if (rc) return die(rc, "register_dir");
      const double s =
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      printf("%s %s %s %s\n", hex(id, idl).c_str(), j.kind.c_str(), j.dest.c_str(),
             j.src.c_str());
      fprintf(stderr, "Indexed %s (%zu index bytes, %zu blocks) in %.3f s\n", j.src.c_str(), len,
              cir_blocks_len(blocks), s);
      if (!index_dir.empty()) {
        const std::string p = index_dir + "/" + hex(id, idl) + ".ds1";
        FILE* f = fopen(p.c_str(), "wb");
        // (a full disk can surface only at fclose, when the buffer is written)
        const bool ok = f && fwrite(index, 1, len, f) == len;
        if (!ok || (f && fclose(f) != 0)) {
          perror(p.c_str());
          if (!ok && f) fclose(f);
          return 1;
        }
      }
      cir_free(index);
    }
    cir_blocks_free(blocks);
    cir_indexes_free(idx);
  } else {
    usage();
    return 2;
  }
  // A one-shot process: every result is written and every GPU call has
  // completed (the scan synchronises before it returns), so the context's
  // teardown -- freeing the pinned staging, streams and device buffers one by
  // one, ~17 ms of a ~0.2 s run (profiles/r04/cli_startup.log) -- is left to
  // process exit, as the error paths above already do.  CIR_CLI_TEARDOWN=1
  // destroys the context first (leak checks).  Under a profiler (rocprofv3
  // sets ROCP_TOOL_LIBRARIES / ROCPROF_* for its tool library) the process
  // still skips cir_destroy but returns normally, so the exit handlers run
  // and the tool writes its trace at finalisation.
  const char* td = getenv("CIR_CLI_TEARDOWN");
  if (!(td && *td && strcmp(td, "0") != 0)) {
    if (fflush(stdout) != 0) {
      perror("stdout");
      return 1;
    }
    if (profiled()) {
      if (trace) fprintf(stderr, "ciruela-index: profiler present: normal exit, no cir_destroy\n");
      return 0;
    }
    if (trace) fprintf(stderr, "ciruela-index: exit without cir_destroy\n");
    fflush(stderr);
    _exit(0);
  }
  const auto t_destroy = std::chrono::steady_clock::now();
  cir_destroy(ctx);
  if (trace) fprintf(stderr, "ciruela-index: cir_destroy %.1f ms\n", ms_since(t_destroy));
  return 0;
}
