// The DIRSIGNATURE.v1 emitter's streaming form (dirsig.cpp Emitter::consume,
// as cir_scan_v1_write drives it) under AddressSanitizer + UBSan: random
// directory / file / symlink entries (names needing escapes, files of 0..n
// digests) are emitted twice -- once whole (finish_malloc), once written out
// in random pieces with the written and footer-fed prefix consumed, a
// simulated footer feed lagging behind by random amounts -- and the written
// bytes must equal the whole index, the footer feed the body.
//   emitter_stream_fuzz CASES SEED
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "dirsig.hpp"

using cir::dirsig::Emitter;
using cir::dirsig::Header;
using cir::dirsig::HashType;

static std::string rand_name(std::mt19937_64& rng) {
  static const char* parts[] = {"a", "b c", "d\\e", "\t", "\xc3\xbc", "x.bin", ".h", "9", "\x7f"};
  std::string s;
  const int n = 1 + (int)(rng() % 4);
  for (int i = 0; i < n; ++i) s += parts[rng() % 9];
  return s;
}

static bool one_case(std::mt19937_64& rng) {
  Header h;
  h.hash = rng() % 2 ? HashType::kBlake2b256 : HashType::kSha512_256;
  h.block_size = 1 + rng() % 65536;
  Emitter whole(h), stream(h);
  if (rng() % 2) stream.reserve_body(rng() % 4096);
  std::string written, fed;
  size_t sunk = 0, footer_fed = 0;
  const size_t min_feed = rng() % 3 == 0 ? 0 : 1 + rng() % 2000;
  auto flush = [&](bool all) {
    const size_t end = stream.index_size();
    if (end > sunk) {
      written.append((const char*)stream.index_at(sunk), end - sunk);
      sunk = end;
    }
    // the footer takes what is complete, sometimes holding some back
    const size_t avail = stream.body_size() - footer_fed;
    size_t take = all ? avail : (avail >= min_feed ? avail - (rng() % 3 ? 0 : avail / 2) : 0);
    fed.append(stream.body_at(footer_fed), take);
    footer_fed += take;
    const size_t upto = std::min(sunk, stream.header_size() + footer_fed);
    if (upto < stream.consumed()) return false;
    stream.consume(upto);
    return true;
  };
  std::vector<uint8_t> digests;
  const int ops = (int)(rng() % 200);
  for (int i = 0; i < ops; ++i) {
    const int kind = (int)(rng() % 10);
    if (kind == 0) {
      const std::string d = "/" + rand_name(rng);
      whole.start_dir(d);
      stream.start_dir(d);
    } else if (kind == 1) {
      const std::string n = rand_name(rng), t = rand_name(rng);
      whole.add_symlink(n, t);
      stream.add_symlink(n, t);
    } else {
      const size_t nh = rng() % 5 == 0 ? rng() % 3000 : rng() % 8;
      digests.resize(32 * nh + 1);
      for (auto& b : digests) b = (uint8_t)rng();
      const std::string n = rand_name(rng);
      const bool exe = rng() % 4 == 0;
      const uint64_t size = rng() % (1ull << 40);
      whole.add_file(n, exe, size, digests.data(), nh);
      stream.add_file(n, exe, size, digests.data(), nh);
    }
    if (rng() % 3 == 0 && !flush(false)) return false;
  }
  if (!flush(true)) return false;
  uint8_t footer[32];
  for (auto& b : footer) b = (uint8_t)rng();
  if (!stream.finish_footer(footer, 32)) return false;
  if (!flush(true)) return false;
  size_t len = 0;
  uint8_t* ref = whole.finish_malloc(footer, 32, &len);
  if (!ref) return false;
  const std::string want((const char*)ref, len);
  free(ref);
  const size_t hl = whole.header_line().size();
  const size_t fl = 65;  // 64 hex digits + newline
  bool ok = written == want && len >= hl + fl && fed.size() >= fl &&
            fed.compare(0, fed.size() - fl, want, hl, len - hl - fl) == 0;
  // a consumed emitter no longer hands its buffer over
  size_t l2 = 0;
  if (stream.consumed() > 0 && stream.finish_malloc(footer, 32, &l2) != nullptr) ok = false;
  return ok;
}

int main(int argc, char** argv) {
  const int cases = argc > 1 ? atoi(argv[1]) : 200;
  std::mt19937_64 rng(argc > 2 ? strtoull(argv[2], nullptr, 10) : 1);
  for (int c = 0; c < cases; ++c)
    if (!one_case(rng)) {
      printf("case %d: streamed index differs\n", c);
      return 1;
    }
  printf("%d cases ok; no sanitizer report\n", cases);
  return 0;
}
