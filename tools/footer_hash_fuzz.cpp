// The footer's host hashers (blake2b_host.cpp, sha512_host.cpp) under
// AddressSanitizer + UBSan: random inputs fed in random piece sizes must give
// the digest of a one-shot feed; then the digests of stdin (fed in `piece`
// bytes, argv[2]) are printed for the test to compare with hashlib.
//   footer_hash_fuzz CASES PIECE < data
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "blake2b_host.hpp"
#include "sha512_host.hpp"

using cir::host::Blake2b256;
using cir::host::Sha512_256;

template <class H>
static void digest(const uint8_t* p, size_t n, size_t piece, uint8_t out[32]) {
  H h;
  if (piece == 0) piece = n ? n : 1;
  for (size_t off = 0; off < n; off += piece) h.update(p + off, n - off < piece ? n - off : piece);
  h.final(out);
}

template <class H>
static bool check(std::mt19937_64& rng, const std::vector<uint8_t>& d) {
  uint8_t one[32], cut[32];
  digest<H>(d.data(), d.size(), 0, one);
  H h;
  size_t off = 0;
  while (off < d.size()) {  // random piece sizes, zero-length updates included
    const size_t k = std::min<size_t>(d.size() - off, rng() % 300);
    h.update(d.data() + off, k);
    off += k;
  }
  h.final(cut);
  return memcmp(one, cut, 32) == 0;
}

int main(int argc, char** argv) {
  const int cases = argc > 1 ? atoi(argv[1]) : 1000;
  const size_t piece = argc > 2 ? (size_t)atoll(argv[2]) : 0;
  std::mt19937_64 rng(7);
  for (int c = 0; c < cases; ++c) {
    std::vector<uint8_t> d(rng() % 1100);
    for (auto& b : d) b = (uint8_t)rng();
    if (!check<Blake2b256>(rng, d) || !check<Sha512_256>(rng, d)) {
      printf("MISMATCH case %d (%zu bytes)\n", c, d.size());
      return 1;
    }
  }
  std::vector<uint8_t> in;
  uint8_t buf[65536];
  size_t r;
  while ((r = fread(buf, 1, sizeof buf, stdin)) > 0) in.insert(in.end(), buf, buf + r);
  uint8_t b2[32], sh[32];
  digest<Blake2b256>(in.data(), in.size(), piece, b2);
  digest<Sha512_256>(in.data(), in.size(), piece, sh);
  for (uint8_t x : b2) printf("%02x", x);
  printf(" ");
  for (uint8_t x : sh) printf("%02x", x);
  printf("\nno sanitizer report\n");
  return 0;
}
