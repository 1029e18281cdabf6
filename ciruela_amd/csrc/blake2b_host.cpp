// Streaming BLAKE2b-256 on one host thread (the index footer): see
// blake2b_host.hpp for why the footer, and only the footer, runs here.
#include "blake2b_host.hpp"

#include <string.h>

namespace cir {
namespace host {

namespace {

// RFC 7693 2.6 (IV) and 2.7 (message schedule); rounds 10 and 11 reuse rows
// 0 and 1.
constexpr uint64_t kIV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                             0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                             0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
constexpr uint8_t kSigma[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

inline uint64_t ror(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

inline void g(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, uint64_t x, uint64_t y) {
  a += b + x;
  d = ror(d ^ a, 32);
  c += d;
  b = ror(b ^ c, 24);
  a += b + y;
  d = ror(d ^ a, 16);
  c += d;
  b = ror(b ^ c, 63);
}

// One round: four column G, then four diagonal G (RFC 7693 3.2).
template <int R>
inline void round(uint64_t v[16], const uint64_t m[16]) {
  constexpr const uint8_t* s = kSigma[R % 10];
  g(v[0], v[4], v[8], v[12], m[s[0]], m[s[1]]);
  g(v[1], v[5], v[9], v[13], m[s[2]], m[s[3]]);
  g(v[2], v[6], v[10], v[14], m[s[4]], m[s[5]]);
  g(v[3], v[7], v[11], v[15], m[s[6]], m[s[7]]);
  g(v[0], v[5], v[10], v[15], m[s[8]], m[s[9]]);
  g(v[1], v[6], v[11], v[12], m[s[10]], m[s[11]]);
  g(v[2], v[7], v[8], v[13], m[s[12]], m[s[13]]);
  g(v[3], v[4], v[9], v[14], m[s[14]], m[s[15]]);
}

}  // namespace

Blake2b256::Blake2b256() {
  for (int i = 0; i < 8; ++i) h_[i] = kIV[i];
  h_[0] ^= 0x01010000ull ^ 32u;  // depth 1, fanout 1, no key, nn = 32
}

void Blake2b256::compress(const uint8_t* block, bool last) {
  uint64_t m[16], v[16];
  memcpy(m, block, 128);  // little-endian host (x86-64)
  for (int i = 0; i < 8; ++i) {
    v[i] = h_[i];
    v[i + 8] = kIV[i];
  }
  v[12] ^= t_;  // the high counter word stays 0 below 2^64 bytes
  if (last) v[14] = ~v[14];
  round<0>(v, m);
  round<1>(v, m);
  round<2>(v, m);
  round<3>(v, m);
  round<4>(v, m);
  round<5>(v, m);
  round<6>(v, m);
  round<7>(v, m);
  round<8>(v, m);
  round<9>(v, m);
  round<10>(v, m);
  round<11>(v, m);
  for (int i = 0; i < 8; ++i) h_[i] ^= v[i] ^ v[i + 8];
}

void Blake2b256::update(const uint8_t* p, size_t n) {
  if (n == 0) return;
  // top up a held-back block; compress it only once more input follows
  if (buflen_ > 0) {
    const size_t k = n < 128 - buflen_ ? n : 128 - buflen_;
    memcpy(buf_ + buflen_, p, k);
    buflen_ += k;
    p += k;
    n -= k;
    if (n == 0) return;
    t_ += 128;
    compress(buf_, false);
    buflen_ = 0;
  }
  // whole blocks straight from the input, the last one held back
  while (n > 128) {
    t_ += 128;
    compress(p, false);
    p += 128;
    n -= 128;
  }
  memcpy(buf_, p, n);
  buflen_ = n;
}

void Blake2b256::final(uint8_t out[32]) {
  // the empty input is one all-zero block with t = 0 (RFC 7693 3.3)
  memset(buf_ + buflen_, 0, 128 - buflen_);
  t_ += buflen_;
  compress(buf_, true);
  memcpy(out, h_, 32);
}

}  // namespace host
}  // namespace cir
