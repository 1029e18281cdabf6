// Streaming SHA-512/256 (FIPS 180-4) on one host thread: the index footer
// of a sha512/256 scan or rewrite.  See sha512_host.hpp.
#include "sha512_host.hpp"

#include <string.h>

namespace cir {
namespace host {

namespace {

// frac(cbrt(p)) * 2^64 for the first 80 primes (FIPS 180-4 4.2.3)
constexpr uint64_t kK[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull,
};

// SHA-512/256 initial value (FIPS 180-4 5.3.6.2)
constexpr uint64_t kIV[8] = {0x22312194fc2bf72cull, 0x9f555fa3c84c64c2ull, 0x2393b86b6f53b151ull,
                             0x963877195940eabdull, 0x96283ee2a88effe3ull, 0xbe5e1e2553863992ull,
                             0x2b0199fc2c85b8aaull, 0x0eb72ddc81c52ca2ull};

inline uint64_t ror(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

inline uint64_t load_be(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return __builtin_bswap64(v);
}

}  // namespace

Sha512_256::Sha512_256() {
  for (int i = 0; i < 8; ++i) h_[i] = kIV[i];
}

void Sha512_256::compress(const uint8_t* block) {
  uint64_t w[80];
  for (int t = 0; t < 16; ++t) w[t] = load_be(block + 8 * t);
  for (int t = 16; t < 80; ++t) {
    const uint64_t s0 = ror(w[t - 15], 1) ^ ror(w[t - 15], 8) ^ (w[t - 15] >> 7);
    const uint64_t s1 = ror(w[t - 2], 19) ^ ror(w[t - 2], 61) ^ (w[t - 2] >> 6);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint64_t a = h_[0], b = h_[1], c = h_[2], d = h_[3], e = h_[4], f = h_[5], g = h_[6],
           h = h_[7];
  for (int t = 0; t < 80; ++t) {
    const uint64_t S1 = ror(e, 14) ^ ror(e, 18) ^ ror(e, 41);
    const uint64_t ch = (e & f) ^ (~e & g);
    const uint64_t t1 = h + S1 + ch + kK[t] + w[t];
    const uint64_t S0 = ror(a, 28) ^ ror(a, 34) ^ ror(a, 39);
    const uint64_t maj = (a & b) ^ (a & c) ^ (b & c);
    const uint64_t t2 = S0 + maj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h_[0] += a;
  h_[1] += b;
  h_[2] += c;
  h_[3] += d;
  h_[4] += e;
  h_[5] += f;
  h_[6] += g;
  h_[7] += h;
}

void Sha512_256::update(const uint8_t* p, size_t n) {
  len_ += n;
  if (buflen_ > 0) {
    const size_t k = n < 128 - buflen_ ? n : 128 - buflen_;
    memcpy(buf_ + buflen_, p, k);
    buflen_ += k;
    p += k;
    n -= k;
    if (buflen_ < 128) return;
    compress(buf_);
    buflen_ = 0;
  }
  for (; n >= 128; p += 128, n -= 128) compress(p);
  memcpy(buf_, p, n);
  buflen_ = n;
}

void Sha512_256::final(uint8_t out[32]) {
  // 0x80, zeros, then the 128-bit big-endian bit length (the high half 0)
  const uint64_t bits = len_ << 3;
  buf_[buflen_++] = 0x80;
  if (buflen_ > 112) {
    memset(buf_ + buflen_, 0, 128 - buflen_);
    compress(buf_);
    buflen_ = 0;
  }
  memset(buf_ + buflen_, 0, 120 - buflen_);
  const uint64_t be = __builtin_bswap64(bits);
  memcpy(buf_ + 120, &be, 8);
  compress(buf_);
  for (int i = 0; i < 4; ++i) {
    const uint64_t be_h = __builtin_bswap64(h_[i]);
    memcpy(out + 8 * i, &be_h, 8);
  }
}

}  // namespace host
}  // namespace cir
