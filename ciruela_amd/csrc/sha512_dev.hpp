// SHA-512/256 (FIPS 180-4) device core for gfx950: the second hash type of
// dir-signature indexes (HashType::sha512_256(), header token "sha512/256";
// the reference's own index fixture, src/cluster/download.rs:357-366, uses
// it).  One lane per chain, like the BLAKE2b lane path.
//
// gfx950 forms: rotates on 32-bit halves with v_alignbit_b32, the 3-input
// xors of the Sigma functions and Ch / Maj as v_bitop3_b32, 64-bit adds as
// v_lshl_add_u64, big-endian loads byte-swapped with v_perm_b32.
#pragma once
#include "blake2b_dev.hpp"
#include "sha512_asm.h"

namespace cir {
namespace dev {
namespace sha {

// frac(cbrt(p)) * 2^64 for the first 80 primes (FIPS 180-4 4.2.3)
__constant__ uint64_t kK[80] = {
0x428a2f98d728ae22ULL,
0x7137449123ef65cdULL,
0xb5c0fbcfec4d3b2fULL,
0xe9b5dba58189dbbcULL,
0x3956c25bf348b538ULL,
0x59f111f1b605d019ULL,
0x923f82a4af194f9bULL,
0xab1c5ed5da6d8118ULL,
0xd807aa98a3030242ULL,
0x12835b0145706fbeULL,
0x243185be4ee4b28cULL,
0x550c7dc3d5ffb4e2ULL,
0x72be5d74f27b896fULL,
0x80deb1fe3b1696b1ULL,
0x9bdc06a725c71235ULL,
0xc19bf174cf692694ULL,
0xe49b69c19ef14ad2ULL,
0xefbe4786384f25e3ULL,
0x0fc19dc68b8cd5b5ULL,
0x240ca1cc77ac9c65ULL,
0x2de92c6f592b0275ULL,
0x4a7484aa6ea6e483ULL,
0x5cb0a9dcbd41fbd4ULL,
0x76f988da831153b5ULL,
0x983e5152ee66dfabULL,
0xa831c66d2db43210ULL,
0xb00327c898fb213fULL,
0xbf597fc7beef0ee4ULL,
0xc6e00bf33da88fc2ULL,
0xd5a79147930aa725ULL,
0x06ca6351e003826fULL,
0x142929670a0e6e70ULL,
0x27b70a8546d22ffcULL,
0x2e1b21385c26c926ULL,
0x4d2c6dfc5ac42aedULL,
0x53380d139d95b3dfULL,
0x650a73548baf63deULL,
0x766a0abb3c77b2a8ULL,
0x81c2c92e47edaee6ULL,
0x92722c851482353bULL,
0xa2bfe8a14cf10364ULL,
0xa81a664bbc423001ULL,
0xc24b8b70d0f89791ULL,
0xc76c51a30654be30ULL,
0xd192e819d6ef5218ULL,
0xd69906245565a910ULL,
0xf40e35855771202aULL,
0x106aa07032bbd1b8ULL,
0x19a4c116b8d2d0c8ULL,
0x1e376c085141ab53ULL,
0x2748774cdf8eeb99ULL,
0x34b0bcb5e19b48a8ULL,
0x391c0cb3c5c95a63ULL,
0x4ed8aa4ae3418acbULL,
0x5b9cca4f7763e373ULL,
0x682e6ff3d6b2b8a3ULL,
0x748f82ee5defb2fcULL,
0x78a5636f43172f60ULL,
0x84c87814a1f0ab72ULL,
0x8cc702081a6439ecULL,
0x90befffa23631e28ULL,
0xa4506cebde82bde9ULL,
0xbef9a3f7b2c67915ULL,
0xc67178f2e372532bULL,
0xca273eceea26619cULL,
0xd186b8c721c0c207ULL,
0xeada7dd6cde0eb1eULL,
0xf57d4f7fee6ed178ULL,
0x06f067aa72176fbaULL,
0x0a637dc5a2c898a6ULL,
0x113f9804bef90daeULL,
0x1b710b35131c471bULL,
0x28db77f523047d84ULL,
0x32caab7b40c72493ULL,
0x3c9ebe0a15c9bebcULL,
0x431d67c49c100d4cULL,
0x4cc5d4becb3e42b6ULL,
0x597f299cfc657e2aULL,
0x5fcb6fab3ad6faecULL,
0x6c44198c4a475817ULL};

// SHA-512/256 initial value (FIPS 180-4 5.3.6.2)
constexpr uint64_t kIV[8] = {
0x22312194fc2bf72cULL,
0x9f555fa3c84c64c2ULL,
0x2393b86b6f53b151ULL,
0x963877195940eabdULL,
0x96283ee2a88effe3ULL,
0xbe5e1e2553863992ULL,
0x2b0199fc2c85b8aaULL,
0x0eb72ddc81c52ca2ULL};

template <int F>
__device__ __forceinline__ uint32_t bop3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, F);
}

// rotr(x, N) for 0 < N < 64 on halves
template <int N>
__device__ __forceinline__ uint64_t rotr(uint64_t x) {
  const uint32_t l = lo32(x), h = hi32(x);
  if constexpr (N < 32)
    return mk64(__builtin_amdgcn_alignbit(h, l, N), __builtin_amdgcn_alignbit(l, h, N));
  else if constexpr (N == 32)
    return mk64(h, l);
  else
    return mk64(__builtin_amdgcn_alignbit(l, h, N - 32), __builtin_amdgcn_alignbit(h, l, N - 32));
}
template <int N>
__device__ __forceinline__ uint64_t shr(uint64_t x) {
  const uint32_t l = lo32(x), h = hi32(x);
  return mk64(__builtin_amdgcn_alignbit(h, l, N), h >> N);
}
// x ^ y ^ z and the SHA bit functions, one v_bitop3_b32 per half
__device__ __forceinline__ uint64_t x3(uint64_t x, uint64_t y, uint64_t z) {
  return mk64(bop3<0x96>(lo32(x), lo32(y), lo32(z)), bop3<0x96>(hi32(x), hi32(y), hi32(z)));
}
// Ch(e, f, g) = (e & f) ^ (~e & g): truth table over (e, f, g) = 0xCA
__device__ __forceinline__ uint64_t ch(uint64_t e, uint64_t f, uint64_t g) {
  return mk64(bop3<0xCA>(lo32(e), lo32(f), lo32(g)), bop3<0xCA>(hi32(e), hi32(f), hi32(g)));
}
// Maj(a, b, c): 0xE8
__device__ __forceinline__ uint64_t maj(uint64_t a, uint64_t b, uint64_t c) {
  return mk64(bop3<0xE8>(lo32(a), lo32(b), lo32(c)), bop3<0xE8>(hi32(a), hi32(b), hi32(c)));
}
__device__ __forceinline__ uint64_t bswap64(uint64_t x) {
  return mk64(__builtin_amdgcn_perm(0u, hi32(x), 0x00010203u),
              __builtin_amdgcn_perm(0u, lo32(x), 0x00010203u));
}

// one compression; w = the 16 message words, big-endian decoded
__device__ __forceinline__ void compress(uint64_t h[8], uint64_t w[16]) {
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  // 5 x 16 rounds: the message-schedule indices stay static inside the
  // unrolled 16, and the round constants are scalar loads per pass (a full
  // unroll hoists all 160 constant dwords into SGPRs and spills).
#pragma unroll 1
  for (int t0 = 0; t0 < 80; t0 += 16) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int t = t0 + i;
    if (t0 > 0) {
      const uint64_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint64_t s0 = x3(rotr<1>(w15), rotr<8>(w15), shr<7>(w15));
      const uint64_t s1 = x3(rotr<19>(w2), rotr<61>(w2), shr<6>(w2));
      w[i] = w[i] + s0 + w[(i + 9) & 15] + s1;
    }
    const uint64_t t1 = hh + x3(rotr<14>(e), rotr<18>(e), rotr<41>(e)) + ch(e, f, g) + kK[t] +
                        w[i];
    const uint64_t t2 = x3(rotr<28>(a), rotr<34>(a), rotr<39>(a)) + maj(a, b, c);
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}

// The same compression as hand-scheduled asm (sha512_asm.h, generated by
// tools/gen_sha_asm.py): the state and the 16-word schedule window pinned to
// v[10:57], so renaming a..h between rounds costs nothing, 27 instructions
// per round (46 with the schedule), round constants as SGPR operands.
#ifndef CIR_SHA_ASM
#define CIR_SHA_ASM 1
#endif
__device__ __forceinline__ void compress_asm(uint64_t h[8], uint64_t w[16]) {
  uint64_t S[8], K[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) S[k] = h[k];
#pragma unroll
  for (int k = 0; k < 16; ++k) K[k] = kK[k];
  asm volatile(CIR_SHA_ROUNDS0 : CIR_SHA_STATE_OPS(S), CIR_SHA_W_OPS(w) : CIR_SHA_K_OPS(K)
               : CIR_SHA_CLOBBERS);
#pragma unroll 1
  for (int t0 = 16; t0 < 80; t0 += 16) {
#pragma unroll
    for (int k = 0; k < 16; ++k) K[k] = kK[t0 + k];
    asm volatile(CIR_SHA_ROUNDS1 : CIR_SHA_STATE_OPS(S), CIR_SHA_W_OPS(w) : CIR_SHA_K_OPS(K)
                 : CIR_SHA_CLOBBERS);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] += S[k];
}

// Little-endian bytes of a padded block: the first n (0..128) message bytes,
// 0x80 at byte n when pad80, zeros elsewhere.  Never reads past p + n.
__device__ __forceinline__ void load_block_padded(uint64_t m[16], const uint8_t* p, uint32_t n,
                                                  bool pad80) {
  const bool al4 = (reinterpret_cast<uintptr_t>(p) & 3u) == 0;
#pragma unroll
  for (int wd = 0; wd < 32; ++wd) {
    uint32_t x = 0;
    const uint32_t b0 = 4u * wd;
    if (al4 && b0 + 4u <= n) {
      x = *reinterpret_cast<const uint32_t*>(p + b0);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (b0 + k < n) x |= (uint32_t)p[b0 + k] << (8 * k);
        else if (pad80 && b0 + k == n) x |= 0x80u << (8 * k);
      }
    }
    if (wd & 1)
      m[wd >> 1] |= (uint64_t)x << 32;
    else
      m[wd >> 1] = x;
  }
}

// SHA-512/256 of [p, p + len) into h (digest = big-endian h[0..3]).
// Blocks: ceil((len + 17) / 128); 0x80 after the message, the 128-bit
// big-endian bit length in the last 16 bytes.
__device__ __forceinline__ void chain(const uint8_t* p, uint64_t len, uint64_t h[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = kIV[k];
  const uint64_t nblk = (len + 17 + 127) / 128;
  const bool al16 = (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  // Block pad_blk holds the tail bytes and the 0x80; blocks before it are
  // full, a block after it (len % 128 >= 112) carries only the length.
  // (Classifying blocks by comparing start with len was miscompiled for
  // the length-only block: the 0x80 landed in it too.)
  const uint64_t pad_blk = len >> 7;
  const uint32_t tail = (uint32_t)(len & 127u);
  for (uint64_t bi = 0; bi < nblk; ++bi) {
    uint64_t m[16];
    const uint8_t* q = p + (bi << 7);
    if (bi < pad_blk) {
      if (al16)
        load_line16(m, q);
      else
        load_block_padded(m, q, 128u, false);
    } else if (bi == pad_blk) {
      // opaque here: the 128 byte-position compares against the tail length
      // must not be hoisted out of the block loop (they would live in SGPR
      // masks and spill)
      uint32_t tn = tail;
      asm volatile("" : "+v"(tn));
      load_block_padded(m, q, tn, true);
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) m[k] = 0;
    }
    // big-endian words in place (the schedule reuses the same 16 registers)
#pragma unroll
    for (int k = 0; k < 16; ++k) m[k] = bswap64(m[k]);
    if (bi + 1 == nblk) {
      m[14] = len >> 61;
      m[15] = len << 3;
    }
#if CIR_SHA_ASM
    compress_asm(h, m);
#else
    compress(h, m);
#endif
  }
}

__device__ __forceinline__ void store_digest_be(uint8_t* out, const uint64_t h[8]) {
  uint4* o = reinterpret_cast<uint4*>(out);
  const uint64_t a = bswap64(h[0]), b = bswap64(h[1]), c = bswap64(h[2]), d = bswap64(h[3]);
  o[0] = make_uint4(lo32(a), hi32(a), lo32(b), hi32(b));
  o[1] = make_uint4(lo32(c), hi32(c), lo32(d), hi32(d));
}

}  // namespace sha
}  // namespace dev
}  // namespace cir
