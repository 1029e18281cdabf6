// BLAKE2b compression variants kept for the micro-benchmarks only
// (tools/valu_ubench.hip): the G-at-a-time order the compiler picks
// (compress_v, with the rotate instruction form selectable) and two chains
// interleaved per lane (compress2, ILP 8).  The product uses compress_sm
// (ciruela_amd/csrc/blake2b_dev.hpp); these measured 4 % slower
// register-only (profiles/r01/order_ubench.log, valu_ubench*.log).
#pragma once
#include "blake2b_dev.hpp"

namespace cir {
namespace dev {

// rotr64(a ^ b, N) on 32-bit halves.  MODE selects the instruction form
// (gfx950 issue costs measured by tools/valu_ubench.hip, profiles/):
//   MODE 0: v_alignbit_b32 x2            (any N)
//   MODE 1: v_perm_b32 x2                (N = 16, 24: byte rotates)
//   MODE 2: (x << 1) + (x >> 63) as one v_lshl_add_u64 + v_lshrrev_b32 (N = 63)
template <int N, int MODE>
__device__ __forceinline__ uint64_t xor_rotr(uint64_t a, uint64_t b) {
  const uint32_t l = lo32(a) ^ lo32(b), h = hi32(a) ^ hi32(b);
  if constexpr (N == 32) {
    return mk64(h, l);
  } else if constexpr (MODE == 1 && (N == 16 || N == 24)) {
    // bytes of {S0, S1} numbered S1 = 0..3, S0 = 4..7; result byte k = sel[k]
    constexpr uint32_t sel = N == 16 ? 0x05040302u : 0x06050403u;
    return mk64(__builtin_amdgcn_perm(h, l, sel), __builtin_amdgcn_perm(l, h, sel));
  } else if constexpr (MODE == 2 && N == 63) {
    const uint64_t x = mk64(l, h);
    return (x << 1) + (uint64_t)(h >> 31);
  } else if constexpr (N < 32) {
    return mk64(__builtin_amdgcn_alignbit(h, l, N), __builtin_amdgcn_alignbit(l, h, N));
  } else {
    return mk64(__builtin_amdgcn_alignbit(l, h, N - 32), __builtin_amdgcn_alignbit(h, l, N - 32));
  }
}


#define CIR_G(a, b, c, d, x, y)   \
  a = a + b + (x);                \
  d = xor_rotr<32, 0>(d, a);      \
  c = c + d;                      \
  b = xor_rotr<24, R24>(b, c);    \
  a = a + b + (y);                \
  d = xor_rotr<16, R16>(d, a);    \
  c = c + d;                      \
  b = xor_rotr<63, R63>(b, c);

#define CIR_ROUND(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
  CIR_G(v0, v4, v8, v12, m[s0], m[s1])                                                   \
  CIR_G(v1, v5, v9, v13, m[s2], m[s3])                                                   \
  CIR_G(v2, v6, v10, v14, m[s4], m[s5])                                                  \
  CIR_G(v3, v7, v11, v15, m[s6], m[s7])                                                  \
  CIR_G(v0, v5, v10, v15, m[s8], m[s9])                                                  \
  CIR_G(v1, v6, v11, v12, m[s10], m[s11])                                                \
  CIR_G(v2, v7, v8, v13, m[s12], m[s13])                                                 \
  CIR_G(v3, v4, v9, v14, m[s14], m[s15])

// F(h, m, t, f) of RFC 7693 section 3.2 with t < 2^64 (t[1] == 0: a block
// is at most 2^32 bytes here) and f0 = last ? ~0 : 0, f1 = 0.
// R16 / R24 / R63: instruction form of the three non-trivial rotates.
template <int R16, int R24, int R63>
__device__ __forceinline__ void compress_v(uint64_t h[8], const uint64_t m[16], uint64_t t,
                                           bool last) {
  uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3];
  uint64_t v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint64_t v8 = CIR_IV0, v9 = CIR_IV1, v10 = CIR_IV2, v11 = CIR_IV3;
  uint64_t v12 = CIR_IV4 ^ t, v13 = CIR_IV5;
  uint64_t v14 = last ? ~CIR_IV6 : CIR_IV6, v15 = CIR_IV7;
  CIR_ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  CIR_ROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  CIR_ROUND(11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4)
  CIR_ROUND(7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8)
  CIR_ROUND(9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13)
  CIR_ROUND(2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9)
  CIR_ROUND(12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11)
  CIR_ROUND(13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10)
  CIR_ROUND(6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5)
  CIR_ROUND(10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0)
  CIR_ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  CIR_ROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  h[0] = xor3(h[0], v0, v8);
  h[1] = xor3(h[1], v1, v9);
  h[2] = xor3(h[2], v2, v10);
  h[3] = xor3(h[3], v3, v11);
  h[4] = xor3(h[4], v4, v12);
  h[5] = xor3(h[5], v5, v13);
  h[6] = xor3(h[6], v6, v14);
  h[7] = xor3(h[7], v7, v15);
}


// Two independent chains interleaved (ILP 8); same rounds as compress_v.
#define CIR_G2(a, b, c, d, x, y, A, B, C, D, X, Y) \
  a = a + b + (x);                                  \
  A = A + B + (X);                                  \
  d = xor_rotr<32, 0>(d, a);                        \
  D = xor_rotr<32, 0>(D, A);                        \
  c = c + d;                                        \
  C = C + D;                                        \
  b = xor_rotr<24, 0>(b, c);                        \
  B = xor_rotr<24, 0>(B, C);                        \
  a = a + b + (y);                                  \
  A = A + B + (Y);                                  \
  d = xor_rotr<16, 0>(d, a);                        \
  D = xor_rotr<16, 0>(D, A);                        \
  c = c + d;                                        \
  C = C + D;                                        \
  b = xor_rotr<63, 0>(b, c);                        \
  B = xor_rotr<63, 0>(B, C);

#define CIR_ROUND2(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15)          \
  CIR_G2(v0, v4, v8, v12, m[s0], m[s1], w0, w4, w8, w12, q[s0], q[s1])                             \
  CIR_G2(v1, v5, v9, v13, m[s2], m[s3], w1, w5, w9, w13, q[s2], q[s3])                             \
  CIR_G2(v2, v6, v10, v14, m[s4], m[s5], w2, w6, w10, w14, q[s4], q[s5])                           \
  CIR_G2(v3, v7, v11, v15, m[s6], m[s7], w3, w7, w11, w15, q[s6], q[s7])                           \
  CIR_G2(v0, v5, v10, v15, m[s8], m[s9], w0, w5, w10, w15, q[s8], q[s9])                           \
  CIR_G2(v1, v6, v11, v12, m[s10], m[s11], w1, w6, w11, w12, q[s10], q[s11])                       \
  CIR_G2(v2, v7, v8, v13, m[s12], m[s13], w2, w7, w8, w13, q[s12], q[s13])                         \
  CIR_G2(v3, v4, v9, v14, m[s14], m[s15], w3, w4, w9, w14, q[s14], q[s15])

__device__ __forceinline__ void compress2(uint64_t h[8], const uint64_t m[16], uint64_t g[8],
                                          const uint64_t q[16], uint64_t t, bool last) {
  uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint64_t v8 = CIR_IV0, v9 = CIR_IV1, v10 = CIR_IV2, v11 = CIR_IV3;
  uint64_t v12 = CIR_IV4 ^ t, v13 = CIR_IV5, v14 = last ? ~CIR_IV6 : CIR_IV6, v15 = CIR_IV7;
  uint64_t w0 = g[0], w1 = g[1], w2 = g[2], w3 = g[3], w4 = g[4], w5 = g[5], w6 = g[6], w7 = g[7];
  uint64_t w8 = CIR_IV0, w9 = CIR_IV1, w10 = CIR_IV2, w11 = CIR_IV3;
  uint64_t w12 = CIR_IV4 ^ t, w13 = CIR_IV5, w14 = last ? ~CIR_IV6 : CIR_IV6, w15 = CIR_IV7;
  CIR_ROUND2(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  CIR_ROUND2(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  CIR_ROUND2(11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4)
  CIR_ROUND2(7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8)
  CIR_ROUND2(9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13)
  CIR_ROUND2(2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9)
  CIR_ROUND2(12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11)
  CIR_ROUND2(13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10)
  CIR_ROUND2(6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5)
  CIR_ROUND2(10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0)
  CIR_ROUND2(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  CIR_ROUND2(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  h[0] ^= v0 ^ v8; h[1] ^= v1 ^ v9; h[2] ^= v2 ^ v10; h[3] ^= v3 ^ v11;
  h[4] ^= v4 ^ v12; h[5] ^= v5 ^ v13; h[6] ^= v6 ^ v14; h[7] ^= v7 ^ v15;
  g[0] ^= w0 ^ w8; g[1] ^= w1 ^ w9; g[2] ^= w2 ^ w10; g[3] ^= w3 ^ w11;
  g[4] ^= w4 ^ w12; g[5] ^= w5 ^ w13; g[6] ^= w6 ^ w14; g[7] ^= w7 ^ w15;
}


}  // namespace dev
}  // namespace cir
