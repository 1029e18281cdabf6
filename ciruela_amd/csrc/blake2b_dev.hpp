// BLAKE2b-256 (RFC 7693, unkeyed, nn = 32) device core for gfx950.
//
// Replaces the compression function of the `blake2 0.7.1` crate that
// ciruela reaches through `BlockHash::hash_bytes` (reference
// src/block_id.rs:37-43: `Blake2b::VariableOutput::new(32)`, `input`,
// `variable_result`) and through dir-signature's per-block hashing
// (`Hashes::hash_file`, called at src/blocks.rs:193).
//
// Mapping (DESIGN.md "Kernels"): one block chain per lane.  A BLAKE2b chain
// is strictly sequential (ceil(len/128) compressions), so parallelism is
// across blocks; each lane keeps the whole 16-word working vector, the
// 8-word chain value and the current + next 128-byte message line in VGPRs.
//
// Arithmetic on CDNA4's 32-bit VALU:
//   * 64-bit adds      -> v_lshl_add_u64 (shift 0)
//   * xor + rotr 32    -> 2 x v_xor_b32, the rotate is a register swap
//   * xor + rotr 24/16 -> 2 x v_xor_b32 + 2 x v_alignbit_b32
//   * xor + rotr 63    -> 2 x v_xor_b32 + 2 x v_alignbit_b32 (swap + 31)
// hipcc lowers a plain u64 rotate to 64-bit shifts + or (5 ops), so the
// rotates are written on 32-bit halves with __builtin_amdgcn_alignbit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace cir {
namespace dev {

__device__ __forceinline__ uint32_t lo32(uint64_t x) { return (uint32_t)x; }
__device__ __forceinline__ uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
__device__ __forceinline__ uint64_t mk64(uint32_t lo, uint32_t hi) {
  return ((uint64_t)hi << 32) | lo;
}
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
// Same value as mk64, built as a 2-vector: an add of it stays one 64-bit add
// of a register pair (the shift/or form gets re-associated into two adds).
__device__ __forceinline__ uint64_t mk64_pair(uint32_t lo, uint32_t hi) {
  const u32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint64_t, v);
}

// a ^ b ^ c on both halves: one full-rate v_bitop3_b32 per half (gfx950).
__device__ __forceinline__ uint64_t xor3(uint64_t a, uint64_t b, uint64_t c) {
  return mk64(__builtin_amdgcn_bitop3_b32(lo32(a), lo32(b), lo32(c), 0x96),
              __builtin_amdgcn_bitop3_b32(hi32(a), hi32(b), hi32(c), 0x96));
}

#define CIR_IV0 0x6a09e667f3bcc908ULL
#define CIR_IV1 0xbb67ae8584caa73bULL
#define CIR_IV2 0x3c6ef372fe94f82bULL
#define CIR_IV3 0xa54ff53a5f1d36f1ULL
#define CIR_IV4 0x510e527fade682d1ULL
#define CIR_IV5 0x9b05688c2b3e6c1fULL
#define CIR_IV6 0x1f83d9abfb41bd6bULL
#define CIR_IV7 0x5be0cd19137e2179ULL
// Parameter block word 0 for digest_length = 32, key_length = 0,
// fanout = 1, depth = 1 (RFC 7693 section 2.5).
#define CIR_P0_256 0x01010020ULL

// ---------------------------------------------------------------------------
// Step-major compression (the production form).  gfx950 issues the 32-bit
// xor at 2 cycles per wave64 and the 64-bit add / funnel shift at 4
// (tools/valu_ubench.hip); a stream that alternates the two classes issues
// slower than the sum of its parts.  So each half-round runs one G step over
// its 4 independent columns (or diagonals) at a time, and a scheduling
// barrier at every change of class keeps the compiler from re-interleaving:
// 8 slow | 8 fast | 4 slow | 8 fast | 16 slow | 8 fast | 12 slow | 8 fast |
// 8 slow.  Same instructions as the G-at-a-time order the compiler picks
// (compress_v, kept in tools/blake2b_variants.hpp); 4 % faster register-only
// (tools/order_ubench.hip).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }

template <int N>
__device__ __forceinline__ uint64_t rotr_lh(uint32_t l, uint32_t h) {
  if constexpr (N == 32)
    return mk64(h, l);
  else if constexpr (N < 32)
    return mk64(__builtin_amdgcn_alignbit(h, l, N), __builtin_amdgcn_alignbit(l, h, N));
  else
    return mk64(__builtin_amdgcn_alignbit(l, h, N - 32), __builtin_amdgcn_alignbit(h, l, N - 32));
}

#define CIR_XOR4(P, Q)                                            \
  tl0 = lo32(P##0) ^ lo32(Q##0); th0 = hi32(P##0) ^ hi32(Q##0);  \
  tl1 = lo32(P##1) ^ lo32(Q##1); th1 = hi32(P##1) ^ hi32(Q##1);  \
  tl2 = lo32(P##2) ^ lo32(Q##2); th2 = hi32(P##2) ^ hi32(Q##2);  \
  tl3 = lo32(P##3) ^ lo32(Q##3); th3 = hi32(P##3) ^ hi32(Q##3);
#define CIR_ROT4(P, N)              \
  P##0 = rotr_lh<N>(tl0, th0);      \
  P##1 = rotr_lh<N>(tl1, th1);      \
  P##2 = rotr_lh<N>(tl2, th2);      \
  P##3 = rotr_lh<N>(tl3, th3);
#define CIR_ADD4(P, Q) P##0 = P##0 + (Q##0); P##1 = P##1 + (Q##1); P##2 = P##2 + (Q##2); P##3 = P##3 + (Q##3);

// 4 independent G: (a_k, b_k, c_k, d_k) with messages x_k, y_k.
__device__ __forceinline__ void g4(uint64_t& a0, uint64_t& a1, uint64_t& a2, uint64_t& a3,
                                   uint64_t& b0, uint64_t& b1, uint64_t& b2, uint64_t& b3,
                                   uint64_t& c0, uint64_t& c1, uint64_t& c2, uint64_t& c3,
                                   uint64_t& d0, uint64_t& d1, uint64_t& d2, uint64_t& d3,
                                   uint64_t x0, uint64_t x1, uint64_t x2, uint64_t x3,
                                   uint64_t y0, uint64_t y1, uint64_t y2, uint64_t y3) {
  uint32_t tl0, tl1, tl2, tl3, th0, th1, th2, th3;
  CIR_ADD4(a, x) CIR_ADD4(a, b)            // slow
  sched_fence();
  CIR_XOR4(d, a) CIR_ROT4(d, 32)          // fast (rotr 32 is a register swap)
  sched_fence();
  CIR_ADD4(c, d)                          // slow
  sched_fence();
  CIR_XOR4(b, c)                          // fast
  sched_fence();
  CIR_ROT4(b, 24) CIR_ADD4(a, y) CIR_ADD4(a, b)  // slow
  sched_fence();
  CIR_XOR4(d, a)                          // fast
  sched_fence();
  CIR_ROT4(d, 16) CIR_ADD4(c, d)          // slow
  sched_fence();
  CIR_XOR4(b, c)                          // fast
  sched_fence();
  CIR_ROT4(b, 63)                         // slow (runs on into the next g4's adds)
}

#define CIR_ROUND_SM(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15)    \
  g4(v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v15, m[s0], m[s2], m[s4], \
     m[s6], m[s1], m[s3], m[s5], m[s7]);                                                       \
  g4(v0, v1, v2, v3, v5, v6, v7, v4, v10, v11, v8, v9, v15, v12, v13, v14, m[s8], m[s10],       \
     m[s12], m[s14], m[s9], m[s11], m[s13], m[s15]);

struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};

// after_col0() runs between round 0's column step (message words 0-7) and
// its diagonal step (words 8-15): a loader can leave the second half of the
// line's LDS reads in flight under the first G step.
template <typename Hook = NoHook>
__device__ __forceinline__ void compress_sm(uint64_t h[8], const uint64_t m[16], uint64_t t,
                                            bool last, Hook after_col0 = Hook()) {
  uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3];
  uint64_t v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint64_t v8 = CIR_IV0, v9 = CIR_IV1, v10 = CIR_IV2, v11 = CIR_IV3;
  uint64_t v12 = CIR_IV4 ^ t, v13 = CIR_IV5;
  uint64_t v14 = last ? ~CIR_IV6 : CIR_IV6, v15 = CIR_IV7;
  g4(v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v15, m[0], m[2], m[4],
     m[6], m[1], m[3], m[5], m[7]);
  if constexpr (!std::is_same_v<Hook, NoHook>) {
    // the column step's results are materialised here, so the compiler
    // cannot sink it past the hook's wait and branch
    asm volatile("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6),
                 "+v"(v7));
    asm volatile("" : "+v"(v8), "+v"(v9), "+v"(v10), "+v"(v11), "+v"(v12), "+v"(v13),
                 "+v"(v14), "+v"(v15));
    sched_fence();
    after_col0();
    sched_fence();
  }
  g4(v0, v1, v2, v3, v5, v6, v7, v4, v10, v11, v8, v9, v15, v12, v13, v14, m[8], m[10],
     m[12], m[14], m[9], m[11], m[13], m[15]);
  CIR_ROUND_SM(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  CIR_ROUND_SM(11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4)
  CIR_ROUND_SM(7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8)
  CIR_ROUND_SM(9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13)
  CIR_ROUND_SM(2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9)
  CIR_ROUND_SM(12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11)
  CIR_ROUND_SM(13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10)
  CIR_ROUND_SM(6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5)
  CIR_ROUND_SM(10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0)
  CIR_ROUND_SM(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  CIR_ROUND_SM(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  sched_fence();
  h[0] = xor3(h[0], v0, v8);
  h[1] = xor3(h[1], v1, v9);
  h[2] = xor3(h[2], v2, v10);
  h[3] = xor3(h[3], v3, v11);
  h[4] = xor3(h[4], v4, v12);
  h[5] = xor3(h[5], v5, v13);
  h[6] = xor3(h[6], v6, v14);
  h[7] = xor3(h[7], v7, v15);
}

__device__ __forceinline__ void compress(uint64_t h[8], const uint64_t m[16], uint64_t t,
                                         bool last) {
  compress_sm(h, m, t, last);
}

__device__ __forceinline__ void init_state(uint64_t h[8]) {
  h[0] = CIR_IV0 ^ CIR_P0_256;
  h[1] = CIR_IV1;
  h[2] = CIR_IV2;
  h[3] = CIR_IV3;
  h[4] = CIR_IV4;
  h[5] = CIR_IV5;
  h[6] = CIR_IV6;
  h[7] = CIR_IV7;
}

// One full 128-byte message line, 16-byte aligned: 8 x global_load_dwordx4.
__device__ __forceinline__ void load_line16(uint64_t m[16], const uint8_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint4 x = q[k];
    m[2 * k] = mk64(x.x, x.y);
    m[2 * k + 1] = mk64(x.z, x.w);
  }
}

// The first n (0..128) bytes of a line at any alignment, zero padded
// (RFC 7693: the last block is padded with zeros).  Never reads past p + n.
// Used for ragged tails and misaligned blocks only.
__device__ __forceinline__ void load_line_safe(uint64_t m[16], const uint8_t* p, uint32_t n) {
  const bool al4 = (reinterpret_cast<uintptr_t>(p) & 3u) == 0;
#pragma unroll
  for (int w = 0; w < 32; ++w) {
    uint32_t x = 0;
    const uint32_t b0 = 4u * w;
    if (al4 && b0 + 4u <= n) {
      x = *reinterpret_cast<const uint32_t*>(p + b0);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (b0 + k < n) x |= (uint32_t)p[b0 + k] << (8 * k);
    }
    if (w & 1)
      m[w >> 1] |= (uint64_t)x << 32;
    else
      m[w >> 1] = x;
  }
}

// Line i of a chain over [p, p + len): full lines use the vector loader when
// the chain start is 16-byte aligned, the rest go through the safe loader.
__device__ __forceinline__ void load_line_any(uint64_t m[16], const uint8_t* p, uint64_t i,
                                              uint64_t nfull, uint32_t rem, bool al16) {
  const uint8_t* q = p + (i << 7);
  if (al16 && i < nfull) {
    load_line16(m, q);
  } else {
    // opaque: keeps the 128 byte-position compares inside the loop (hoisted,
    // they would occupy SGPR masks and spill)
    uint32_t n = i < nfull ? 128u : rem;
    asm volatile("" : "+v"(n));
    load_line_safe(m, q, n);
  }
}

// Digest of one chain (a block of len bytes at p) into h[0..3].
// Compressions: max(1, ceil(len / 128)); the last one carries the final flag
// and t = len (an exact multiple of 128 is compressed as final, not followed
// by an empty block; the empty input is one all-zero final block, t = 0).
// General path (ragged lengths, any alignment): one message buffer, no
// prefetch, so it stays under the 128-VGPR budget of 4 waves per SIMD.
__device__ __forceinline__ void hash_chain(const uint8_t* p, uint64_t len, uint64_t h[8]) {
  init_state(h);
  const uint32_t nfull = (uint32_t)(len >> 7);
  const uint32_t rem = (uint32_t)(len & 127u);
  const uint32_t total = nfull + ((rem != 0u || len == 0) ? 1u : 0u);
  const bool al16 = (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  uint64_t m[16];
  for (uint32_t i = 0; i < total; ++i) {
    load_line_any(m, p, i, nfull, rem, al16);
    const bool last = i + 1 == total;
    compress(h, m, last ? len : (uint64_t)(i + 1) << 7, last);
  }
}

// hash_chain with the next line loaded while the current one compresses
// (16-byte aligned chains; others take hash_chain): a chain whose wave shares
// its SIMD with few others no longer waits on memory once per line.  The
// last line (full or short) goes through load_line_any.
__device__ __forceinline__ void hash_chain_prefetch(const uint8_t* p, uint64_t len,
                                                    uint64_t h[8]) {
  if (reinterpret_cast<uintptr_t>(p) & 15u) {
    hash_chain(p, len, h);
    return;
  }
  init_state(h);
  const uint32_t nfull = (uint32_t)(len >> 7);
  const uint32_t rem = (uint32_t)(len & 127u);
  const uint32_t total = nfull + ((rem != 0u || len == 0) ? 1u : 0u);
  const uint32_t nu = total - 1u;  // full lines that are not the last
  uint64_t ma[16], mb[16];
  if (nu) load_line16(ma, p);
  for (uint32_t i = 0; i < nu; i += 2) {
    if (i + 1u < nu) load_line16(mb, p + ((uint64_t)(i + 1u) << 7));
    compress(h, ma, (uint64_t)(i + 1u) << 7, false);
    if (i + 1u >= nu) break;
    if (i + 2u < nu) load_line16(ma, p + ((uint64_t)(i + 2u) << 7));
    compress(h, mb, (uint64_t)(i + 2u) << 7, false);
  }
  load_line_any(ma, p, nu, nfull, rem, true);
  compress(h, ma, len, true);
}

// The first rem (0..128) bytes of a 16-byte aligned line, zero padded, with
// 16-byte vector loads: a vector that starts below rem is read whole (it
// lies inside one 16-byte aligned span, so inside the page that holds the
// chain's last byte) and the bytes at and past rem are masked off.
__device__ __forceinline__ void load_line_tail16(uint64_t m[16], const uint8_t* p, uint32_t rem) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint4 x = make_uint4(0, 0, 0, 0);
    if (16u * k < rem) x = q[k];
    uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int keep = (int)rem - (16 * k + 4 * j);  // bytes of word j below rem
      w[j] = keep >= 4 ? w[j] : keep <= 0 ? 0u : w[j] & ((1u << (8 * keep)) - 1u);
    }
    m[2 * k] = mk64(w[0], w[1]);
    m[2 * k + 1] = mk64(w[2], w[3]);
  }
}

// hash_chain for a 16-byte aligned chain start: every line by 16-byte vector
// loads (the short last one masked by load_line_tail16), no byte loads.
__device__ __forceinline__ void hash_chain_al16(const uint8_t* p, uint64_t len, uint64_t h[8]) {
  init_state(h);
  const uint32_t nfull = (uint32_t)(len >> 7);
  const uint32_t rem = (uint32_t)(len & 127u);
  const uint32_t total = nfull + ((rem != 0u || len == 0) ? 1u : 0u);
  uint64_t m[16];
  for (uint32_t i = 0; i < total; ++i) {
    // one loader for every line (n = 128 reads the whole line); n is opaque
    // so the per-word masks stay in the loop instead of SGPR-mask hoisting
    uint32_t n = i < nfull ? 128u : rem;
    asm volatile("" : "+v"(n));
    load_line_tail16(m, p + ((uint64_t)i << 7), n);
    const bool last = i + 1 == total;
    compress(h, m, last ? len : (uint64_t)(i + 1) << 7, last);
  }
}

// ---------------------------------------------------------------------------
// Quad-per-chain mode for long chains (>= kQuadMinLines lines).  A BLAKE2b
// round is 4 independent G on the columns, then 4 on the diagonals; lane i of
// a quad (4 lanes) keeps column i = (v[i], v[4+i], v[8+i], v[12+i]) and
// h[i], h[4+i].  The diagonal step needs b, c, d from lanes i+1, i+2, i+3:
// DPP quad_perm rotates them in and back out.  Message words come from the
// quad's 128-B line in LDS through 48 per-lane precomputed addresses (one per
// round x {column x, column y, diagonal x, diagonal y}).  ~700 instructions
// per compression per lane instead of ~2000: a chain finishes ~2.8x sooner,
// at ~1.4x the total instruction count of lane-per-chain mode.
// ---------------------------------------------------------------------------
// DPP quad_perm read of another lane's 32-bit value.  update_dpp with a zero
// "old" lets the compiler fold the permute into the consuming VOP2
// instruction (v_xor_b32_dpp) instead of emitting a v_mov_b32_dpp.
template <int CTRL>
__device__ __forceinline__ uint32_t qd(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
}
constexpr int kQuadFromNext = 0x39;   // lane i <- lane i+1  (quad_perm [1,2,3,0])
constexpr int kQuadFromNext2 = 0x4E;  // lane i <- lane i+2  (quad_perm [2,3,0,1])
constexpr int kQuadFromPrev = 0x93;   // lane i <- lane i+3  (quad_perm [3,0,1,2])

// One G of quad mode in hand-ordered asm.  The state arrives in the layout of
// the previous half round; the column <-> diagonal moves happen inside the G:
// the permuted b and c feed their 64-bit adds directly as VOP2 DPP carry
// pairs (v_add_co_u32_dpp + v_addc_co_u32_dpp; VOP3 v_lshl_add_u64 has no DPP
// form on gfx9) and b's second read is a v_xor_b32_dpp, so no value is moved
// across lanes on its own: 22 VALU instructions per G (the compiled form
// was 24, ~680 per compression before the DPP folding; 6-7 % less latency
// per compression, tools/quad_dpp_ubench.hip).  Two DPP adds per step is the
// minimum under the gfx9 DPP hazard rule (a DPP source must be written >= 2
// instructions earlier): every 2-step frame assignment of the rows was
// searched.  One asm block is a whole compression
// (compress_quad_asm, message words in registers): the compiler puts an
// s_nop between two inline-asm blocks.
// a, b, c, d, t (the rotr-32 result) and u (xor scratch) are pinned to
// v[40:51] so that every block names the same registers; the compiler cannot
// see the DPP reads inside the asm, so the blocks keep the DPP read-after-
// write distance themselves: b is written by the last two instructions of a
// step and first read across lanes by the third instruction of the next one
// (2 wait states, the gfx9 DPP rule); c and d are read across lanes >= 5
// instructions after their writes.  The last round ends with s_nop 1 for the
// compiler-generated DPP reads of the finalisation.
// Every quad-mode asm block starts its 8-byte instructions on an 8-byte
// boundary (the assembler pads with one s_nop 0 when needed; inside the
// blocks the 4-byte instructions come in pairs).  A VOP2 DPP instruction
// that straddles it issues ~10 % slower for a wave alone
// (tools/align_ubench.hip), and the quad kernels moved 7-10 % with nothing
// but their code offset (profiles/r02/quad_fast/ab_fastpad.log).
#define CIR_QALIGN ".p2align 3\n"
#define CIR_QP_39 " quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf"
#define CIR_QP_4E " quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"
#define CIR_QP_93 " quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf"
// second half of G (no cross-lane reads), shared by both forms
#define CIR_QG_TAIL(Y)                                                        \
  "v_lshl_add_u64 v[40:41], v[40:41], 0, " Y "\n"                             \
  "v_lshl_add_u64 v[40:41], v[40:41], 0, v[42:43]\n"                          \
  "v_xor_b32 v50, v48, v40\n"                                                 \
  "v_xor_b32 v51, v49, v41\n"                                                 \
  "v_alignbit_b32 v46, v51, v50, 16\n"                                        \
  "v_alignbit_b32 v47, v50, v51, 16\n"                                        \
  "v_lshl_add_u64 v[44:45], v[44:45], 0, v[46:47]\n"                          \
  "v_xor_b32 v50, v42, v44\n"                                                 \
  "v_xor_b32 v51, v43, v45\n"                                                 \
  "v_alignbit_b32 v42, v50, v51, 31\n"                                        \
  "v_alignbit_b32 v43, v51, v50, 31\n"
// column step of round 0: every operand in its own lane
#define CIR_QG_PLAIN(X, Y)                                                    \
  "v_lshl_add_u64 v[40:41], v[40:41], 0, " X "\n"                             \
  "v_lshl_add_u64 v[40:41], v[40:41], 0, v[42:43]\n"                          \
  "v_xor_b32 v48, v47, v41\n"                                                 \
  "v_xor_b32 v49, v46, v40\n"                                                 \
  "v_lshl_add_u64 v[44:45], v[44:45], 0, v[48:49]\n"                          \
  "v_xor_b32 v50, v42, v44\n"                                                 \
  "v_xor_b32 v51, v43, v45\n"                                                 \
  "v_alignbit_b32 v42, v51, v50, 24\n"                                        \
  "v_alignbit_b32 v43, v50, v51, 24\n" CIR_QG_TAIL(Y)
// b from lane PB, c from lane PC, d from lane PD
#define CIR_QG_DPP(PB, PC, PD, X, Y)                                          \
  "v_lshl_add_u64 v[40:41], v[40:41], 0, " X "\n"                             \
  "v_add_co_u32_dpp v40, vcc, v42, v40" PB "\n"                               \
  "v_addc_co_u32_dpp v41, vcc, v43, v41, vcc" PB "\n"                         \
  "v_xor_b32_dpp v48, v47, v41" PD "\n"                                       \
  "v_xor_b32_dpp v49, v46, v40" PD "\n"                                       \
  "v_add_co_u32_dpp v44, vcc, v44, v48" PC "\n"                               \
  "v_addc_co_u32_dpp v45, vcc, v45, v49, vcc" PC "\n"                         \
  "v_xor_b32_dpp v50, v42, v44" PB "\n"                                       \
  "v_xor_b32_dpp v51, v43, v45" PB "\n"                                       \
  "v_alignbit_b32 v42, v51, v50, 24\n"                                        \
  "v_alignbit_b32 v43, v50, v51, 24\n" CIR_QG_TAIL(Y)
// Whole compression in one block (message words prefetched into registers:
// no s_nop between rounds).  Word k of the schedule is operand m(k mod 40):
// rounds 10 and 11 repeat rounds 0 and 1.
#define CIR_M(k) "%[m" #k "]"
#define CIR_QR(K0, K1, K2, K3)                                                \
  CIR_QG_DPP(CIR_QP_93, CIR_QP_4E, CIR_QP_39, CIR_M(K0), CIR_M(K1))           \
  CIR_QG_DPP(CIR_QP_39, CIR_QP_4E, CIR_QP_93, CIR_M(K2), CIR_M(K3))
// column step of round 0 straight from the chain value and the constants
// (the hand-scheduled loop): a = h0 (v[52:53]), b = h1 (v[54:55]), c = cv,
// d = (v46, dh) are read where they are instead of being copied into
// v[40:47] first (4 moves fewer per compression); the step writes a, b, c,
// d into v[40:47] as CIR_QG_PLAIN does.  Its first xor is the 8-byte VOP3
// encoding: CIR_QFAST's lone 4-byte s_waitcnt ahead of it would otherwise
// leave every later DPP instruction straddling an 8-byte boundary (~10 %
// slower for a wave alone, see CIR_QALIGN; a config-3 run without it lost
// 10 % of the quad part, profiles/r03/).
#define CIR_QG_PLAIN_H(X, Y)                                                  \
  "v_lshl_add_u64 v[40:41], v[52:53], 0, " X "\n"                             \
  "v_lshl_add_u64 v[40:41], v[40:41], 0, v[54:55]\n"                          \
  "v_xor_b32_e64 v48, %[dh], v41\n"                                           \
  "v_xor_b32 v49, v46, v40\n"                                                 \
  "v_lshl_add_u64 v[44:45], %[cv], 0, v[48:49]\n"                             \
  "v_xor_b32 v50, v54, v44\n"                                                 \
  "v_xor_b32 v51, v55, v45\n"                                                 \
  "v_alignbit_b32 v42, v51, v50, 24\n"                                        \
  "v_alignbit_b32 v43, v50, v51, 24\n" CIR_QG_TAIL(Y)
#define CIR_QCOMPRESS_REST                                                    \
  CIR_QG_DPP(CIR_QP_39, CIR_QP_4E, CIR_QP_93, CIR_M(2), CIR_M(3))             \
  CIR_QR(4, 5, 6, 7) CIR_QR(8, 9, 10, 11) CIR_QR(12, 13, 14, 15)              \
  CIR_QR(16, 17, 18, 19) CIR_QR(20, 21, 22, 23) CIR_QR(24, 25, 26, 27)        \
  CIR_QR(28, 29, 30, 31) CIR_QR(32, 33, 34, 35) CIR_QR(36, 37, 38, 39)        \
  CIR_QR(0, 1, 2, 3) CIR_QR(4, 5, 6, 7) "s_nop 1\n"
#define CIR_QCOMPRESS CIR_QG_PLAIN(CIR_M(0), CIR_M(1)) CIR_QCOMPRESS_REST
#define CIR_MO(k) [m##k] "v"(m[k])

__device__ __forceinline__ void compress_quad_asm(uint64_t& a, uint64_t& b, uint64_t& c,
                                                  uint64_t& d, const uint64_t (&m)[40]) {
  uint64_t t, u;
  asm volatile(CIR_QALIGN CIR_QCOMPRESS
               : "+{v[40:41]}"(a), "+{v[42:43]}"(b), "+{v[44:45]}"(c), "+{v[46:47]}"(d),
                 "=&{v[48:49]}"(t), "=&{v[50:51]}"(u)
               : CIR_MO(0), CIR_MO(1), CIR_MO(2), CIR_MO(3), CIR_MO(4), CIR_MO(5), CIR_MO(6),
                 CIR_MO(7), CIR_MO(8), CIR_MO(9), CIR_MO(10), CIR_MO(11), CIR_MO(12),
                 CIR_MO(13), CIR_MO(14), CIR_MO(15), CIR_MO(16), CIR_MO(17), CIR_MO(18),
                 CIR_MO(19), CIR_MO(20), CIR_MO(21), CIR_MO(22), CIR_MO(23), CIR_MO(24),
                 CIR_MO(25), CIR_MO(26), CIR_MO(27), CIR_MO(28), CIR_MO(29), CIR_MO(30),
                 CIR_MO(31), CIR_MO(32), CIR_MO(33), CIR_MO(34), CIR_MO(35), CIR_MO(36),
                 CIR_MO(37), CIR_MO(38), CIR_MO(39)
               : "vcc");
}

#define CIR_NO(k) [n##k] "=&v"(next[k])
#define CIR_PA(k) [p##k] "v"(pa[k])

// One compression of the hand-scheduled quad loop (quad_fast in
// kernels.hip), setup to finalisation in one block, so the compiler adds no
// waits, moves or branches between compressions:
//   d.lo = dv0.lo ^ (t & m0) (v_bitop3), a = h0, b = h1, c = cv, d.hi
//   s_waitcnt vmcnt(2)      the line loaded two compressions ago has landed
//   2 x ds_write_b128       that line (regs u/w) -> the quad's LDS line
//   2 x global_load_dwordx4 a later line -> u/w, then ptr += step
//   40 x ds_read_b64        the written line's message words -> next
//   24 G steps              on the current words m
//   finalisation            h0 ^= a ^ c[i+2]; h1 ^= b[i+3] ^ d[i+1] (DPP)
//   s_waitcnt lgkmcnt(0)    next has landed (the reads ran under the G steps)
// A wave alone issues ~1 instruction per 4 cycles whatever its kind
// (tools/glue_ubench.hip), so the loop's cost is its instruction count.
#define CIR_RD(k) "ds_read_b64 %[n" #k "], %[p" #k "]\n"
#define CIR_RD40                                                              \
  CIR_RD(0) CIR_RD(1) CIR_RD(2) CIR_RD(3) CIR_RD(4) CIR_RD(5) CIR_RD(6) CIR_RD(7) \
  CIR_RD(8) CIR_RD(9) CIR_RD(10) CIR_RD(11) CIR_RD(12) CIR_RD(13) CIR_RD(14)  \
  CIR_RD(15) CIR_RD(16) CIR_RD(17) CIR_RD(18) CIR_RD(19) CIR_RD(20) CIR_RD(21) \
  CIR_RD(22) CIR_RD(23) CIR_RD(24) CIR_RD(25) CIR_RD(26) CIR_RD(27) CIR_RD(28) \
  CIR_RD(29) CIR_RD(30) CIR_RD(31) CIR_RD(32) CIR_RD(33) CIR_RD(34) CIR_RD(35) \
  CIR_RD(36) CIR_RD(37) CIR_RD(38) CIR_RD(39)
#define CIR_QFAST                                                             \
  CIR_QALIGN                                                                  \
  "v_bitop3_b32 v46, %[dl], %[t], %[lm] bitop3:0x78\n"                        \
  "s_waitcnt vmcnt(2)\n"                                                      \
  "ds_write_b128 %[wr], %[u]\n"                                               \
  "ds_write_b128 %[wr], %[w] offset:16\n"                                     \
  "global_load_dwordx4 %[u], %[ptr], off\n"                                   \
  "global_load_dwordx4 %[w], %[ptr], off offset:16\n"                         \
  "v_lshl_add_u64 %[ptr], %[ptr], 0, %[step]\n" CIR_RD40                      \
  CIR_QG_PLAIN_H(CIR_M(0), CIR_M(1)) CIR_QCOMPRESS_REST                       \
  "v_xor_b32_dpp v48, v44, v40" CIR_QP_4E "\n"                                \
  "v_xor_b32_dpp v49, v45, v41" CIR_QP_4E "\n"                                \
  "v_xor_b32_dpp v54, v42, v54" CIR_QP_93 "\n"                                \
  "v_xor_b32_dpp v55, v43, v55" CIR_QP_93 "\n"                                \
  "v_xor_b32 v52, v52, v48\n"                                                 \
  "v_xor_b32 v53, v53, v49\n"                                                 \
  "v_xor_b32_dpp v54, v46, v54" CIR_QP_39 "\n"                                \
  "v_xor_b32_dpp v55, v47, v55" CIR_QP_39 "\n"                                \
  "s_waitcnt lgkmcnt(0)\n"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // a VGPR quad for asm operands

__device__ __forceinline__ void compress_quad_fast(uint64_t& h0, uint64_t& h1, uint64_t cv,
                                                   uint32_t dl, uint32_t dh, uint32_t t,
                                                   uint32_t m0, const uint64_t (&m)[40],
                                                   uint64_t (&next)[40],
                                                   const uint32_t (&pa)[40], uint32_t wr,
                                                   u32x4& u, u32x4& w, const uint8_t*& ptr,
                                                   uint64_t step) {
  uint64_t a, b, c, d, x, y;
  asm volatile(CIR_QFAST
               : "+{v[52:53]}"(h0), "+{v[54:55]}"(h1), "=&{v[40:41]}"(a), "=&{v[42:43]}"(b),
                 "=&{v[44:45]}"(c), "=&{v[46:47]}"(d), "=&{v[48:49]}"(x), "=&{v[50:51]}"(y),
                 [u] "+v"(u), [w] "+v"(w), [ptr] "+v"(ptr), CIR_NO(0),
                 CIR_NO(1), CIR_NO(2), CIR_NO(3), CIR_NO(4), CIR_NO(5), CIR_NO(6), CIR_NO(7),
                 CIR_NO(8), CIR_NO(9), CIR_NO(10), CIR_NO(11), CIR_NO(12), CIR_NO(13),
                 CIR_NO(14), CIR_NO(15), CIR_NO(16), CIR_NO(17), CIR_NO(18), CIR_NO(19),
                 CIR_NO(20), CIR_NO(21), CIR_NO(22), CIR_NO(23), CIR_NO(24), CIR_NO(25),
                 CIR_NO(26), CIR_NO(27), CIR_NO(28), CIR_NO(29), CIR_NO(30), CIR_NO(31),
                 CIR_NO(32), CIR_NO(33), CIR_NO(34), CIR_NO(35), CIR_NO(36), CIR_NO(37),
                 CIR_NO(38), CIR_NO(39)
               : CIR_MO(0), CIR_MO(1), CIR_MO(2), CIR_MO(3), CIR_MO(4), CIR_MO(5), CIR_MO(6),
                 CIR_MO(7), CIR_MO(8), CIR_MO(9), CIR_MO(10), CIR_MO(11), CIR_MO(12),
                 CIR_MO(13), CIR_MO(14), CIR_MO(15), CIR_MO(16), CIR_MO(17), CIR_MO(18),
                 CIR_MO(19), CIR_MO(20), CIR_MO(21), CIR_MO(22), CIR_MO(23), CIR_MO(24),
                 CIR_MO(25), CIR_MO(26), CIR_MO(27), CIR_MO(28), CIR_MO(29), CIR_MO(30),
                 CIR_MO(31), CIR_MO(32), CIR_MO(33), CIR_MO(34), CIR_MO(35), CIR_MO(36),
                 CIR_MO(37), CIR_MO(38), CIR_MO(39), CIR_PA(0), CIR_PA(1), CIR_PA(2),
                 CIR_PA(3), CIR_PA(4), CIR_PA(5), CIR_PA(6), CIR_PA(7), CIR_PA(8), CIR_PA(9),
                 CIR_PA(10), CIR_PA(11), CIR_PA(12), CIR_PA(13), CIR_PA(14), CIR_PA(15),
                 CIR_PA(16), CIR_PA(17), CIR_PA(18), CIR_PA(19), CIR_PA(20), CIR_PA(21),
                 CIR_PA(22), CIR_PA(23), CIR_PA(24), CIR_PA(25), CIR_PA(26), CIR_PA(27),
                 CIR_PA(28), CIR_PA(29), CIR_PA(30), CIR_PA(31), CIR_PA(32), CIR_PA(33),
                 CIR_PA(34), CIR_PA(35), CIR_PA(36), CIR_PA(37), CIR_PA(38), CIR_PA(39),
                 [wr] "v"(wr), [cv] "v"(cv), [dl] "v"(dl), [dh] "v"(dh), [t] "s"(t),
                 [lm] "v"(m0), [step] "s"(step)
               : "vcc", "memory");
}

// Software-pipelined quad mode (quad_run's asm path): the 40 message words
// of line k+1 are read from LDS into a second register set while line k
// compresses, so a compression never waits on the LDS round trip (write,
// 40 reads, ~300-500 cycles for a wave alone).
__device__ __forceinline__ void quad_read_msg(uint64_t (&m)[40], const uint8_t* line,
                                              const uint32_t (&addr)[48]) {
#pragma unroll
  for (int k = 0; k < 40; ++k) m[k] = *reinterpret_cast<const uint64_t*>(line + addr[k]);
}

__device__ __forceinline__ void compress_quad_regs(uint64_t& h0, uint64_t& h1,
                                                   const uint64_t (&m)[40], uint64_t cv,
                                                   uint64_t dv) {
  uint64_t a = h0, b = h1, c = cv, d = dv;
  compress_quad_asm(a, b, c, d, m);
  const uint64_t cc = mk64(qd<kQuadFromNext2>(lo32(c)) ^ lo32(a), qd<kQuadFromNext2>(hi32(c)) ^ hi32(a));
  h0 = h0 ^ cc;
  const uint64_t bb = mk64(qd<kQuadFromPrev>(lo32(b)) ^ lo32(h1), qd<kQuadFromPrev>(hi32(b)) ^ hi32(h1));
  h1 = mk64(qd<kQuadFromNext>(lo32(d)) ^ lo32(bb), qd<kQuadFromNext>(hi32(d)) ^ hi32(bb));
}

// Bytes [32k, 32k + 32) of a line at p, of which the first n (0..32) are
// real (zero padded); never reads past p + n.
__device__ __forceinline__ void load32_safe(uint4& u, uint4& w, const uint8_t* p, uint32_t n,
                                            bool al16) {
  if (al16 && n == 32) {
    u = reinterpret_cast<const uint4*>(p)[0];
    w = reinterpret_cast<const uint4*>(p)[1];
    return;
  }
  uint32_t x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    x[k] = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (4u * k + j < n) x[k] |= (uint32_t)p[4 * k + j] << (8 * j);
  }
  u = make_uint4(x[0], x[1], x[2], x[3]);
  w = make_uint4(x[4], x[5], x[6], x[7]);
}

__device__ __forceinline__ void store_digest(uint8_t* out, const uint64_t h[8]) {
  uint4* o = reinterpret_cast<uint4*>(out);
  o[0] = make_uint4(lo32(h[0]), hi32(h[0]), lo32(h[1]), hi32(h[1]));
  o[1] = make_uint4(lo32(h[2]), hi32(h[2]), lo32(h[3]), hi32(h[3]));
}

}  // namespace dev
}  // namespace cir
