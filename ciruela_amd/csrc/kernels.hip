// gfx950 kernels of the block-hash path.
//
//   k_chunks         : the hot path (cir_hash_chunks_dev, >= kQuadSmallBatch
//                      blocks): 64 equal blocks per wave, one block chain per
//                      lane, message lines streamed HBM -> LDS by LDS-DMA
//                      (global_load_lds_dwordx4) in full 128-byte lines; the
//                      ragged rest of the file in the same launch.
//   k_uniform_glds   : the same body without the ragged rest (diagnostics).
//   k_uniform_direct : same contract, each lane loads its own line straight
//                      into VGPRs one line ahead (A/B variant of the loader).
//   k_quad_chunks    : small files (< kQuadSmallBatch blocks): 4 lanes per
//                      block chain, 16 chains per wave (DPP quad_perm).
//   k_quad_relay +
//   k_quad_relay_fin.: the blocks of a file past k whole waves per SIMD, as
//                      quad chains cut into segments handed from wave to
//                      wave (beside the k waves of k_chunks / k_quad_chunks).
//   k_quad_long +
//   k_lane_rest      : descriptor batches ordered longest chain first: long
//                      chains in quad mode, the rest one lane per chain.
//   k_chain_step     : the resumable single chain of the index footer.
//   k_general        : ragged / misaligned blocks, chunk or descriptor form.
//   k_sha_desc       : SHA-512/256 descriptors (dir-signature's 2nd hash).
//   k_verify         : digest compare of the daemon-side batch verify.
//   k_compress_only  : register-only compressions (live VALU ceiling).
//   k_fill_splitmix64: synthetic test data (bench / tests only).
//
// Reference semantics: Hashes::hash_file's per-block split (dir-signature
// 0.2.9, reached from src/blocks.rs:193 and src/client/sync/uploads.rs:56)
// and BlockHash::hash_bytes (src/block_id.rs:37-43).
#include "kernels.hpp"

#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "blake2b_dev.hpp"
#include "uniform.hpp"
#include "sha512_dev.hpp"

namespace cir {
namespace dev {

static inline unsigned grid_for(uint64_t n, uint64_t per) { return (unsigned)((n + per - 1) / per); }

// Pure uniform launch: nblk = gridDim.x * 256 equal blocks.
__global__ __launch_bounds__(kThreads, 5) void k_uniform_glds(const uint8_t* __restrict__ data,
                                                               uint64_t bs, uint32_t lines,
                                                               uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWaves * kWaveLds];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // scalar
  const uint64_t blk0 = ((uint64_t)blockIdx.x * kWaves + wave) * 64u;
  uniform_glds_wave(data + blk0 * bs, bs, lines, out + blk0 * 32u, lds + wave * kWaveLds);
}

// Hashes::hash_file over one device-resident file (16-B aligned, bs % 128
// == 0), fused in one launch: the whole blocks [0, nfull) 64 per wave
// through LDS (workgroups ngen_wg.., the file's last wave possibly partial),
// and when ngen_wg == 1 the short last block (block nfull) on one lane of
// workgroup 0 with vector loads (hash_chain_al16).  With a context the short
// block runs in quad mode on another stream instead (launch_chunks_split).
// 4 waves per SIMD (128-VGPR budget; 107 VGPRs, no spills): at 5 (96 VGPRs)
// the ragged branch spilled 6 VGPRs to scratch.  4 and 5 waves run config 2
// within 0.2 % of each other (profiles/r02/ablib_occ4_vs_occ5.log): the body
// is issue-bound.
__global__ __launch_bounds__(kThreads, 4) void k_chunks(const uint8_t* __restrict__ data,
                                                         uint64_t nbytes, uint64_t bs,
                                                         uint32_t lines, uint64_t nfull,
                                                         uint32_t ngen_wg,
                                                         uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWaves * kWaveLds];
  if (blockIdx.x < ngen_wg) {
    if (threadIdx.x != 0) return;
    uint64_t h[8];
    hash_chain_al16(data + nfull * bs, nbytes - nfull * bs, h);  // launched only 16-B aligned
    store_digest(out + nfull * 32u, h);
    return;
  }
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // scalar
  const uint64_t blk0 = ((uint64_t)(blockIdx.x - ngen_wg) * kWaves + wave) * 64u;
  if (blk0 >= nfull) return;
  const uint64_t nv = nfull - blk0;
  if (nv >= 64)
    uniform_glds_wave(data + blk0 * bs, bs, lines, out + blk0 * 32u, lds + wave * kWaveLds);
  else
    uniform_glds_wave<true>(data + blk0 * bs, bs, lines, out + blk0 * 32u, lds + wave * kWaveLds,
                            (uint32_t)nv);
}

__global__ __launch_bounds__(kThreads, 4) void k_uniform_direct(const uint8_t* __restrict__ data,
                                                                 uint64_t bs, uint32_t lines,
                                                                 uint8_t* __restrict__ out) {
  const uint64_t b = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  const uint8_t* p = data + b * bs;
  uint64_t h[8];
  init_state(h);
  uint64_t ma[16], mb[16];
  load_line16(ma, p);
  for (uint32_t i = 0; i < lines; i += 2) {
    if (i + 1 < lines) load_line16(mb, p + (uint64_t)(i + 1) * 128u);
    compress(h, ma, (uint64_t)(i + 1) * 128u, i + 1 == lines);
    if (i + 1 >= lines) break;
    if (i + 2 < lines) load_line16(ma, p + (uint64_t)(i + 2) * 128u);
    compress(h, mb, (uint64_t)(i + 2) * 128u, i + 2 == lines);
  }
  store_digest(out + b * 32u, h);
}

// Chunk form (off == nullptr): block b = [b*bs, min((b+1)*bs, nbytes)) of
// data, b = first + j.  Descriptor form: block b = (off[b], len[b]) of data,
// b = perm ? perm[j] : j.
__global__ __launch_bounds__(kThreads, 4) void k_general(const uint8_t* __restrict__ data,
                                                          uint64_t nbytes, uint64_t bs,
                                                          uint64_t first,
                                                          const uint64_t* __restrict__ off,
                                                          const uint32_t* __restrict__ len,
                                                          const uint32_t* __restrict__ perm,
                                                          uint64_t n, uint8_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (j >= n) return;
  uint64_t b, o, l;
  if (off == nullptr) {
    b = first + j;
    o = b * bs;
    const uint64_t rest = nbytes - o;
    l = rest < bs ? rest : bs;
  } else {
    b = perm ? perm[j] : j;
    o = off[b];
    l = len[b];
  }
  uint64_t h[8];
  hash_chain(data + o, l, h);
  store_digest(out + b * 32u, h);
}

// ---------------------------------------------------------------------------
// Mixed-length descriptor batch, ordered longest chain first (order.hip):
// workgroups [0, nq_wg) run quad-per-chain mode (4 lanes per chain, 16 chains
// per wave, s_setprio 3) over the first *n_long chains if <= 64 nq_wg; the
// rest run lane-per-chain over the remaining ones.  One launch, so the long
// chains start first and the short ones fill the machine around them.
// ---------------------------------------------------------------------------
__constant__ uint8_t kSigma[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

constexpr int kQuadWaveLds = 16 * 128;  // one 128-B line per quad

__device__ __forceinline__ void quad_addr(uint32_t (&addr)[48], uint32_t line, uint32_t i) {
#pragma unroll
  for (int r = 0; r < 12; ++r) {
    addr[4 * r + 0] = line + 8u * kSigma[r][2 * i];
    addr[4 * r + 1] = line + 8u * kSigma[r][2 * i + 1];
    addr[4 * r + 2] = line + 8u * kSigma[r][8 + 2 * i];
    addr[4 * r + 3] = line + 8u * kSigma[r][9 + 2 * i];
  }
}

__device__ __forceinline__ uint64_t iv_lo(uint32_t i) {
  return i == 0 ? CIR_IV0 : i == 1 ? CIR_IV1 : i == 2 ? CIR_IV2 : CIR_IV3;
}
__device__ __forceinline__ uint64_t iv_hi(uint32_t i) {
  return i == 0 ? CIR_IV4 : i == 1 ? CIR_IV5 : i == 2 ? CIR_IV6 : CIR_IV7;
}

// Initial chain value of quad lane i: (h[i], h[4+i]).
__device__ __forceinline__ void quad_init(uint32_t i, uint64_t& h0, uint64_t& h1) {
  h0 = i == 0 ? iv_lo(0) ^ CIR_P0_256 : iv_lo(i);
  h1 = iv_hi(i);
}

// Advance a quad's chain over L bytes at p, t0 bytes already compressed.
// final: the last line (partial, or the empty block of an empty input)
// carries the final flag; otherwise L must be a multiple of 128.
// Pipelined: line it+1 goes regs -> LDS -> the other message set (ma / mb)
// while line it compresses.  At the top of each half the previous reads have
// landed (lgkmcnt(0)), so the LDS line is free for the next write and the
// asm's operands need no wait; the next set's 40 reads stay in flight across
// the compression (the asm names only the current set).  A compression never
// waits on the LDS round trip (write, 40 reads: ~300-500 cycles for a wave
// alone).
__device__ __forceinline__ void quad_run(uint64_t& h0, uint64_t& h1, uint64_t t0,
                                         const uint8_t* p, uint32_t L, bool active, bool final,
                                         uint8_t* lds, const uint32_t (&addr)[48], uint32_t line,
                                         uint32_t i) {
  const uint32_t nfull = L >> 7, rem = L & 127u;
  const uint32_t total =
      !active ? 0u : final ? nfull + ((rem != 0u || (L == 0u && t0 == 0u)) ? 1u : 0u) : nfull;
  const bool al16 = (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  const uint64_t cv = iv_lo(i), dv0 = iv_hi(i);
  auto fetch = [&](uint32_t it, uint4& u, uint4& w) {
    const uint32_t lb = it < nfull ? 128u : rem;
    const uint32_t n = lb > 32u * i ? min(32u, lb - 32u * i) : 0u;
    load32_safe(u, w, p + (uint64_t)it * 128u + 32u * i, n, al16);
  };
  uint4 u = make_uint4(0, 0, 0, 0), w = u;
  if (total) fetch(0, u, w);
  uint64_t ma[40], mb[40];
  auto stage = [&](uint32_t it, uint64_t (&m)[40]) {
    *reinterpret_cast<uint4*>(lds + line + 32u * i) = u;
    *reinterpret_cast<uint4*>(lds + line + 32u * i + 16u) = w;
    if (it + 1 < total) fetch(it + 1, u, w);
    quad_read_msg(m, lds, addr);
  };
  auto step = [&](uint32_t it, const uint64_t (&m)[40]) {
    const bool last = final && it + 1 == total;
    const uint64_t t = t0 + (last ? (uint64_t)L : (uint64_t)(it + 1) * 128u);
    const uint64_t dv = dv0 ^ (i == 0 ? t : 0ull) ^ ((i == 2 && last) ? ~0ull : 0ull);
    compress_quad_regs(h0, h1, m, cv, dv);
  };
  constexpr int kLgkm0 = 0xC07F;  // s_waitcnt lgkmcnt(0), vmcnt/expcnt untouched
  if (total) stage(0, ma);
  for (uint32_t it = 0; it < total; it += 2) {
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    if (it + 1 < total) stage(it + 1, mb);
    step(it, ma);
    if (it + 1 >= total) break;
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    if (it + 2 < total) stage(it + 2, ma);
    step(it + 1, mb);
  }
}

// The chain of quad q of this wave (block b at p, L bytes; have = false for a
// quad past the end) is hashed into out + 32 b.
// Hand-scheduled quad loop (compress_quad_fast): lines [0, nu) of this
// quad's chain, nu even, >= 4 and wave-uniform, every line full, not final
// and 16-B aligned for every active quad of the wave.  Line j+1 waits in
// register set (j+1) % 2 until compression j writes it to LDS and reloads
// the set with line min(j+3, nu-1) (clamped, so nothing past the uniform
// part is read; the repeats are never used); compression j reads line j+1's
// message words while it runs.  No branch, no compiler-inserted wait
// between compressions.
// quad_fast in two halves: quad_fast_begin loads the first three lines and
// reads line 0's message words (no chain value needed yet), quad_fast_run
// compresses.  The relay (k_quad_relay) runs the first half while its
// segment waits for the predecessor's chain value.
struct QuadFast {
  uint64_t ma[40], mb[40];
  uint32_t pa[40];
  uint32_t wr;
  u32x4 u0, w0, u1, w1;
  const uint8_t* ptr;
};

__device__ __forceinline__ void quad_fast_begin(QuadFast& f, const uint8_t* p, uint8_t* lds,
                                                const uint32_t (&addr)[48], uint32_t line,
                                                uint32_t i) {
  // LDS byte address of the kernel's shared array: a generic pointer into
  // LDS is the shared aperture's base in its high half and the LDS offset in
  // its low half, so the low 32 bits are what ds_read / ds_write take
  const uint32_t base = (uint32_t)reinterpret_cast<uintptr_t>(lds);
#pragma unroll
  for (int k = 0; k < 40; ++k) f.pa[k] = base + addr[k];
  f.wr = base + line + 32u * i;
  const uint8_t* src = p + 32u * i;
  const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
  *reinterpret_cast<u32x4*>(lds + line + 32u * i) = s4[0];
  *reinterpret_cast<u32x4*>(lds + line + 32u * i + 16u) = s4[1];
  quad_read_msg(f.ma, lds, addr);
  f.u1 = s4[8];  // lines 1 and 2
  f.w1 = s4[9];
  f.u0 = s4[16];
  f.w0 = s4[17];
  // the compiler's own waits for these loads go here, not into the loop
  asm volatile("" : "+v"(f.u1), "+v"(f.w1), "+v"(f.u0), "+v"(f.w0));
  f.ptr = src + 384;
}

__device__ __forceinline__ void quad_fast_run(QuadFast& f, uint64_t& h0, uint64_t& h1,
                                              uint32_t nu, uint32_t i, uint32_t t0) {
  const uint64_t cv = iv_lo(i), dv0 = iv_hi(i);
  const uint32_t m0 = i == 0 ? ~0u : 0u;  // lane 0 of the quad carries t
  const uint32_t dl = lo32(dv0), dh = hi32(dv0);
  for (uint32_t j = 0; j < nu; j += 2) {
    compress_quad_fast(h0, h1, cv, dl, dh, t0 + (j + 1u) * 128u, m0, f.ma, f.mb, f.pa, f.wr, f.u1,
                       f.w1, f.ptr, j + 4u < nu ? 128u : 0u);
    compress_quad_fast(h0, h1, cv, dl, dh, t0 + (j + 2u) * 128u, m0, f.mb, f.ma, f.pa, f.wr, f.u0,
                       f.w0, f.ptr, j + 5u < nu ? 128u : 0u);
  }
  // the last loads are in flight into u0/w0/u1/w1: keep the registers until
  // they have landed
  asm volatile("s_waitcnt vmcnt(0)" ::"v"(f.u0), "v"(f.w0), "v"(f.u1), "v"(f.w1) : "memory");
}

__device__ __forceinline__ void quad_fast(uint64_t& h0, uint64_t& h1, const uint8_t* p,
                                          uint32_t nu, uint8_t* lds,
                                          const uint32_t (&addr)[48], uint32_t line,
                                          uint32_t i, uint32_t t0 = 0) {
  QuadFast f;
  quad_fast_begin(f, p, lds, addr, line, i);
  quad_fast_run(f, h0, h1, nu, i, t0);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) v = min(v, (uint32_t)__shfl_xor((int)v, s));
  return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, s));
  return __builtin_amdgcn_readfirstlane(v);
}

// Lines of a quad's chain that quad_fast may take: full, not final, from a
// 16-B aligned start (0 for an inactive quad of the wave: it does not run).
constexpr uint32_t kQuadFastMin = 8;

__device__ __forceinline__ void quad_chain(bool have, uint64_t b, const uint8_t* p, uint32_t L,
                                           uint8_t* __restrict__ out, uint8_t* lds,
                                           uint32_t wave_lds) {
  const uint32_t lane = threadIdx.x & 63u, i = lane & 3u, q = lane >> 2;
  const uint32_t line = wave_lds + q * 128u;  // this quad's line in LDS
  uint32_t addr[48];
  quad_addr(addr, line, i);
  uint64_t h0, h1;
  quad_init(i, h0, h1);
  uint32_t t0 = 0;
  {
    const bool al16 = (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
    const uint32_t nf = !have ? 0xffffffffu : (al16 && L > 0u) ? (L - 1u) >> 7 : 0u;
    const uint32_t nu = wave_min_u32(nf) & ~1u;
    if (nu >= kQuadFastMin && nu != 0xfffffffeu) {
      if (have) quad_fast(h0, h1, p, nu, lds, addr, line, i);
      t0 = nu * 128u;
    }
  }
  quad_run(h0, h1, t0, p + t0, have ? L - t0 : 0u, have, true, lds, addr, line, i);
  if (have) *reinterpret_cast<uint64_t*>(out + b * 32u + 8u * i) = h0;
}

// One quad's chain advanced over n bytes at p (t0 bytes already compressed;
// final: the last line carries the final flag): the lines quad_fast can take
// (16-B aligned, t stays below 2^32), then the general loop.  The index
// footer (k_chain_step) and hash_bytes (k_single).
__device__ __forceinline__ void quad_single(uint64_t& h0, uint64_t& h1, uint64_t t0,
                                            const uint8_t* p, uint32_t n, bool final,
                                            uint8_t* lds, const uint32_t (&addr)[48],
                                            uint32_t i) {
  uint32_t done = 0;
  const bool al16 = (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  if (al16 && t0 + n < (1ull << 32)) {
    const uint32_t nf = final ? (n > 0u ? (n - 1u) >> 7 : 0u) : n >> 7;
    const uint32_t nu = nf & ~1u;
    if (nu >= kQuadFastMin) {
      quad_fast(h0, h1, p, nu, lds, addr, 0u, i, (uint32_t)t0);
      done = nu * 128u;
    }
  }
  quad_run(h0, h1, t0 + done, p + done, n - done, true, final, lds, addr, 0u, i);
}

__device__ __forceinline__ void quad_chains(const uint8_t* __restrict__ arena,
                                            const uint64_t* __restrict__ off,
                                            const uint32_t* __restrict__ len,
                                            const uint32_t* __restrict__ perm, uint32_t first,
                                            uint32_t nlong, uint8_t* __restrict__ out,
                                            uint8_t* lds, uint32_t wave_lds) {
  const uint32_t c = first + ((threadIdx.x & 63u) >> 2);
  const bool have = c < nlong;
  uint32_t b = 0, L = 0;
  uint64_t o = 0;
  if (have) {
    b = perm[c];
    o = off[b];
    L = len[b];
  }
  quad_chain(have, b, arena + o, L, out, lds, wave_lds);
}

// Hashes::hash_file split of one device-resident file, blocks [b0, nblk):
// every block in quad mode (16 per wave).  The whole file when it has fewer
// than kQuadSmallBatch blocks; otherwise the ragged rest beside k_chunks'
// uniform part (launch_chunks_split).
// kBase: the base part beside a relay (launch_chunks_split) runs at priority
// 2, so the relay's segments (priority 3) issue first on a shared SIMD.
template <bool kBase = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_quad_chunks(
    const uint8_t* __restrict__ data, uint64_t nbytes, uint64_t bs, uint64_t b0, uint64_t nblk,
    uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWaves * kQuadWaveLds];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t first = b0 + ((uint64_t)blockIdx.x * kWaves + wave) * 16u;
  if (first >= nblk) return;
  __builtin_amdgcn_s_setprio(kBase ? 2 : 3);
  const uint64_t b = first + ((threadIdx.x & 63u) >> 2);
  const bool have = b < nblk;
  const uint64_t o = have ? b * bs : 0;
  const uint64_t rest = nbytes - o;
  quad_chain(have, b, data + o, have ? (uint32_t)(rest < bs ? rest : bs) : 0u, out, lds,
             wave * kQuadWaveLds);
}

// ---------------------------------------------------------------------------
// Relay: the whole blocks of a file beyond k whole lane waves per SIMD.
// Lane mode holds 64 chains per wave, so a file of 65536 k + E blocks (E
// small, 1024 SIMDs) costs k + 1 lane waves on the SIMDs that get the extra
// chains: 65537 x 32 KiB ran 1.51 ms against 1.16 ms for 65536.  Instead the
// first 65536 k blocks run in lane mode (k_chunks) and the E extra chains in
// quad mode, 16 per group (one wave), each chain cut into segments of
// seg_lines lines that run one after another in different workgroups: a
// segment's wave waits for its predecessor's flag, picks the chain values up
// from `state`, compresses its lines at s_setprio 3 and hands on.  The extra
// work is spread thin over many SIMDs instead of doubling a few of them.
// Workgroup x = segment x / ngroups of group x % ngroups, so segments are
// dispatched in order and a waiting wave's predecessor is always resident
// or done.  A wave that waits longer than max_polls polls leaves its segment
// (and every later one) to k_quad_relay_finish, queued behind on the same
// stream, so the relay always drains and the digests never depend on timing.
// flags[g] = segments of group g done (zeroed before the launch).
// ---------------------------------------------------------------------------
constexpr uint32_t kRelayGroupChains = 16;
constexpr int kRelaySleep = 8;  // s_sleep units (64 clocks): ~0.25 us between polls
// Each segment adds its lines' quad-mode work (~1 us per line) to the lane
// wave of the SIMD it lands on, so short chains take short segments: at
// 32 lines, 16-line segments cost the lane part 12 %.  8 = the hand-
// scheduled loop's minimum (kQuadFastMin).  Each hand-off costs ~4 us.
constexpr uint32_t kRelayMinSegLines = 8;

// Lines [l0, l1) of a chain of full 128-B lines at blk (16-B aligned);
// final: l1 is the chain's last line.  nu is wave-uniform because every chain
// of the wave has the same lines.
__device__ __forceinline__ void quad_lines(uint64_t& h0, uint64_t& h1, const uint8_t* blk,
                                           uint32_t l0, uint32_t l1, bool final, bool have,
                                           uint8_t* lds, const uint32_t (&addr)[48],
                                           uint32_t line, uint32_t i) {
  const uint32_t n = l1 - l0;
  uint32_t done = 0;
  const uint32_t nu = (final ? n - 1u : n) & ~1u;
  if (nu >= kQuadFastMin) {
    if (have) quad_fast(h0, h1, blk + (uint64_t)l0 * 128u, nu, lds, addr, line, i, l0 * 128u);
    done = nu;
  }
  quad_run(h0, h1, (uint64_t)(l0 + done) * 128u, blk + (uint64_t)(l0 + done) * 128u,
                 have ? (n - done) * 128u : 0u, have, final, lds, addr, line, i);
}

// This lane's index in the wave, recomputed where it is called (volatile: the
// compiler may not keep it, or anything derived from it, live in a VGPR
// across the compression loop instead).
__device__ __forceinline__ uint32_t lane_now() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n v_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// The chains a relay hands on, c = 0 .. n-1: the blocks b0 + c of a file
// of bs-byte blocks (chunk form, every chain the same length: kUniform) or
// the chains first + c of an ordered descriptor batch.  The order is by
// length bin (order.hip), exact only below 2048 lines: above that one bin
// spans several lengths in arbitrary order, so a group's first chain need not
// be its longest and relay_segment takes the group's maximum.
struct RelayFile {
  static constexpr bool kUniform = true;
  const uint8_t* data;
  uint64_t bs, b0;
  uint32_t n;
  __device__ __forceinline__ uint64_t block(uint32_t c) const { return b0 + c; }
  __device__ __forceinline__ const uint8_t* ptr(uint32_t c) const { return data + (b0 + c) * bs; }
  __device__ __forceinline__ uint64_t bytes(uint32_t) const { return bs; }
};

struct RelayDesc {
  static constexpr bool kUniform = false;
  const uint8_t* arena;
  const uint64_t* off;
  const uint32_t* len;
  const uint32_t* perm;
  uint64_t first;
  uint32_t n;
  __device__ __forceinline__ uint64_t block(uint32_t c) const { return perm[first + c]; }
  __device__ __forceinline__ const uint8_t* ptr(uint32_t c) const { return arena + off[block(c)]; }
  __device__ __forceinline__ uint64_t bytes(uint32_t c) const { return len[block(c)]; }
};

// Extra blocks a relay takes at most, as lines / relay_cap_div(lines) of a
// lane wave per SIMD (and at most 5/8 of one): 1/2 of a wave of 16-line
// chains, 5/8 from 20 lines on.  With the prefetching lane part and the
// fence-free hand-off this pays at every measured short shape (4 KiB x
// 73728 1403-1424 -> 1675-1700 GiB/s, x 106496 1337-1407 -> 1515-1562,
// 8 KiB x 98304 1581-1603 -> 1793-1832, 2 KiB x 139264 1431-1439 ->
// 1718-1725; 16-line chains past 1/4 of a wave neither gain nor lose;
// profiles/r02/relay/capdiv/), where lines / 512 (below 64 lines) and
// lines / 256 had not before.
__host__ __device__ __forceinline__ uint64_t relay_cap_div(uint64_t) { return 32; }

// Compressions of a chain of L bytes (the empty input compresses once).
__device__ __forceinline__ uint32_t chain_lines(uint64_t L) {
  return L ? (uint32_t)((L + 127u) >> 7) : 1u;
}

// Segment s of group g: lines [s * seg_lines, l1_max) of each of its chains
// (clipped to the chain; a chain that ended in an earlier segment sits it
// out).  Per-lane values are rebuilt from the lane index after each loop, so
// a relay wave needs no more registers than k_quad_chunks' waves.
// max_polls > 0: wait for the predecessor's flag first (0 = the finisher,
// which does not wait); the segment's first lines are loaded before the
// wait, so a hand-off costs the flag and the chain value's round trips
// only.  Returns early (nothing written) when the wait gives up, or when
// the group's chains all ended before this segment (descriptor relays
// launch the most segments any group can need).
template <typename R>
__device__ __forceinline__ void relay_segment(const R& r, uint32_t g, uint32_t s, uint32_t l1_max,
                                              uint32_t seg_lines, uint32_t* flags,
                                              uint64_t* state, uint8_t* __restrict__ out,
                                              uint8_t* lds, uint32_t max_polls, bool publish) {
  const uint32_t l0 = s * seg_lines;
  auto chain = [&](uint32_t lane) { return g * kRelayGroupChains + (lane >> 2); };
  // the group's longest chain decides whether this segment has work and
  // whether it finishes the group (the final flag): every chain of the group,
  // not only its first, must have ended when the flag says so
  uint32_t group_lines;
  if constexpr (R::kUniform) {
    group_lines = chain_lines(r.bytes(0));
  } else {
    const uint32_t c = chain(lane_now());
    group_lines = wave_max_u32(c < r.n ? chain_lines(r.bytes(c)) : 0u);
  }
  if (l0 >= group_lines && s > 0) return;
  const bool group_final = l1_max >= group_lines;
  // lines of this lane's chain in the segment; nu = the wave's common run
  // of full, not final, 16-B aligned lines for the hand-scheduled loop
  uint32_t nu = 0;
  {
    const uint32_t c = chain(lane_now());
    uint32_t avail = 0xffffffffu;  // quads without a chain here do not bound it
    if (c < r.n) {
      const uint64_t L = r.bytes(c);
      const uint32_t T = chain_lines(L);
      if (T > l0) {
        const uint32_t e = min(l1_max, T - 1u);  // the last line is never in the loop
        const bool al16 = (reinterpret_cast<uintptr_t>(r.ptr(c)) & 15u) == 0;
        avail = (al16 && e > l0) ? e - l0 : 0u;
      }
    }
    nu = wave_min_u32(avail);
    nu = nu == 0xffffffffu ? 0u : nu & ~1u;
    if (nu < kQuadFastMin) nu = 0;
  }
  auto active = [&](uint32_t c) { return c < r.n && chain_lines(r.bytes(c)) > l0; };
  QuadFast f;
  if (nu) {
    const uint32_t lane = lane_now(), c = chain(lane);
    if (active(c)) {
      uint32_t addr[48];
      quad_addr(addr, (lane >> 2) * 128u, lane & 3u);
      quad_fast_begin(f, r.ptr(c) + (uint64_t)l0 * 128u, lds, addr, (lane >> 2) * 128u,
                      lane & 3u);
    }
  }
  if (s > 0 && max_polls) {
    // wait at normal priority (s_sleep: the SIMD's other waves keep issuing)
    for (uint32_t k = 0;; ++k) {
      const uint32_t fl = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(flags + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      if (fl == s) break;
      if (k >= max_polls) return;  // the finisher takes over from here
      __builtin_amdgcn_s_sleep(kRelaySleep);
    }
    // compiler barrier: the chain-value loads below stay after the flag load
    // (in the ISA they also depend on it through the scalar branch)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
  __builtin_amdgcn_s_setprio(3);
  uint64_t h0, h1;
  {
    const uint32_t lane = lane_now();
    if (s == 0) {
      quad_init(lane & 3u, h0, h1);
    } else {
      uint64_t* st = state + ((uint64_t)g * 64u + lane) * 2u;
      // agent-scope loads (sc1): coherent across XCDs without the L2
      // invalidate of an acquire fence; issued after the flag was seen
      h0 = __hip_atomic_load(st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      h1 = __hip_atomic_load(st + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (nu) {
    const uint32_t lane = lane_now();
    if (active(chain(lane))) quad_fast_run(f, h0, h1, nu, lane & 3u, l0 * 128u);
  }
  {
    const uint32_t lane = lane_now(), c = chain(lane);
    const bool have = active(c);
    uint64_t L = 0;
    bool fin = false;
    const uint8_t* p = nullptr;
    if (have) {
      const uint64_t bytes = r.bytes(c);
      const uint32_t T = chain_lines(bytes);
      fin = T <= l1_max;
      const uint64_t t0 = (uint64_t)(l0 + nu) * 128u;
      L = (fin ? bytes : (uint64_t)min(l1_max, T) * 128u) - t0;
      p = r.ptr(c) + t0;
    }
    uint32_t addr[48];
    quad_addr(addr, (lane >> 2) * 128u, lane & 3u);
    quad_run(h0, h1, (uint64_t)(l0 + nu) * 128u, p, (uint32_t)L, have, fin, lds, addr,
             (lane >> 2) * 128u, lane & 3u);
  }
  const uint32_t lane = lane_now(), c = chain(lane);
  if (active(c)) {
    if (chain_lines(r.bytes(c)) <= l1_max) {
      *reinterpret_cast<uint64_t*>(out + r.block(c) * 32u + 8u * (lane & 3u)) = h0;
    } else {
      uint64_t* st = state + ((uint64_t)g * 64u + lane) * 2u;
      __hip_atomic_store(st, h0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(st + 1, h1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (!publish) return;
  // The hand-off protocol (fence-free; +1-5 % on relayed shapes against
  // agent-scope acquire/release fences, which write back / invalidate the
  // whole L2: profiles/r02/relay/light/).  Its ISA assumptions, checked on
  // the built code object by tests/test_relay_isa.py:
  //   * the chain values are stored and loaded with sc1 (agent-scope relaxed
  //     atomics: written through to, and read from, the level every XCD
  //     sees);
  //   * the producer's s_waitcnt vmcnt(0) completes those stores before the
  //     flag store is issued (gfx9 counts stores in vmcnt, in order);
  //   * the consumer reads the chain values only after the flag load has
  //     returned the expected value (the poll loop's scalar branch).
  // The digests themselves are read only after the kernel.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0)
    __hip_atomic_store(flags + g, group_final ? 0xffffffffu : s + 1u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_quad_relay(
    const uint8_t* __restrict__ data, uint64_t bs, uint64_t b0, uint32_t nrel, uint32_t ngroups,
    uint32_t seg_lines, uint32_t* flags, uint64_t* state, uint8_t* __restrict__ out,
    uint32_t max_polls) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kQuadWaveLds];
  const uint32_t g = blockIdx.x % ngroups, s = blockIdx.x / ngroups;
  const RelayFile r{data, bs, b0, nrel};
  relay_segment(r, g, s, (s + 1u) * seg_lines, seg_lines, flags, state, out, lds,
                max_polls ? max_polls : 1u, true);
}

// Behind k_quad_relay on its stream: every group whose last segment has not
// run (a wave gave up waiting) is finished from its last handed-on state.
// Then the group's flag goes back to 0 for the next relay on this stream
// (the scratch's flags are zeroed once, when it is allocated).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_quad_relay_finish(
    const uint8_t* __restrict__ data, uint64_t bs, uint64_t b0, uint32_t nrel, uint32_t seg_lines,
    uint32_t* flags, uint64_t* state, uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kQuadWaveLds];
  const uint32_t g = blockIdx.x;
  const uint32_t s = __builtin_amdgcn_readfirstlane(flags[g]);
  const RelayFile r{data, bs, b0, nrel};
  if (s != 0xffffffffu)  // else the relay finished this group
    relay_segment(r, g, s, 0xffffffffu, seg_lines, flags, state, out, lds, 0u, false);
  if (threadIdx.x == 0) flags[g] = 0;
}

// The chains of an ordered batch that run in quad mode: its long chains when
// they all fit the quad part (64 nq_wg), none otherwise.  Beyond the quad
// part's 16384 chains (one exclusive wave per SIMD) the long chains are as
// many as a lane wave per SIMD can hold or more, and one lane per chain is
// the faster mode for them (lane mode costs 30 issue slots per chain-line,
// quad 33); splitting them instead ran the rest in lane mode only after the
// exclusive quad part had let go of the SIMDs, with the lane workgroups
// packed onto the CUs that freed first: 256 KiB x 65536 descriptors 31 ms
// (profiles/r02/desc/).
__device__ __forceinline__ uint32_t quad_part_chains(uint32_t n_long, uint32_t nq_wg) {
  return n_long <= nq_wg * 64u ? n_long : 0u;
}

// Relay of a small descriptor batch (quad regime, launch_mixed): the host
// launches one when n = 16384 k + extra (16 chains per quad wave, one wave
// per SIMD per k), extra <= 1/2 of that; it runs only when every chain of
// the batch is in the quad part (count[0] == n, so the split is exact) and
// the longest relayed chain has >= min_lines lines (the chunk-form rule:
// 64 at k = 1, 32 above, 128 past 1/4 of a wave).
__device__ __forceinline__ bool desc_qrelay_on(const uint32_t* count, const uint32_t* len,
                                               const uint32_t* perm, uint64_t n, uint32_t extra,
                                               uint32_t min_lines) {
  if (extra == 0 || min_lines == 0 || count[0] != n) return false;
  return chain_lines(len[perm[n - extra]]) >= min_lines;
}

// Quad part of an ordered batch: chains [0, quad_part_chains()).
// Latency-bound (one 1 MiB chain = 8192 dependent compressions), so it keeps
// a line's 40 message words in registers and runs at s_setprio 3; it is its
// own kernel so the lane part keeps its occupancy.  kExclusive: each wave
// touches a255, so it holds the SIMD's whole 512-register file and no lane
// wave can share its SIMD (batches with a lane part beside the quad part).
// relay_extra / relay_min_lines (small batches only): the last relay_extra
// chains run in k_desc_relay instead when desc_qrelay_on (the base then
// runs at priority 2 so the relay's segments issue first).
template <bool kExclusive>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_quad_long(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ perm, uint32_t* n_long,
    uint32_t nq_wg, uint8_t* __restrict__ out, uint64_t n, uint32_t relay_extra,
    uint32_t relay_min_lines) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWaves * kQuadWaveLds];
  if constexpr (kExclusive) {
    asm volatile("v_accvgpr_write_b32 a255, 0" ::: "a255");
    // this workgroup holds its CU: count it for k_gate (n_long[1])
    if (threadIdx.x == 0) __hip_atomic_fetch_add(n_long + 1, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
  }
  const bool relayed = desc_qrelay_on(n_long, len, perm, n, relay_extra, relay_min_lines);
  const uint32_t nl = relayed ? (uint32_t)(n - relay_extra) : quad_part_chains(*n_long, nq_wg);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t first = (blockIdx.x * kWaves + wave) * 16u;
  if (first >= nl) return;
  if (relayed)
    __builtin_amdgcn_s_setprio(2);
  else
    __builtin_amdgcn_s_setprio(3);
  quad_chains(arena, off, len, perm, first, nl, out, lds, wave * kQuadWaveLds);
}

// The lane part of an exclusive mixed batch waits until every quad
// workgroup holds its CU (so lane waves cannot take the CUs the quad part
// needs whole): one wave polls the quad part's started-workgroup counter,
// sleeping ~3.4 us between polls, for at most max_rounds polls (~2 ms; the
// gate never waits on anything else, so it cannot deadlock: if the quad part
// is held up by other work, the lane part just starts after the bound).
// Round 1 waited a fixed ~20 us (k_delay): with several contexts' streams in
// one process the quad part's dispatch lagged behind that and config 3 lost
// 12 % (profiles/r02/queue_probe_v2_hiq.log, lead.log).
__global__ void k_gate(const uint32_t* started, uint32_t target, uint32_t max_rounds) {
  for (uint32_t r = 0; r < max_rounds; ++r) {
    if (__hip_atomic_load(started, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return;
    __builtin_amdgcn_s_sleep(127);
  }
}

// Lane part: chains [nl, n) of the order, one lane per chain.
//
// Pacing (pace != 0, exclusive mixed batches): the quad part's longest chain
// sets the batch's time, and whatever else runs meanwhile lowers the chip's
// clock -- beside a full-width lane part the quad waves ran at 2.20 GHz
// instead of 2.39 alone (profiles/r02/lane_pacing/).  So when every long
// chain is in the quad part, only as many lane workgroups run as finish the
// lane work (count[4..5]) within the longest quad chain (count[2]) at `pace`
// lane compressions per workgroup per quad compression; the other
// workgroups exit at once.  Waves claim tiles of 64 chains of the order from
// count[6], so a helper launch behind the quad part (k_lane_tiles, helper)
// finishes whatever the paced part left when the quad part ended: a pace
// set too high costs the leftover's time on the whole chip instead of
// stretching the lane part past the quad part.  Config 3, one library, one
// process per value (profiles/r02/lane_pacing/pace_sweep.log): pace 0 826
// GiB/s, 40 863, 52 877-887, 60 896, 80 878-880 (without the helper, 56
// fell to 771); with the hand-scheduled quad loop: 0 886-892, 48 952-957,
// 60 948-957, 72 937-941, 90 907; after the ordering fixes: 0 908-918, 48
// 977-993, 64 1012-1021, 80 970-973, 100 930-934.
constexpr uint32_t kLanePace = 64;

// Workgroups of a paced lane part, or 0 when the batch is not paced (no
// pacing asked, no long chain, or more long chains than the quad part holds).
__device__ __forceinline__ uint64_t lane_paced_wgs(const uint32_t* count, uint32_t nq_wg,
                                                    uint32_t pace) {
  const uint32_t nlong = count[0];
  if (pace == 0 || nlong == 0 || nlong > nq_wg * 64u) return 0;
  const uint64_t lq = (uint64_t)count[2] * pace;
  const uint64_t work = *reinterpret_cast<const unsigned long long*>(count + 4);
  return max<uint64_t>(1, (work + lq - 1) / lq);
}

__device__ __forceinline__ void lane_chain(const uint8_t* __restrict__ arena,
                                           const uint64_t* __restrict__ off,
                                           const uint32_t* __restrict__ len, uint32_t b,
                                           uint8_t* __restrict__ out) {
  uint64_t h[8];
  hash_chain(arena + off[b], len[b], h);
  store_digest(out + (uint64_t)b * 32u, h);
}

// Unpaced lane part: one lane per chain, one pass, the next line loaded while
// the current one compresses (hash_chain_prefetch: +2-5 % on lane-only
// batches, +30 % where few waves share a SIMD; 4 waves per SIMD, ~10 VGPRs
// spilled around the chain loop, not in it).  With pace != 0 it leaves a
// paced batch to k_lane_tiles.
// Relay of a descriptor batch (launch_mixed): the host launches one when
// the batch is k = 1 .. kRelayMaxK lane waves per SIMD plus `extra` chains
// (extra = n mod slots, slots = 64 x SIMDs); whether it runs is decided on
// the device, where the lengths are: only with no quad part (no long chains,
// or more than it holds: then every chain is lane mode and extra is exact),
// when the longest relayed chain (the first of the last `extra`, the order
// being longest first) has >= 16 lines and extra <= min(cap8 / 8, lines /
// 256) of slots (the chunk-form rule, relay_plan; cap8 = 5).  The relay
// waves go in behind a gate on the lane part's workgroups (launch_mixed):
// without it they were dispatched first, on the high-priority stream, and
// kept lane workgroups off the SIMDs (32 KiB x 106496 descriptors 1678 ->
// 1213 GiB/s with 40960 relayed).  k_lane_rest, the relay and its finisher
// all evaluate this, so they agree on the split.
__device__ __forceinline__ bool desc_relay_on(const uint32_t* count, uint32_t nq_wg,
                                              const uint32_t* len, const uint32_t* perm,
                                              uint64_t n, uint32_t extra, uint32_t slots,
                                              uint32_t cap8) {
  if (extra == 0 || quad_part_chains(count[0], nq_wg) != 0) return false;
  const uint64_t lines = chain_lines(len[perm[n - extra]]);
  return lines >= 16 && (uint64_t)extra * 8 <= (uint64_t)slots * cap8 &&
         (uint64_t)extra * relay_cap_div(lines) <= (uint64_t)slots * lines;
}

// Segment length of a descriptor relay: at least min_seg lines, about
// nseg_max segments for the longest relayed chain.
__device__ __forceinline__ uint32_t desc_relay_seg(const uint32_t* len, const uint32_t* perm,
                                                   uint64_t n, uint32_t extra, uint32_t nseg_max,
                                                   uint32_t min_seg) {
  const uint32_t lines = chain_lines(len[perm[n - extra]]);
  const uint32_t seg = ((lines + nseg_max - 1u) / nseg_max + 1u) & ~1u;
  return max(seg, min_seg);
}

// Lane regime (qmin == 0: desc_relay_on) or quad regime (qmin = the
// shortest chain worth relaying: desc_qrelay_on).
__device__ __forceinline__ bool desc_any_relay_on(const uint32_t* count, uint32_t nq_wg,
                                                  const uint32_t* len, const uint32_t* perm,
                                                  uint64_t n, uint32_t extra, uint32_t slots,
                                                  uint32_t qmin, uint32_t cap8) {
  return qmin ? desc_qrelay_on(count, len, perm, n, extra, qmin)
              : desc_relay_on(count, nq_wg, len, perm, n, extra, slots, cap8);
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_desc_relay(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ perm, uint64_t n,
    const uint32_t* count, uint32_t nq_wg, uint32_t extra, uint32_t slots, uint32_t ngroups,
    uint32_t nseg_max, uint32_t polls, uint32_t qmin, uint32_t min_seg, uint32_t cap8,
    uint32_t* flags, uint64_t* state, uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kQuadWaveLds];
  if (!desc_any_relay_on(count, nq_wg, len, perm, n, extra, slots, qmin, cap8)) return;
  const uint32_t g = blockIdx.x % ngroups, s = blockIdx.x / ngroups;
  const uint32_t seg = desc_relay_seg(len, perm, n, extra, nseg_max, min_seg);
  const RelayDesc r{arena, off, len, perm, n - extra, extra};
  // polls == 0: the bound from the longest chain (see launch_relay)
  const uint32_t lines = chain_lines(len[perm[n - extra]]);
  const uint32_t max_polls = polls ? polls : max(32768u, lines * 64u);
  relay_segment(r, g, s, (s + 1u) * seg, seg, flags, state, out, lds, max_polls, true);
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_desc_relay_finish(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ perm, uint64_t n,
    const uint32_t* count, uint32_t nq_wg, uint32_t extra, uint32_t slots, uint32_t nseg_max,
    uint32_t qmin, uint32_t min_seg, uint32_t cap8, uint32_t* flags, uint64_t* state,
    uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kQuadWaveLds];
  if (!desc_any_relay_on(count, nq_wg, len, perm, n, extra, slots, qmin, cap8)) return;
  const uint32_t g = blockIdx.x;
  const uint32_t s = __builtin_amdgcn_readfirstlane(flags[g]);
  const uint32_t seg = desc_relay_seg(len, perm, n, extra, nseg_max, min_seg);
  const RelayDesc r{arena, off, len, perm, n - extra, extra};
  if (s != 0xffffffffu)
    relay_segment(r, g, s, 0xffffffffu, seg, flags, state, out, lds, 0u, false);
  if (threadIdx.x == 0) flags[g] = 0;
}

__global__ __launch_bounds__(kThreads, 4) void k_lane_rest(const uint8_t* __restrict__ arena,
                                                            const uint64_t* __restrict__ off,
                                                            const uint32_t* __restrict__ len,
                                                            const uint32_t* __restrict__ perm,
                                                            uint64_t n, uint32_t* count,
                                                            uint32_t nq_wg, uint32_t pace,
                                                            uint32_t relay_extra, uint32_t slots,
                                                            uint32_t relay_cap8,
                                                            uint8_t* __restrict__ out) {
  // beside a relay: count this workgroup in (count[3]) for the relay's gate
  if (relay_extra && threadIdx.x == 0)
    __hip_atomic_fetch_add(count + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane_paced_wgs(count, nq_wg, pace) != 0) return;
  const uint32_t nl = quad_part_chains(count[0], nq_wg);
  const uint64_t j = nl + (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  // the last relay_extra chains are relayed (k_desc_relay) when it runs
  const uint64_t end = desc_relay_on(count, nq_wg, len, perm, n, relay_extra, slots, relay_cap8)
                           ? n - relay_extra
                           : n;
  if (j >= end) return;
  const uint32_t b = perm[j];
  uint64_t h[8];
  hash_chain_prefetch(arena + off[b], len[b], h);
  store_digest(out + (uint64_t)b * 32u, h);
}

// Paced lane part (helper == 0): only lane_paced_wgs() workgroups run, and
// waves claim tiles of 64 chains of the order from count[6]; the helper
// (helper == 1, queued behind the quad part on its stream) claims whatever
// the paced part left when the quad part ended, with the whole grid.  Both
// leave an unpaced batch to k_lane_rest.  The tile loop costs registers
// (120 VGPRs, 4 waves per SIMD): a lane-only batch through it ran 5.3 ms
// instead of 3.9.
__global__ __launch_bounds__(kThreads, 4) void k_lane_tiles(const uint8_t* __restrict__ arena,
                                                             const uint64_t* __restrict__ off,
                                                             const uint32_t* __restrict__ len,
                                                             const uint32_t* __restrict__ perm,
                                                             uint64_t n, uint32_t* count,
                                                             uint32_t nq_wg, uint32_t pace,
                                                             uint32_t helper,
                                                             uint8_t* __restrict__ out) {
  const uint64_t active = lane_paced_wgs(count, nq_wg, pace);
  if (active == 0 || (!helper && blockIdx.x >= active)) return;
  const uint32_t nl = count[0];  // every long chain is in the quad part
  // nothing left (the helper behind a paced part that finished): leave
  // without touching the tile counter, so thousands of idle waves do not
  // queue their atomics on one address (~0.18 ms at config 3)
  const uint32_t seen = __hip_atomic_load(count + 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (nl + (uint64_t)seen * 64u >= n) return;
  const uint32_t lane = threadIdx.x & 63u;
  for (;;) {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(count + 6, 1u);
    t = __builtin_amdgcn_readfirstlane(t);
    const uint64_t j0 = nl + (uint64_t)t * 64u;
    if (j0 >= n) break;
    const uint64_t j = j0 + lane;
    if (j < n) lane_chain(arena, off, len, perm[j], out);
  }
}

// Resumable single chain (the index footer, fed incrementally): one quad.
// st[0..7] = chain value, st[8] = bytes compressed so far.  After the final
// call st[0..3] is the digest.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_chain_step(uint64_t* __restrict__ st,
                                                   const uint8_t* __restrict__ data, uint32_t n,
                                                   int final) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[128];
  const uint32_t i = threadIdx.x;
  if (i >= 4) return;
  uint32_t addr[48];
  quad_addr(addr, 0u, i);
  const uint64_t t0 = st[8];
  uint64_t h0 = st[i], h1 = st[4 + i];
  if (t0 == 0 && st[9] == 0) quad_init(i, h0, h1);  // st[9] = 0: fresh state
  quad_single(h0, h1, t0, data, n, final != 0, lds, addr, i);
  st[i] = h0;
  st[4 + i] = h1;
  if (i == 0) {
    st[8] = t0 + n;
    st[9] = 1;
  }
}

hipError_t launch_chain_step(uint64_t* st, const uint8_t* data, uint32_t n, bool final,
                             hipStream_t s) {
  hipLaunchKernelGGL(k_chain_step, dim3(1), dim3(64), 0, s, st, data, n, final ? 1 : 0);
  return hipGetLastError();
}

// BlockHash::hash_bytes of one host buffer in one launch (the low-latency
// single-block path, src/block_id.rs:37-43 as called per received block at
// src/daemon/tracking/fetch_blocks.rs:77): the workgroup pulls the pinned,
// device-mapped host bytes over PCIe into device scratch (16-B vectors, four
// loads in flight per lane), then one quad hashes the chain from there
// (L2-resident, prefetched one line ahead) and writes the 32-byte digest
// straight into device-mapped host memory.  No staging copies, no ordering
// kernel, no D2H copy: one launch per call.  src == scratch: the bytes are
// already in device memory (inputs above kSinglePull, uploaded by SDMA, which
// moves them faster than one workgroup's PCIe reads).
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_single(
    const uint8_t* __restrict__ src, uint32_t n, uint8_t* __restrict__ scratch,
    uint8_t* __restrict__ dout) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[128];
  const uint32_t nv = src == scratch ? 0u : (n + 15u) >> 4;  // 16-B vectors to pull
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(scratch);
  for (uint32_t v = threadIdx.x; v < nv; v += 4u * kThreads) {
    uint4 r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t j = v + (uint32_t)k * kThreads;
      if (j < nv) r[k] = s4[j];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t j = v + (uint32_t)k * kThreads;
      if (j < nv) d4[j] = r[k];
    }
  }
  __threadfence_block();
  __syncthreads();
  const uint32_t i = threadIdx.x;
  if (i >= 4) return;
  __builtin_amdgcn_s_setprio(3);
  uint32_t addr[48];
  quad_addr(addr, 0u, i);
  uint64_t h0, h1;
  quad_init(i, h0, h1);
  quad_single(h0, h1, 0, scratch, n, true, lds, addr, i);
  reinterpret_cast<uint64_t*>(dout)[i] = h0;
}

hipError_t launch_single(const uint8_t* h_src, uint32_t n, uint8_t* d_scratch, uint8_t* h_out,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_single, dim3(1), dim3(kThreads), 0, s, h_src, n, d_scratch, h_out);
  return hipGetLastError();
}

// SHA-512/256 over a descriptor batch, one lane per block (dir-signature's
// HashType::sha512_256()).  5 waves per SIMD: the asm rounds need 93 VGPRs
// (the compiled ones 168, at 3 waves).
__global__ __launch_bounds__(kThreads, 5) void k_sha_desc(const uint8_t* __restrict__ arena,
                                                           const uint64_t* __restrict__ off,
                                                           const uint32_t* __restrict__ len,
                                                           const uint32_t* __restrict__ perm,
                                                           uint64_t n, uint8_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (j >= n) return;
  const uint64_t b = perm ? perm[j] : j;
  uint64_t h[8];
  sha::chain(arena + off[b], len[b], h);
  sha::store_digest_be(out + b * 32u, h);
}

hipError_t launch_sha_desc(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                           const uint32_t* perm, uint64_t n, uint8_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sha_desc, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, arena, off,
                     len, perm, n, out);
  return hipGetLastError();
}

// Register-only compressions (no memory traffic): `lines` compressions per
// lane on a message kept in registers -- the measured VALU ceiling the bench
// reports next to the HBM roofline (diagnostics, not part of the reference).
__global__ __launch_bounds__(kThreads, 4) void k_compress_only(uint8_t* __restrict__ out,
                                                              uint32_t lines) {
  const uint64_t b = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  uint64_t h[8], m[16];
  init_state(h);
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = b * 0x9e3779b97f4a7c15ULL + k;
  for (uint32_t i = 0; i < lines; ++i) {
    m[0] ^= i;  // keep the message live and varying (static index: no scratch)
    compress(h, m, (uint64_t)(i + 1) * 128u, i + 1 == lines);
  }
  store_digest(out + b * 32u, h);
}

hipError_t launch_compress_only(uint64_t nlanes, uint32_t lines, uint8_t* out, hipStream_t s) {
  if (nlanes == 0) return hipSuccess;
  hipLaunchKernelGGL(k_compress_only, dim3(grid_for(nlanes, kThreads)), dim3(kThreads), 0, s, out,
                     lines);
  return hipGetLastError();
}

// Daemon-side verify (fetch_blocks.rs:77 `hash_bytes(&data) == blk.hash`):
// one lane per digest, mismatches counted per wave with a ballot.
__global__ void k_verify(const uint8_t* __restrict__ got, const uint8_t* __restrict__ want,
                         uint64_t n, uint8_t* __restrict__ ok, uint32_t* __restrict__ nbad,
                         const uint8_t* __restrict__ flag) {
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool bad = false;
  if (b < n) {
    const uint4* g = reinterpret_cast<const uint4*>(got + 32 * b);
    const uint4* w = reinterpret_cast<const uint4*>(want + 32 * b);
    const uint4 g0 = g[0], g1 = g[1], w0 = w[0], w1 = w[1];
    const uint32_t diff = (g0.x ^ w0.x) | (g0.y ^ w0.y) | (g0.z ^ w0.z) | (g0.w ^ w0.w) |
                          (g1.x ^ w1.x) | (g1.y ^ w1.y) | (g1.z ^ w1.z) | (g1.w ^ w1.w);
    bad = diff != 0 || (flag && flag[b]);
    if (ok) ok[b] = bad ? 0 : 1;
  }
  const uint64_t mask = __ballot(bad);
  if (nbad && (threadIdx.x & 63) == 0 && mask) atomicAdd(nbad, (uint32_t)__popcll(mask));
}

hipError_t launch_verify(const uint8_t* got, const uint8_t* want, uint64_t n, uint8_t* ok,
                         uint32_t* nbad, hipStream_t s, const uint8_t* flag) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_verify, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, got, want, n,
                     ok, nbad, flag);
  return hipGetLastError();
}

__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t k) {
  uint64_t z = seed + (k + 1) * 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// Word k of the buffer.  block_words == 0: one splitmix64 stream over the
// whole buffer (word k = output k of splitmix64(seed)).  Otherwise every
// block of block_words words has its own stream seeded with
// seed ^ (first_block + block index)  (SURVEY.md 8d config 4).
__global__ void k_fill_splitmix64(uint64_t* __restrict__ p, uint64_t nwords, uint64_t seed,
                                  uint64_t block_words, uint64_t first_block) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nwords; k += stride) {
    uint64_t sd = seed, i = k;
    if (block_words) {
      sd = seed ^ (first_block + k / block_words);
      i = k % block_words;
    }
    p[k] = splitmix64_at(sd, i);
  }
}


hipError_t launch_uniform(Loader loader, const uint8_t* data, uint64_t bs, uint64_t nblk,
                          uint8_t* out, hipStream_t s) {
  if (nblk == 0) return hipSuccess;
  if (nblk % kThreads != 0 || bs % 128u != 0 || bs == 0) return hipErrorInvalidValue;
  const uint32_t lines = (uint32_t)(bs / 128u);
  if (loader == Loader::kGlds) {
    hipLaunchKernelGGL(k_uniform_glds, dim3(grid_for(nblk, kThreads)), dim3(kThreads), 0, s, data,
                       bs, lines, out);
  } else {
    hipLaunchKernelGGL(k_uniform_direct, dim3(grid_for(nblk, kThreads)), dim3(kThreads), 0, s,
                       data, bs, lines, out);
  }
  return hipGetLastError();
}

// SIMDs of the current device (4 per CU), cached per device (several host
// threads may ask at once: the cache slots are atomic).
static uint64_t device_simds() {
  static std::atomic<uint64_t> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1024;
  uint64_t v = cache[dev].load(std::memory_order_relaxed);
  if (v == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    v = 4ull * (uint64_t)cus;
    cache[dev].store(v, std::memory_order_relaxed);
  }
  return v;
}

// Does a chunk-form file of nblk blocks run every block in quad mode?  Lane
// mode holds 64 chains per wave, so its time steps with whole waves per SIMD:
// a file of 1 < w <= 1.625 lane waves per SIMD costs as much as w = 2 on the
// SIMDs that got two, while quad mode (16 chains per wave) grows smoothly.
// Measured after the hand-scheduled quad loop (profiles/r02/crossover.log,
// MI355X, 1024 SIMDs): 32 KiB x 81920 lane 1.94 ms / quad 1.67; x 98304
// 1.95 / 1.94; x 65536 lane 1.16 / quad 1.34; x 131072 lane 2.14 / quad 2.50;
// 256 KiB x 98304 lane 14.9 / quad 12.9.  Below 0.75 lane waves per SIMD
// (the small-batch limit) quad mode always.
static bool chunks_in_quad(uint64_t nblk, uint64_t bs) {
  if (bs < 128ull * kQuadSmallMinLines || bs > 0xffffffffull) return false;
  if (nblk < kQuadSmallBatch) return true;
  const uint64_t wave_slots = 64ull * device_simds();  // one lane wave per SIMD
  return nblk > wave_slots && nblk * 8 <= wave_slots * 13;
}

hipError_t launch_chunks(const uint8_t* data, uint64_t nbytes, uint64_t bs, uint8_t* out,
                         hipStream_t s) {
  if (nbytes == 0) return hipSuccess;
  if (bs == 0) return hipErrorInvalidValue;
  const uint64_t nblk = (nbytes + bs - 1) / bs;
  if (chunks_in_quad(nblk, bs)) {
    hipLaunchKernelGGL(k_quad_chunks<>, dim3((unsigned)((nblk + 63) / 64)), dim3(kThreads), 0, s,
                       data, nbytes, bs, (uint64_t)0, nblk, out);
    return hipGetLastError();
  }
  const bool uni_ok = bs % 128u == 0 && (reinterpret_cast<uintptr_t>(data) & 15u) == 0 &&
                      bs / 128u <= 0xffffffffull && bs <= 0xffffffffull / 8u;
  if (!uni_ok)  // misaligned base or bs % 128 != 0: every block ragged
    return launch_general_chunks(data, nbytes, bs, 0, nblk, out, s);
  const uint64_t nfull = nbytes / bs;
  const uint32_t ngen_wg = nfull < nblk ? 1u : 0u;  // the short last block
  const uint64_t grid = ngen_wg + grid_for(grid_for(nfull, 64), kWaves);
  if (grid > 0x7fffffffull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_chunks, dim3((unsigned)grid), dim3(kThreads), 0, s, data, nbytes, bs,
                     (uint32_t)(bs / 128u), nfull, ngen_wg, out);
  return hipGetLastError();
}

// launch_chunks with the short last block hashed in quad mode on qs,
// concurrently with the whole blocks on s.  One lane-mode chain of up to bs
// bytes without line prefetch runs ~25-35 % longer than a uniform wave's
// chains and trailed the launch; in quad mode it takes about a third of a
// lane-mode chain's time.  Forked from s (`fork`), joined back (`join`).
// Falls back to launch_chunks where the split does not apply.
// A relay aims at one segment wave per SIMD in total (kRelayTargetWaves x
// SIMDs).  Relays run up to 32 whole lane waves per SIMD (17 - 20 measured:
// 32 KiB x 1114113 blocks 2066-2070 -> 2193 GiB/s, x 1310721 2094-2099 ->
// 2193-2203, as descriptors +3-5 %; profiles/r02/relay/maxk/).
constexpr uint64_t kRelayMaxK = 32;
// With k >= 3 lane waves per SIMD the lane part is launched with
// kRelayLanePad bytes of extra LDS per workgroup: two k_chunks workgroups
// per CU (2 x 64 KiB of 160), so two lane waves per SIMD (2 x 112 VGPRs)
// leave room for a relay wave (244) -- three would not.
constexpr uint32_t kRelayLanePad = 32768;
// Quad-regime base (k_quad_chunks: 4 waves, 8 KiB static LDS): padded to
// 81 KiB per workgroup, one workgroup per CU, so one base wave per SIMD
// (248 VGPRs) beside a relay wave.
constexpr uint32_t kRelayQuadPad = 73 * 1024;
// Descriptor lane part (k_lane_rest, no LDS of its own) beside a relay:
// two workgroups per CU.
constexpr uint32_t kRelayDescLanePad = 64 * 1024;

// The lane-regime cap, in eighths of a lane wave per SIMD (relay_plan,
// desc_relay_on): beyond 5/8 one more lane wave costs less than the relayed
// chains' quad-mode work (profiles/r02/relay/).
constexpr uint64_t kRelayCap8 = 5;
// The k = 1 quad-regime relay's segments: its chain is as long as the
// base's and has no slack, so every hand-off adds to it (profiles/r02/relay/qshort/).
constexpr uint32_t kRelayQuad1Seg = 32;

// Quad regime: extra chains of up to 1/2 of a quad wave per SIMD relay
// (chunk form and descriptors); past 1/4 only chains of >= 128 lines
// (32 KiB x 24576 1283 -> 1535 GiB/s, 1 MiB x 24576 1301 -> 1690; 3/4 is no
// better than none: profiles/r02/relay/qfrac/).
static bool quad_relay_fits(uint64_t extra, uint64_t qslots) { return extra * 2 <= qslots; }
static uint32_t quad_relay_min_lines(uint64_t k, uint64_t extra, uint64_t qslots) {
  return extra * 4 > qslots ? 128u : (k == 1 ? 64u : 32u);
}

// How a chunk-form file of nfull whole blocks (+ maybe a short last one)
// splits when it relays: the first `base` blocks as whole waves on the
// caller's stream -- lane mode (k_chunks, quad == false) or quad mode
// (k_quad_chunks, quad == true) -- and blocks [base, base + nrel) relayed
// on the quad stream.  `pad`: extra LDS per base workgroup that keeps room
// for a relay wave (244 VGPRs) on every SIMD.
struct RelayPlan {
  uint64_t base = 0, nrel = 0;
  bool quad = false;
  uint32_t pad = 0;
  uint32_t min_seg = kRelayMinSegLines;  // shortest segment (lines)
  bool relay_first = false;              // enqueue the relay before the base
};

// Lane regime (nfull >= one lane wave per SIMD): k = 1 .. kRelayMaxK whole
// lane waves per SIMD plus extra blocks up to min(5/8, lines/32) of a lane
// wave per SIMD (relay_cap_div); beyond that one more lane wave (or the quad band of
// chunks_in_quad) costs less than the relayed chains' quad-mode work
// (profiles/r02/relay/).  Quad regime (below one lane wave per SIMD):
// k >= 1 whole quad waves per SIMD plus up to 1/2 of one (1/64 past the
// small-batch limit), chains of >= 64 lines at k = 1 (>= 32 above, >= 128
// past 1/4 of a wave: shorter relays cost more than they save).
// 16 <= lines, bs < 2^31.
static bool relay_plan(uint64_t nfull, uint64_t bs, RelayPlan& p) {
  p = RelayPlan();
  if (bs % 128u != 0 || bs < 128u * 16u || bs >= (1ull << 31)) return false;
  const uint64_t simds = device_simds(), lines = bs / 128u;
  const uint64_t lane_slots = 64ull * simds, quad_slots = 16ull * simds;
  if (nfull >= lane_slots) {
    const uint64_t k = nfull / lane_slots, extra = nfull % lane_slots;
    const uint64_t cap =
        std::min(lane_slots * kRelayCap8 / 8, lane_slots * lines / relay_cap_div(lines));
    if (k > kRelayMaxK || extra == 0 || extra > cap) return false;
    p.base = nfull - extra;
    p.nrel = extra;
    p.pad = k > 2 ? kRelayLanePad : 0u;
  } else {
    // short chains cost more hand-offs and launches than they save
    // (profiles/r02/relay/qshort/); past the small-batch limit (k = 3)
    // lane mode takes over from 1/64 of a quad wave of extra blocks on
    const uint64_t k = nfull / quad_slots, extra = nfull % quad_slots;
    if (extra == 0 || k < 1 || !quad_relay_fits(extra, quad_slots) ||
        lines < quad_relay_min_lines(k, extra, quad_slots) ||
        (nfull >= kQuadSmallBatch && extra * 64 > quad_slots))
      return false;
    p.base = nfull - extra;
    p.nrel = extra;
    p.quad = true;
    p.pad = kRelayQuadPad;
    // Beside quad-mode base waves the relay is enqueued first (the base is
    // short here) with 8-line segments; at k = 1 it has no slack at all (its
    // chain is as long as the base's and every hand-off adds to it): 32-line
    // segments (profiles/r02/relay/qshort/)
    p.min_seg = k == 1 ? kRelayQuad1Seg : kRelayMinSegLines;
    p.relay_first = true;
  }
  if ((p.nrel + kRelayGroupChains - 1) / kRelayGroupChains > kRelayMaxGroups) return false;
  return true;
}

uint64_t relay_blocks(uint64_t nfull, uint64_t bs) {
  RelayPlan p;
  return relay_plan(nfull, bs, p) ? p.nrel : 0;
}

static bool desc_may_relay_slots(uint64_t n, uint64_t slots) {
  return n >= slots && n / slots <= kRelayMaxK && n % slots != 0 &&
         (n % slots + kRelayGroupChains - 1) / kRelayGroupChains <= kRelayMaxGroups;
}

// Blocks [b0, b0 + nrel) of a file of whole bs-byte blocks as relayed quad
// chains on qs (the relay, then its finisher, which zeroes the flags
// again).  Segments of at least kRelayMinSegLines lines, as many as make
// ~one segment wave per SIMD.
static hipError_t launch_relay(const uint8_t* data, uint64_t bs, uint64_t b0, uint64_t nrel,
                               uint32_t min_seg, uint8_t* out, hipStream_t qs,
                               const RelayScratch& r) {
  const uint32_t lines = (uint32_t)(bs / 128u);
  const uint32_t groups = (uint32_t)((nrel + kRelayGroupChains - 1) / kRelayGroupChains);
  if (groups > r.groups) return hipErrorInvalidValue;
  const uint64_t target = device_simds();
  uint32_t nseg = (uint32_t)std::max<uint64_t>(1, target / groups);
  nseg = std::min(nseg, std::max(1u, lines / min_seg));
  uint32_t seg = ((lines + nseg - 1) / nseg + 1u) & ~1u;
  nseg = (lines + seg - 1) / seg;
  // each poll takes >= ~0.5 us (the sleep and an L2-missing load); a segment
  // waits at most for the chain before it (~1.1-2.5 us per line), so this
  // bound is never reached in a healthy run (CIR_RELAY_POLLS overrides it,
  // read per call: the finisher test)
  uint32_t max_polls = std::max<uint32_t>(32768u, lines * 64u);
  if (const char* v = getenv("CIR_RELAY_POLLS")) max_polls = (uint32_t)strtoul(v, nullptr, 10);
  hipLaunchKernelGGL(k_quad_relay, dim3(groups * nseg), dim3(64), 0, qs, data, bs, b0,
                     (uint32_t)nrel, groups, seg, r.flags, r.state, out, max_polls);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_quad_relay_finish, dim3(groups), dim3(64), 0, qs, data, bs, b0,
                     (uint32_t)nrel, seg, r.flags, r.state, out);
  return hipGetLastError();
}

hipError_t launch_chunks_split(const uint8_t* data, uint64_t nbytes, uint64_t bs, uint8_t* out,
                               hipStream_t s, hipStream_t qs, hipEvent_t fork, hipEvent_t join,
                               const RelayScratch* relay) {
  if (nbytes == 0) return hipSuccess;
  if (bs == 0) return hipErrorInvalidValue;
  const uint64_t nblk = (nbytes + bs - 1) / bs;
  const uint64_t nfull = nbytes / bs;
  const bool uni_ok = bs % 128u == 0 && (reinterpret_cast<uintptr_t>(data) & 15u) == 0 &&
                      bs / 128u <= 0xffffffffull && bs <= 0xffffffffull / 8u;
  const uint64_t grid = grid_for(grid_for(nfull, 64), kWaves);
  RelayPlan plan;
  if (relay && relay->flags && qs && qs != s && uni_ok && relay_plan(nfull, bs, plan)) {
    // k whole lane (or quad) waves per SIMD on s; the extra whole blocks
    // relayed and the short last block (if any) in quad mode, both on qs.
    // The longer part is enqueued first, so it starts first: the base, or
    // the relay when its chain is as long as the base's (quad regime, k = 1).
    hipError_t e = hipEventRecord(fork, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(qs, fork, 0);
    if (e != hipSuccess) return e;
    auto base = [&]() -> hipError_t {
      if (plan.quad)
        hipLaunchKernelGGL(k_quad_chunks<true>, dim3((unsigned)grid_for(plan.base, 64)),
                           dim3(kThreads), plan.pad, s, data, nbytes, bs, (uint64_t)0, plan.base,
                           out);
      else
        hipLaunchKernelGGL(k_chunks, dim3((unsigned)grid_for(grid_for(plan.base, 64), kWaves)),
                           dim3(kThreads), plan.pad, s, data, nbytes, bs, (uint32_t)(bs / 128u),
                           plan.base, 0u, out);
      return hipGetLastError();
    };
    auto rest = [&]() -> hipError_t {
      if (nfull < nblk) {
        hipLaunchKernelGGL(k_quad_chunks<>, dim3(1), dim3(kThreads), 0, qs, data, nbytes, bs,
                           nfull, nblk, out);
        const hipError_t e2 = hipGetLastError();
        if (e2 != hipSuccess) return e2;
      }
      return launch_relay(data, bs, plan.base, plan.nrel, plan.min_seg, out, qs, *relay);
    };
    e = plan.relay_first ? rest() : base();
    if (e == hipSuccess) e = plan.relay_first ? base() : rest();
    if (e == hipSuccess) e = hipEventRecord(join, qs);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, join, 0);
    return e;
  }
  if (!qs || qs == s || chunks_in_quad(nblk, bs) || !uni_ok || nfull == nblk ||
      bs < 128ull * kQuadSmallMinLines || grid > 0x7fffffffull)
    return launch_chunks(data, nbytes, bs, out, s);
  hipError_t e = hipEventRecord(fork, s);
  if (e == hipSuccess) e = hipStreamWaitEvent(qs, fork, 0);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_quad_chunks<>, dim3(1), dim3(kThreads), 0, qs, data, nbytes, bs, nfull, nblk,
                     out);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_chunks, dim3((unsigned)grid), dim3(kThreads), 0, s, data, nbytes, bs,
                     (uint32_t)(bs / 128u), nfull, 0u, out);
  e = hipGetLastError();
  if (e == hipSuccess) e = hipEventRecord(join, qs);
  if (e == hipSuccess) e = hipStreamWaitEvent(s, join, 0);
  return e;
}

hipError_t launch_general_chunks(const uint8_t* data, uint64_t nbytes, uint64_t bs,
                                 uint64_t first, uint64_t n, uint8_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_general, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, data, nbytes,
                     bs, first, (const uint64_t*)nullptr, (const uint32_t*)nullptr,
                     (const uint32_t*)nullptr, n, out);
  return hipGetLastError();
}

hipError_t launch_general_desc(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                               const uint32_t* perm, uint64_t n, uint8_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_general, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, arena,
                     (uint64_t)0, (uint64_t)0, (uint64_t)0, off, len, perm, n, out);
  return hipGetLastError();
}


// The descriptor relay (k_desc_relay + its finisher) of the last `extra`
// chains of an ordered batch on stream st; the kernels decide on the device
// whether it runs (qmin == 0: lane regime, else quad regime).
static hipError_t launch_desc_relay(const uint8_t* arena, const uint64_t* off,
                                    const uint32_t* len, const uint32_t* perm, uint64_t n,
                                    uint32_t* n_long, uint32_t nq, uint32_t extra,
                                    uint32_t slots, uint32_t groups, uint32_t nseg_max,
                                    uint32_t qmin, uint32_t min_seg, uint32_t cap8,
                                    uint32_t gate_target, const RelayScratch& r, uint8_t* out,
                                    hipStream_t st) {
  uint32_t polls = 0;  // 0: the device's bound; CIR_RELAY_POLLS=0: give up at once
  if (const char* v = getenv("CIR_RELAY_POLLS"))
    polls = std::max(1u, (uint32_t)strtoul(v, nullptr, 10));
  if (gate_target) {
    // the relay's waves go in after the lane workgroups hold their CUs
    // (count[3], bounded wait), so they take the room the lane part's
    // padding leaves instead of taking the SIMDs first
    hipLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, st, n_long + 3, gate_target, 600u);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_desc_relay, dim3(groups * nseg_max), dim3(64), 0, st, arena, off, len,
                     perm, n, n_long, nq, extra, slots, groups, nseg_max, polls, qmin, min_seg,
                     cap8, r.flags, r.state, out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_desc_relay_finish, dim3(groups), dim3(64), 0, st, arena, off, len, perm, n,
                     n_long, nq, extra, slots, nseg_max, qmin, min_seg, cap8, r.flags, r.state,
                     out);
  return hipGetLastError();
}

hipError_t launch_mixed(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                        const uint32_t* perm, uint32_t* n_long, uint64_t n, uint8_t* out,
                        hipStream_t s, hipStream_t qs, hipEvent_t fork, hipEvent_t qjoin,
                        const RelayScratch* relay, const hipEvent_t* tev) {
  if (n == 0) return hipSuccess;
  // tev (diagnostics): quad part start / end on its stream, lane part start /
  // end on s (the lane part's kernels after the gate)
  auto mark = [&](int k, hipStream_t st) {
    return tev ? hipEventRecord(tev[k], st) : hipSuccess;
  };
  // a relay of the chains past k whole lane waves per SIMD (desc_relay_on
  // decides on the device whether it runs)
  const uint64_t slots = 64ull * device_simds();
  // the most a lane-regime relay takes, in eighths of a lane wave per SIMD
  const uint32_t cap8 = (uint32_t)kRelayCap8;
  uint32_t extra = 0, groups = 0, nseg_max = 1;
  if (relay && relay->flags && qs != s && desc_may_relay_slots(n, slots)) {
    extra = (uint32_t)(n % slots);
    groups = (extra + kRelayGroupChains - 1) / kRelayGroupChains;
    if (groups > relay->groups) {
      extra = 0;
    } else {
      nseg_max = (uint32_t)std::max<uint64_t>(1, device_simds() / groups);
    }
  }
  const uint64_t nq = std::min<uint64_t>((n + 63) / 64, quad_max_wg(n));
  const uint64_t lane_grid = grid_for(n, kThreads);
  if (lane_grid > 0x7fffffffull) return hipErrorInvalidValue;
  const uint32_t pace = qs != s ? kLanePace : 0u;  // only beside a concurrent quad part
  const bool exclusive = n >= kQuadSmallBatch;
  // small batch: a relay of the chains past k whole quad waves per SIMD
  // (desc_qrelay_on decides on the device)
  const uint64_t qslots = 16ull * device_simds();
  uint32_t qextra = 0;
  // (a relay runs only on the device's own quad-part stream, never on the
  // caller's: relays share the device's scratch, one stream orders them)
  if (!exclusive && relay && relay->flags && qs != s &&
      n >= qslots &&
      n % qslots != 0 && quad_relay_fits(n % qslots, qslots))
    qextra = (uint32_t)(n % qslots);
  // Small batches run both parts on s, one after the other (the lane part
  // holds only chains of < 8 lines): qs only carries a relay, and without
  // one the fork to qs and the join back cost ~25 us of a 0.4 ms batch
  // (32 KiB x 16384, profiles/r02/desc/serial/)
  const bool serial = !exclusive && n < kQuadSmallBatch && qextra == 0;
  const bool qs_used = qs != s && !serial;
  hipError_t e = hipEventRecord(fork, s);
  if (e == hipSuccess && qs_used) e = hipStreamWaitEvent(qs, fork, 0);
  if (e != hipSuccess) return e;
  if (exclusive) {
    // The quad workgroups need whole CUs (one 504-register wave per SIMD):
    // they are dispatched first, and the lane part starts once all of them
    // hold their CUs (k_gate), so its waves fill the other CUs instead of
    // taking every SIMD first.
    e = mark(0, qs);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_quad_long<true>), dim3((unsigned)nq), dim3(kThreads), 0, qs,
                       arena, off, len, perm, n_long, (uint32_t)nq, out, n, 0u, 0u);
    e = hipGetLastError();
    if (e == hipSuccess) e = mark(1, qs);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, s, n_long + 1, (uint32_t)nq, 600u);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    // unpaced batches: k_lane_rest; paced ones: k_lane_tiles (each leaves
    // the other case at once), and the helper behind the quad part
    if (extra) {
      // on qs behind the quad part (which is empty whenever the relay runs)
      const uint64_t lane_wgs = std::min<uint64_t>(lane_grid, 2ull * device_simds() / 4ull);
      e = launch_desc_relay(arena, off, len, perm, n, n_long, (uint32_t)nq, extra,
                            (uint32_t)slots, groups, nseg_max, 0u, kRelayMinSegLines, cap8,
                            (uint32_t)lane_wgs, *relay, out,
                            qs);
      if (e != hipSuccess) return e;
    }
    // beside a relay at most two lane waves per SIMD (2 x 128 VGPRs, two
    // 64 KiB-padded workgroups per CU), so a relay wave (244) always fits;
    // the lane body is issue-bound, two waves per SIMD run it as fast
    e = mark(2, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lane_rest, dim3((unsigned)lane_grid), dim3(kThreads),
                       extra ? kRelayDescLanePad : 0u, s, arena, off, len, perm, n, n_long,
                       (uint32_t)nq, pace, extra, (uint32_t)slots, cap8, out);
    if (pace != 0) {
      e = hipGetLastError();
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(k_lane_tiles, dim3((unsigned)lane_grid), dim3(kThreads), 0, s, arena,
                         off, len, perm, n, n_long, (uint32_t)nq, pace, 0u, out);
      e = hipGetLastError();
      if (e == hipSuccess) e = mark(3, s);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(k_lane_tiles, dim3((unsigned)lane_grid), dim3(kThreads), 0, qs, arena,
                         off, len, perm, n, n_long, (uint32_t)nq, pace, 1u, out);
    } else {
      e = hipGetLastError();
      if (e == hipSuccess) e = mark(3, s);
      if (e != hipSuccess) return e;
    }
  } else {
    // Every relay runs on qs (they share the device's relay scratch, so one
    // stream orders them); the quad part runs on the lane part's stream (the
    // caller's) after the lane part, which is empty whenever
    // the relay runs, padded to one workgroup per CU beside a relay to leave
    // room for the relay's waves.
    uint32_t qmin = 0;
    if (qextra) {
      const uint32_t qgroups = (qextra + kRelayGroupChains - 1) / kRelayGroupChains;
      const uint32_t qk = (uint32_t)(n / qslots);
      qmin = quad_relay_min_lines(qk, qextra, qslots);
      const uint32_t qnseg =
          (uint32_t)std::max<uint64_t>(1, device_simds() / qgroups);
      e = launch_desc_relay(arena, off, len, perm, n, n_long, (uint32_t)nq, qextra,
                            (uint32_t)qslots, qgroups, qnseg, qmin,
                            qk == 1 ? kRelayQuad1Seg : kRelayMinSegLines, 0u, 0u, *relay,
                            out, qs);
      if (e != hipSuccess) return e;
    }
    e = mark(2, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lane_rest, dim3((unsigned)lane_grid), dim3(kThreads), 0, s, arena, off,
                       len, perm, n, n_long, (uint32_t)nq, 0u, 0u, (uint32_t)slots, 0u, out);
    e = hipGetLastError();
    if (e == hipSuccess) e = mark(3, s);
    if (e != hipSuccess) return e;
    e = mark(0, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_quad_long<false>), dim3((unsigned)nq), dim3(kThreads),
                       qextra ? kRelayQuadPad : 0u, s, arena, off, len, perm, n_long,
                       (uint32_t)nq, out, n, qextra, qmin);
    e = hipGetLastError();
    if (e == hipSuccess) e = mark(1, s);
    if (e != hipSuccess) return e;
  }
  e = hipGetLastError();
  if (e == hipSuccess && qs_used) e = hipEventRecord(qjoin, qs);
  if (e == hipSuccess && qs_used) e = hipStreamWaitEvent(s, qjoin, 0);
  return e;
}

// The device's own clocks, read by one wave: the constant-rate wall clock
// (s_memrealtime) and the shader clock counter (s_memtime) before and after
// a spin of `spin` wall-clock ticks (bounded by an iteration cap, so the wave
// always ends).  Lanes 0-3 store rt0, rt1, c0, c1 with per-lane addresses.
__global__ void k_clock_probe(uint64_t* __restrict__ out, uint64_t spin) {
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  uint64_t rt1 = rt0;
  for (uint32_t it = 0; it < (1u << 22) && rt1 - rt0 < spin; ++it)
    rt1 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  const unsigned l = threadIdx.x;
  if (l < 4) out[l] = l == 0 ? rt0 : l == 1 ? rt1 : l == 2 ? c0 : c1;
}

hipError_t launch_clock_probe(uint64_t* out, uint64_t spin, hipStream_t s) {
  hipLaunchKernelGGL(k_clock_probe, dim3(1), dim3(64), 0, s, out, spin);
  return hipGetLastError();
}

hipError_t launch_fill_splitmix64(uint64_t* p, uint64_t nwords, uint64_t seed,
                                  uint64_t block_words, uint64_t first_block, hipStream_t s) {
  if (nwords == 0) return hipSuccess;
  uint64_t grid = (nwords + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(k_fill_splitmix64, dim3((unsigned)grid), dim3(256), 0, s, p, nwords, seed,
                     block_words, first_block);
  return hipGetLastError();
}

}  // namespace dev
}  // namespace cir
