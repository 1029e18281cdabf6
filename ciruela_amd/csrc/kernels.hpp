// Host-side launchers for the gfx950 kernels in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cir {
namespace dev {

constexpr int kThreads = 256;  // 4 waves per workgroup

enum class Loader : int { kGlds = 0, kDirect = 1 };

// Chains of at least this many 128-B lines (128 KiB) run 4 lanes per chain.
// config 3 A/B (profiles/r01/cfg3_quad_threshold.log): 2048 lines 659 GiB/s,
// 1024 782, 512 760, 256 769 -- below 2048, the ragged 1 MiB blocks no
// longer trail the lane kernel.
constexpr uint32_t kQuadMinLines = 1024;
constexpr int kQuadMaxWg = 256;  // at most 256 x 64 = 16384 chains in quad mode

// Small batches: lane mode is latency-bound below about one wave per SIMD
// (64 x 1024 = 65536 chains; lane mode measured 2232 GiB/s at 8 M x 4 KiB
// but 1024 GiB/s at 32 K x 1 MiB and 258 at 8 K x 4 MiB).  Batches of at
// most 49152 chains run every chain of at least kQuadSmallMinLines lines in
// quad mode (4 x the waves, ~1/3 the latency per compression): 1648-1700
// GiB/s at 32 K x 1 MiB, 757-784 at 8 K x 4 MiB (asm quad G).  The two
// modes cross at ~49152 chains (within 4 % there at 32 KiB, 256 KiB and
// 1 MiB); at 65535 lane mode is ahead (1606 vs 1438 GiB/s at 32 KiB, 1916
// vs 1703 at 256 KiB; profiles/r01/quad_asm_ab.md).
constexpr uint64_t kQuadSmallBatch = 49153;
constexpr uint32_t kQuadSmallMinLines = 8;
inline uint32_t quad_min_lines(uint64_t n) {
  return n < kQuadSmallBatch ? kQuadSmallMinLines : kQuadMinLines;
}
inline uint64_t quad_max_wg(uint64_t n) {
  return n < kQuadSmallBatch ? (n + 63) / 64 : (uint64_t)kQuadMaxWg;
}

// nblk equal blocks of bs bytes at data (bs % 128 == 0, data 16-byte aligned,
// nblk % 256 == 0).  out: nblk x 32 bytes.
hipError_t launch_uniform(Loader loader, const uint8_t* data, uint64_t bs, uint64_t nblk,
                          uint8_t* out, hipStream_t s);

// Hashes::hash_file on one device-resident file: ceil(nbytes / bs) blocks, the
// last one short, digest i -> out + 32 i.  One launch (uniform body through
// LDS-DMA when bs % 128 == 0 and data is 16-byte aligned, ragged rest fused).
hipError_t launch_chunks(const uint8_t* data, uint64_t nbytes, uint64_t bs, uint8_t* out,
                         hipStream_t s);

// Device scratch of the relays (k_quad_relay, k_desc_relay): a flag and
// 64 x 16 B of chain values per group of 16 chains (one quad-mode wave).
// Every relay runs on the device's quad-part stream (qs), so relays of
// different calls are ordered by that one stream.
struct RelayScratch {
  uint32_t* flags = nullptr;
  uint64_t* state = nullptr;
  uint32_t groups = 0;  // capacity
};
constexpr uint32_t kRelayMaxGroups = 4096;
inline size_t relay_scratch_bytes(uint32_t groups) { return (size_t)groups * (4 + 64 * 16); }

// launch_chunks with the ragged rest in quad mode on qs, concurrently with
// the uniform part on s (fork / join events); a file of k whole lane waves
// per SIMD plus a few blocks runs the extra blocks as relayed
// quad chains on qs (relay, when given); launch_chunks where neither
// applies (small or misaligned files, no rest, qs null or == s).
hipError_t launch_chunks_split(const uint8_t* data, uint64_t nbytes, uint64_t bs, uint8_t* out,
                               hipStream_t s, hipStream_t qs, hipEvent_t fork, hipEvent_t join,
                               const RelayScratch* relay = nullptr);
// Number of blocks launch_chunks_split would relay (0: no relay) for a file
// of nfull whole blocks of bs bytes on the current device.
uint64_t relay_blocks(uint64_t nfull, uint64_t bs);

// Blocks first .. first+n-1 of Hashes::hash_file's split of [data, data+nbytes).
hipError_t launch_general_chunks(const uint8_t* data, uint64_t nbytes, uint64_t bs,
                                 uint64_t first, uint64_t n, uint8_t* out, hipStream_t s);

// Per-descriptor BlockHash::hash_bytes; digest of block b goes to out + 32*b.
// perm (nullable) is the processing order (a permutation of 0..n-1).
hipError_t launch_general_desc(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                               const uint32_t* perm, uint64_t n, uint8_t* out, hipStream_t s);

// Descriptor batch in the order perm (longest chain first); the first
// *n_long chains (device count) run in quad mode when 64 * quad_max_wg(n) hold them, on
// qs, the rest one lane per chain on s; the quad part forks from s (`fork`)
// and joins back into it (`qjoin`).
// relay (nullable): scratch for relaying the chains past k whole lane (or
// quad) waves per SIMD (k_desc_relay; decided on the device).
// tev (nullable, diagnostics): 4 timing events recorded around the quad
// part (0, 1; on its stream) and the lane part (2, 3; on s).
hipError_t launch_mixed(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                        const uint32_t* perm, uint32_t* n_long, uint64_t n, uint8_t* out,
                        hipStream_t s, hipStream_t qs, hipEvent_t fork, hipEvent_t qjoin,
                        const RelayScratch* relay = nullptr,
                        const hipEvent_t* tev = nullptr);

// Longest-chain-first order of a descriptor batch (order.hip): *perm points
// into `scratch` (order_scratch_bytes(n) bytes, device memory).
size_t order_scratch_bytes(uint64_t n);
// *n_long = number of chains with >= quad_min_lines(n) lines (device memory);
// (*n_long)[1] = 0, the started-workgroup counter of the quad part;
// (*n_long)[2] = the longest chain's compressions; (*n_long)[4..5] (u64) =
// the other chains' compressions + kLaneChainCost each.
constexpr uint32_t kLaneChainCost = 4;
hipError_t launch_order_desc(const uint32_t* len, uint64_t n, void* scratch, size_t bytes,
                             uint32_t** perm, uint32_t** n_long, hipStream_t s);

// Bounds of an untrusted descriptor batch (order.hip): in `scratch`
// (bound_scratch_bytes(n) bytes of device memory) *slen = the lengths with
// every out-of-range block's set to 0 (off + len wraps or passes
// arena_bytes), *flag = 1 per out-of-range block; *nflag (device u32, zeroed
// here; NULL: a counter inside the scratch) = their number.
size_t bound_scratch_bytes(uint64_t n);
hipError_t launch_desc_bound(const uint64_t* off, const uint32_t* len, uint64_t n,
                             uint64_t arena_bytes, void* scratch, uint32_t* nflag,
                             uint32_t** slen, uint8_t** flag, hipStream_t s);
// out + 32 b = 32 zero bytes for every flagged block b.
hipError_t launch_desc_zero(const uint8_t* flag, uint64_t n, uint8_t* out, hipStream_t s);

// SHA-512/256 per descriptor (one lane per block), digest b -> out + 32 b.
hipError_t launch_sha_desc(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                           const uint32_t* perm, uint64_t n, uint8_t* out, hipStream_t s);

// Resumable single-chain BLAKE2b-256 (quad mode).  st: 16 x u64 of device
// memory, zeroed before the first call.  Non-final calls take a multiple of
// 128 bytes; the final call takes the rest (>= 1 byte unless the whole input
// is empty) and leaves the digest in st[0..3].
hipError_t launch_chain_step(uint64_t* st, const uint8_t* data, uint32_t n, bool final,
                             hipStream_t s);

// One BLAKE2b-256 chain over n bytes of device-mapped pinned host memory
// h_src (16-B aligned, readable up to n rounded up to 16), staged through
// d_scratch (same rounding) by the kernel itself; the digest is written to
// device-mapped host memory h_out (32 B).  One launch, nothing else.
hipError_t launch_single(const uint8_t* h_src, uint32_t n, uint8_t* d_scratch, uint8_t* h_out,
                         hipStream_t s);

// Compare n digests (32 B each, both 16-B aligned) with the expected ones:
// ok[b] = 1 / 0 (ok may be null); *nbad += mismatches (nbad may be null).
// flag (nullable): a flagged block is a mismatch whatever its digest.
hipError_t launch_verify(const uint8_t* got, const uint8_t* want, uint64_t n, uint8_t* ok,
                         uint32_t* nbad, hipStream_t s, const uint8_t* flag = nullptr);

// nlanes x `lines` register-only compressions (diagnostic VALU ceiling).
hipError_t launch_compress_only(uint64_t nlanes, uint32_t lines, uint8_t* out, hipStream_t s);

// one wave reads the device's wall clock and shader clock counters around a
// spin of `spin` wall-clock ticks: out[0..3] = rt0, rt1, c0, c1 (device memory)
hipError_t launch_clock_probe(uint64_t* out, uint64_t spin, hipStream_t s);
hipError_t launch_fill_splitmix64(uint64_t* p, uint64_t nwords, uint64_t seed,
                                  uint64_t block_words, uint64_t first_block, hipStream_t s);

}  // namespace dev
}  // namespace cir
