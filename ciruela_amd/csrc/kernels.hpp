// Host-side launchers for the gfx950 kernels in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cir {
namespace dev {

constexpr int kThreads = 256;  // 4 waves per workgroup

enum class Loader : int { kGlds = 0, kDirect = 1 };

// nblk equal blocks of bs bytes at data (bs % 128 == 0, data 16-byte aligned,
// nblk % 256 == 0).  out: nblk x 32 bytes.
hipError_t launch_uniform(Loader loader, const uint8_t* data, uint64_t bs, uint64_t nblk,
                          uint8_t* out, hipStream_t s);

// Hashes::hash_file on one device-resident file: ceil(nbytes / bs) blocks, the
// last one short, digest i -> out + 32 i.  One launch (uniform body through
// LDS-DMA when bs % 128 == 0 and data is 16-byte aligned, ragged rest fused).
hipError_t launch_chunks(const uint8_t* data, uint64_t nbytes, uint64_t bs, uint8_t* out,
                         hipStream_t s);

// Blocks first .. first+n-1 of Hashes::hash_file's split of [data, data+nbytes).
hipError_t launch_general_chunks(const uint8_t* data, uint64_t nbytes, uint64_t bs,
                                 uint64_t first, uint64_t n, uint8_t* out, hipStream_t s);

// Per-descriptor BlockHash::hash_bytes; digest of block b goes to out + 32*b.
// perm (nullable) is the processing order (a permutation of 0..n-1).
hipError_t launch_general_desc(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                               const uint32_t* perm, uint64_t n, uint8_t* out, hipStream_t s);

// Longest-chain-first order of a descriptor batch (order.hip): *perm points
// into `scratch` (order_scratch_bytes(n) bytes, device memory).
size_t order_scratch_bytes(uint64_t n);
hipError_t launch_order_desc(const uint32_t* len, uint64_t n, void* scratch, size_t bytes,
                             uint32_t** perm, hipStream_t s);

hipError_t launch_fill_splitmix64(uint64_t* p, uint64_t nwords, uint64_t seed,
                                  uint64_t block_words, uint64_t first_block, hipStream_t s);

}  // namespace dev
}  // namespace cir
