// Processing order of a mixed-length descriptor batch (config 3).
//
// One lane hashes one block, so a wave costs as much as its longest chain.
// Sorting descriptors by compression count (descending) puts chains of equal
// length in the same waves and dispatches the longest ones first, so they
// overlap with the short ones instead of trailing the launch.  The sort runs
// on the device (hipCUB radix sort on 16-bit keys) inside the timed call.
#include <hipcub/hipcub.hpp>

#include "kernels.hpp"

namespace cir {
namespace dev {

constexpr int kKeyBits = 16;  // k_chain_keys' key width

__global__ void k_chain_keys(const uint32_t* __restrict__ len, uint64_t n, uint32_t min_lines,
                             uint16_t* __restrict__ key, uint32_t* __restrict__ idx,
                             uint32_t* __restrict__ count) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t l = len[i];
  const uint32_t k = l == 0 ? 1u : (l >> 7) + ((l & 127u) != 0);  // compressions, <= 2^25
  // 16-bit sort key, monotone in k: exact below 32768 lines (4 MiB), then
  // steps of 1024 lines (128 KiB) up to 2^25 lines.  With 2-byte keys
  // rocPRIM sorts batches above 100 K items by onesweep (~4 launches); with
  // 4-byte keys it chose block sort + merge sort up to 1 M items (~21
  // launches).  The launches, not the work, dominate the ordering: ~7 us
  // each, ~45 us each with several contexts' queues in one process
  // (profiles/r02/gtrace*).
  key[i] = (uint16_t)(k < 32768u ? k : 32768u + ((k - 32768u) >> 10));
  idx[i] = (uint32_t)i;
  // count[0] = long chains, count[2] = the longest chain (compressions),
  // count[4..5] = the lane part's work (launch_mixed's pacing): compressions
  // plus kLaneChainCost per chain for its setup and digest store
  if (k >= min_lines) {
    atomicAdd(count, 1u);
  } else {
    atomicAdd(reinterpret_cast<unsigned long long*>(count + 4),
              (unsigned long long)(k + kLaneChainCost));
  }
  atomicMax(count + 2, k);
}

size_t order_scratch_bytes(uint64_t n) {
  size_t temp = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, temp, (const uint16_t*)nullptr,
                                                     (uint16_t*)nullptr, (const uint32_t*)nullptr,
                                                     (uint32_t*)nullptr, (int)n, 0, kKeyBits);
  return 256 + ((temp + 255) & ~(size_t)255) + 4 * ((n * 4 + 255) & ~(uint64_t)255);
}

hipError_t launch_order_desc(const uint32_t* len, uint64_t n, void* scratch, size_t bytes,
                             uint32_t** perm, uint32_t** n_long, hipStream_t s) {
  const uint64_t arr = (n * 4 + 255) & ~(uint64_t)255;
  uint32_t* count = static_cast<uint32_t*>(scratch);
  uint8_t* p = static_cast<uint8_t*>(scratch) + 256;
  bytes -= 256;
  // count[0] = n_long; count[1] = quad workgroups started (launch_mixed's
  // gate); count[2] = longest chain; count[4..5] = lane work (k_chain_keys)
  hipError_t e0 = hipMemsetAsync(count, 0, 32, s);
  if (e0 != hipSuccess) return e0;
  *n_long = count;
  uint16_t* key_in = reinterpret_cast<uint16_t*>(p);
  uint16_t* key_out = reinterpret_cast<uint16_t*>(p + arr);
  uint32_t* idx_in = reinterpret_cast<uint32_t*>(p + 2 * arr);
  uint32_t* idx_out = reinterpret_cast<uint32_t*>(p + 3 * arr);
  void* temp = p + 4 * arr;
  size_t temp_bytes = bytes - 4 * arr;
  hipLaunchKernelGGL(k_chain_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, len, n,
                     quad_min_lines(n), key_in, idx_in, count);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (n == 1) {  // one chain (hash_bytes, an index footer): nothing to order
    *perm = idx_in;
    return hipSuccess;
  }
  e = hipcub::DeviceRadixSort::SortPairsDescending(temp, temp_bytes, key_in, key_out, idx_in,
                                                   idx_out, (int)n, 0, kKeyBits, s);
  *perm = idx_out;
  return e;
}

}  // namespace dev
}  // namespace cir
