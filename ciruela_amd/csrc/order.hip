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

// Key, identity index and (for chains of >= min_lines lines) an entry in
// the long-chain list of every descriptor.  The list is appended per wave
// (one atomic per wave, positions by popcount), so its order is arbitrary;
// count[0] ends as the number of long chains.
__global__ void k_chain_keys(const uint32_t* __restrict__ len, uint64_t n, uint32_t min_lines,
                             uint16_t* __restrict__ key, uint32_t* __restrict__ idx,
                             uint32_t* __restrict__ count, uint32_t* __restrict__ long_list) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool lng = false;
  if (i < n) {
    const uint32_t l = len[i];
    const uint32_t k = l == 0 ? 1u : (l >> 7) + ((l & 127u) != 0);  // compressions, <= 2^25
    // 16-bit sort key, monotone in k: exact below 32768 lines (4 MiB), then
    // steps of 1024 lines (128 KiB) up to 2^25 lines.  With 2-byte keys
    // rocPRIM sorts batches above 100 K items by onesweep (~4 launches); with
    // 4-byte keys it chose block sort + merge sort up to 1 M items (~21
    // launches).  The launches, not the work, dominate the ordering: ~7 us
    // each, ~45 us each with several contexts' queues in one process
    // (profiles/r02/traces/).
    key[i] = (uint16_t)(k < 32768u ? k : 32768u + ((k - 32768u) >> 10));
    idx[i] = (uint32_t)i;
    lng = k >= min_lines;
  }
  const uint64_t mask = __ballot(lng);
  if (mask == 0) return;
  const uint32_t lane = __lane_id();
  const int leader = __ffsll((unsigned long long)mask) - 1;
  uint32_t base = 0;
  if ((int)lane == leader) base = atomicAdd(count, (uint32_t)__popcll(mask));
  base = (uint32_t)__shfl((int)base, leader);
  if (lng) long_list[base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull))] = (uint32_t)i;
}

// scratch: 256 B of counters, then five n-entry arrays (keys in/out, index
// in/out, long list), then the sort's temporary storage.
size_t order_scratch_bytes(uint64_t n) {
  size_t temp = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, temp, (const uint16_t*)nullptr,
                                                     (uint16_t*)nullptr, (const uint32_t*)nullptr,
                                                     (uint32_t*)nullptr, (int)n, 0, kKeyBits);
  return 256 + ((temp + 255) & ~(size_t)255) + 5 * ((n * 4 + 255) & ~(uint64_t)255);
}

static void order_layout(void* scratch, uint64_t n, OrderView* ov) {
  const uint64_t arr = (n * 4 + 255) & ~(uint64_t)255;
  uint8_t* p = static_cast<uint8_t*>(scratch) + 256;
  ov->count = static_cast<uint32_t*>(scratch);
  ov->key_in = reinterpret_cast<uint16_t*>(p);
  ov->key_out = reinterpret_cast<uint16_t*>(p + arr);
  ov->idx_in = reinterpret_cast<uint32_t*>(p + 2 * arr);
  ov->idx_out = reinterpret_cast<uint32_t*>(p + 3 * arr);
  ov->long_list = reinterpret_cast<uint32_t*>(p + 4 * arr);
  ov->temp = p + 5 * arr;
  ov->n = n;
}

hipError_t launch_order_keys(const uint32_t* len, uint64_t n, void* scratch, size_t bytes,
                             OrderView* ov, hipStream_t s) {
  (void)bytes;
  order_layout(scratch, n, ov);
  // count[0] = n_long; count[1] = quad workgroups started (launch_mixed's gate)
  hipError_t e = hipMemsetAsync(ov->count, 0, 8, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_chain_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, len, n,
                     quad_min_lines(n), ov->key_in, ov->idx_in, ov->count, ov->long_list);
  e = hipGetLastError();
  ov->perm = n == 1 ? ov->idx_in : ov->idx_out;  // one chain: nothing to order
  return e;
}

hipError_t launch_order_sort(OrderView* ov, size_t bytes, hipStream_t s) {
  if (ov->n <= 1) return hipSuccess;
  const size_t used = static_cast<uint8_t*>(ov->temp) - reinterpret_cast<uint8_t*>(ov->count);
  size_t temp_bytes = bytes - used;
  return hipcub::DeviceRadixSort::SortPairsDescending(ov->temp, temp_bytes, ov->key_in,
                                                      ov->key_out, ov->idx_in, ov->idx_out,
                                                      (int)ov->n, 0, kKeyBits, s);
}

}  // namespace dev
}  // namespace cir
