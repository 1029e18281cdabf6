// Processing order of a mixed-length descriptor batch (config 3).
//
// One lane hashes one block, so a wave costs as much as its longest chain.
// Sorting descriptors by compression count (descending) puts chains of equal
// length in the same waves and dispatches the longest ones first, so they
// overlap with the short ones instead of trailing the launch.  The sort runs
// on the device (hipCUB radix sort on 16-bit keys) inside the timed call.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "kernels.hpp"

namespace cir {
namespace dev {

constexpr int kKeyBits = 16;  // k_chain_keys' key width

// Keys and the counters of a batch.  count[0] = long chains, count[2] = the
// longest chain (compressions), count[4..5] = the lane part's work
// (launch_mixed's pacing): compressions plus kLaneChainCost per chain for its
// setup and digest store.  A bounded grid strides over the batch and each
// workgroup adds its partial sums once: one atomic per wave and counter cost
// ~0.36 ms at config 3's 986 K descriptors (15 K waves on three addresses).
constexpr unsigned kKeyGridMax = 512;

__global__ __launch_bounds__(256) void k_chain_keys(const uint32_t* __restrict__ len, uint64_t n,
                                                    uint32_t min_lines,
                                                    uint16_t* __restrict__ key,
                                                    uint32_t* __restrict__ idx,
                                                    uint32_t* __restrict__ count) {
  uint32_t nl = 0, mx = 0;
  uint64_t w = 0;
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t l = len[i];
    const uint32_t k = l == 0 ? 1u : (l >> 7) + ((l & 127u) != 0);  // compressions, <= 2^25
    // 16-bit sort key, monotone in k: exact below 32768 lines (4 MiB), then
    // steps of 1024 lines (128 KiB) up to 2^25 lines.  With 2-byte keys
    // rocPRIM sorts batches above 100 K items by onesweep (~4 launches);
    // with 4-byte keys it chose block sort + merge sort up to 1 M items
    // (~21 launches).  The launches, not the work, dominate the ordering:
    // ~7 us each, ~45 us each with several contexts' queues in one process
    // (profiles/r02/gtrace*).
    key[i] = (uint16_t)(k < 32768u ? k : 32768u + ((k - 32768u) >> 10));
    idx[i] = (uint32_t)i;
    if (k >= min_lines)
      ++nl;
    else
      w += k + kLaneChainCost;
    mx = max(mx, k);
  }
#pragma unroll
  for (int sft = 1; sft < 64; sft <<= 1) {  // every lane is here: no early return above
    nl += (uint32_t)__shfl_xor((int)nl, sft);
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, sft));
    w += (uint64_t)__shfl_xor((unsigned long long)w, sft);
  }
  __shared__ uint32_t s_nl[4], s_mx[4];
  __shared__ uint64_t s_w[4];
  const uint32_t wave = threadIdx.x >> 6;
  if (lane == 0) {
    s_nl[wave] = nl;
    s_mx[wave] = mx;
    s_w[wave] = w;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t nw = blockDim.x >> 6;
    for (uint32_t v = 1; v < nw; ++v) {
      nl += s_nl[v];
      mx = max(mx, s_mx[v]);
      w += s_w[v];
    }
    if (nl) atomicAdd(count, nl);
    if (w) atomicAdd(reinterpret_cast<unsigned long long*>(count + 4), (unsigned long long)w);
    atomicMax(count + 2, mx);
  }
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
  // gate); count[2] = longest chain; count[4..5] = lane work (k_chain_keys);
  // count[6] = lane tiles claimed (k_lane_rest)
  hipError_t e0 = hipMemsetAsync(count, 0, 32, s);
  if (e0 != hipSuccess) return e0;
  *n_long = count;
  uint16_t* key_in = reinterpret_cast<uint16_t*>(p);
  uint16_t* key_out = reinterpret_cast<uint16_t*>(p + arr);
  uint32_t* idx_in = reinterpret_cast<uint32_t*>(p + 2 * arr);
  uint32_t* idx_out = reinterpret_cast<uint32_t*>(p + 3 * arr);
  void* temp = p + 4 * arr;
  size_t temp_bytes = bytes - 4 * arr;
  const uint64_t kgrid = std::min<uint64_t>((n + 255) / 256, kKeyGridMax);
  hipLaunchKernelGGL(k_chain_keys, dim3((unsigned)kgrid), dim3(256), 0, s, len, n,
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
