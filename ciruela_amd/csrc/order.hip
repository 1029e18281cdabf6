// Processing order of a mixed-length descriptor batch (config 3).
//
// One lane hashes one block, so a wave costs as much as its longest chain.
// Ordering descriptors by compression count (descending) puts chains of equal
// length in the same waves and dispatches the longest ones first, so they
// overlap with the short ones instead of trailing the launch.  The order is
// built on the device inside the timed call, by a counting sort over 4096
// length bins in two kernels (plus one memset):
//   k_chain_keys   bin of every chain, a per-workgroup LDS histogram added
//                  into the global one, and the batch's counters;
//   k_order_place  each workgroup scans the histogram (descending bins),
//                  reserves its chunk's slots per bin with one atomic per
//                  used bin, and places its chains through LDS cursors.
// Round 1-2 used hipCUB's radix sort on 16-bit keys: ~10 launches, ~0.13 ms
// with one context per process, ~0.5 ms with four (each launch ~50 us once
// several contexts' streams share the hardware queues; profiles/r02/early_quad/).
#include <algorithm>

#include "kernels.hpp"

namespace cir {
namespace dev {

constexpr uint32_t kBins = 4096;
constexpr unsigned kOrderGrid = 512;  // workgroups of both kernels (at most)

// Length bin, monotone in k (compressions): exact below 2048 (256 KiB, so
// the quad thresholds of 8 and 1024 lines never share a bin with shorter
// chains), then 128 bins per power of two up to 2^25 (< 0.8 % apart).
__device__ __forceinline__ uint32_t length_bin(uint32_t k) {
  if (k < 2048u) return k;
  const uint32_t e = 31u - (uint32_t)__builtin_clz(k);  // 11 .. 25
  return 2048u + (e - 11u) * 128u + ((k >> (e - 7u)) & 127u);
}

// Bins of a batch, the global histogram (hist, kBins counters) and the
// batch's counters.  count[0] = long chains (>= min_lines lines), count[2] =
// the longest chain (compressions), count[4..5] = the lane part's work
// (launch_mixed's pacing): compressions plus kLaneChainCost per chain for
// its setup and digest store.  A bounded grid strides over the batch and
// each workgroup adds its partial sums once: one atomic per wave and
// counter cost ~0.36 ms at config 3's 986 K descriptors (15 K waves on three
// addresses).
__global__ __launch_bounds__(256) void k_chain_keys(const uint32_t* __restrict__ len, uint64_t n,
                                                    uint32_t min_lines,
                                                    uint16_t* __restrict__ key,
                                                    uint32_t* __restrict__ count,
                                                    uint32_t* __restrict__ hist) {
  __shared__ uint32_t lh[kBins];
  for (uint32_t b = threadIdx.x; b < kBins; b += blockDim.x) lh[b] = 0;
  __syncthreads();
  uint32_t nl = 0, mx = 0;
  uint64_t w = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t l = len[i];
    const uint32_t k = l == 0 ? 1u : (l >> 7) + ((l & 127u) != 0);  // compressions, <= 2^25
    const uint32_t b = length_bin(k);
    key[i] = (uint16_t)b;
    atomicAdd(&lh[b], 1u);
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
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
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
  for (uint32_t b = threadIdx.x; b < kBins; b += blockDim.x)
    if (lh[b]) atomicAdd(&hist[b], lh[b]);
}

// Place chunk c = [c * C, min((c + 1) * C, n)) of the batch into perm in
// descending bin order.  cursor: kBins zeroed counters (slots taken per bin).
__global__ __launch_bounds__(256) void k_order_place(const uint16_t* __restrict__ key,
                                                     uint64_t n, uint64_t chunk,
                                                     const uint32_t* __restrict__ hist,
                                                     uint32_t* __restrict__ cursor,
                                                     uint32_t* __restrict__ perm) {
  __shared__ uint32_t base[kBins];  // first slot of bin b: chains in bins above b
  __shared__ uint32_t lc[kBins];    // this chunk's count per bin, then its cursors
  __shared__ uint32_t part[256];
  constexpr uint32_t kPer = kBins / 256;  // bins per thread in the scan
  const uint32_t t = threadIdx.x;
  // exclusive scan from the top bin down: thread t owns bins
  // kBins-1-kPer*t .. kBins-kPer*(t+1)
  uint32_t v[kPer], sum = 0;
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j) {
    v[j] = hist[kBins - 1u - (kPer * t + j)];
    sum += v[j];
  }
  part[t] = sum;
  for (uint32_t b = t; b < kBins; b += 256) lc[b] = 0;
  __syncthreads();
  for (uint32_t s = 1; s < 256; s <<= 1) {  // inclusive scan of the partials
    const uint32_t x = t >= s ? part[t - s] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t run = t ? part[t - 1] : 0u;
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j) {
    base[kBins - 1u - (kPer * t + j)] = run;
    run += v[j];
  }
  const uint64_t i0 = (uint64_t)blockIdx.x * chunk;
  const uint64_t i1 = min(n, i0 + chunk);
  for (uint64_t i = i0 + t; i < i1; i += 256) atomicAdd(&lc[key[i]], 1u);
  __syncthreads();
  // reserve this chunk's slots: one global atomic per bin it uses
  for (uint32_t b = t; b < kBins; b += 256) {
    const uint32_t c = lc[b];
    if (c) base[b] += atomicAdd(&cursor[b], c);
    lc[b] = 0;
  }
  __syncthreads();
  for (uint64_t i = i0 + t; i < i1; i += 256) {
    const uint32_t b = key[i];
    perm[base[b] + atomicAdd(&lc[b], 1u)] = (uint32_t)i;
  }
}

namespace {
// scratch: [256 B counters][hist kBins x 4][cursor kBins x 4][key][perm]
constexpr uint64_t kHead = 256 + 2ull * kBins * 4;
}  // namespace

size_t order_scratch_bytes(uint64_t n) {
  const uint64_t arr = (n * 4 + 255) & ~(uint64_t)255;
  return kHead + 2 * arr;
}

// ---- bounds of an untrusted descriptor batch ------------------------------
// The *_dev_bounded entry points take descriptors from another party's data
// (the daemon's received blocks, fetch_blocks.rs:77): block i is in range
// when off[i] + len[i] neither wraps nor passes arena_bytes.  One pass over
// the descriptors writes the lengths the hash kernels then read: len[i] for
// a block in range, 0 for one out of range -- a zero-length chain reads
// nothing (every loader reads at most its n bytes), so no kernel touches
// memory outside the arena -- and flags the out-of-range ones.

__global__ __launch_bounds__(256) void k_desc_bound(const uint64_t* __restrict__ off,
                                                    const uint32_t* __restrict__ len, uint64_t n,
                                                    uint64_t arena_bytes,
                                                    uint32_t* __restrict__ slen,
                                                    uint8_t* __restrict__ flag,
                                                    uint32_t* __restrict__ nflag) {
  uint32_t bad_here = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t o = off[i];
    const uint32_t l = len[i];
    const uint64_t end = o + l;
    const bool bad = end < o || end > arena_bytes;
    slen[i] = bad ? 0u : l;
    flag[i] = bad ? 1 : 0;
    bad_here += bad;
  }
#pragma unroll
  for (int sft = 1; sft < 64; sft <<= 1) bad_here += (uint32_t)__shfl_xor((int)bad_here, sft);
  if ((threadIdx.x & 63u) == 0 && bad_here) atomicAdd(nflag, bad_here);
}

// Digests of the flagged blocks: 32 zero bytes (the hash kernels wrote the
// empty input's digest there).
__global__ __launch_bounds__(256) void k_desc_zero(const uint8_t* __restrict__ flag, uint64_t n,
                                                   uint8_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    if (flag[i]) {
      uint4* o = reinterpret_cast<uint4*>(out + 32 * i);
      o[0] = make_uint4(0, 0, 0, 0);
      o[1] = make_uint4(0, 0, 0, 0);
    }
}

size_t bound_scratch_bytes(uint64_t n) {
  const uint64_t arr = (n * 4 + 255) & ~(uint64_t)255;
  return 256 + arr + ((n + 255) & ~(uint64_t)255);
}

hipError_t launch_desc_bound(const uint64_t* off, const uint32_t* len, uint64_t n,
                             uint64_t arena_bytes, void* scratch, uint32_t* nflag,
                             uint32_t** slen, uint8_t** flag, hipStream_t s) {
  // scratch: [256 B: an own counter][slen][flag]
  const uint64_t arr = (n * 4 + 255) & ~(uint64_t)255;
  uint8_t* base = static_cast<uint8_t*>(scratch);
  *slen = reinterpret_cast<uint32_t*>(base + 256);
  *flag = base + 256 + arr;
  if (!nflag) nflag = reinterpret_cast<uint32_t*>(base);
  hipError_t e = hipMemsetAsync(nflag, 0, 4, s);
  if (e != hipSuccess || n == 0) return e;
  const uint64_t grid = std::min<uint64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(k_desc_bound, dim3((unsigned)grid), dim3(256), 0, s, off, len, n,
                     arena_bytes, *slen, *flag, nflag);
  return hipGetLastError();
}

hipError_t launch_desc_zero(const uint8_t* flag, uint64_t n, uint8_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t grid = std::min<uint64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(k_desc_zero, dim3((unsigned)grid), dim3(256), 0, s, flag, n, out);
  return hipGetLastError();
}

hipError_t launch_order_desc(const uint32_t* len, uint64_t n, void* scratch, size_t bytes,
                             uint32_t** perm, uint32_t** n_long, hipStream_t s) {
  const uint64_t arr = (n * 4 + 255) & ~(uint64_t)255;
  uint8_t* base = static_cast<uint8_t*>(scratch);
  uint32_t* count = reinterpret_cast<uint32_t*>(base);
  uint32_t* hist = reinterpret_cast<uint32_t*>(base + 256);
  uint32_t* cursor = hist + kBins;
  uint8_t* p = base + kHead;
  // count[0] = n_long; count[1] = quad workgroups started (launch_mixed's
  // gate); count[2] = longest chain; count[4..5] = lane work (k_chain_keys);
  // count[6] = lane tiles claimed (k_lane_rest); then the histogram and the
  // per-bin cursors: one memset for all of them
  hipError_t e = hipMemsetAsync(count, 0, kHead, s);
  if (e != hipSuccess) return e;
  *n_long = count;
  const uint64_t kgrid = std::min<uint64_t>((n + 255) / 256, kOrderGrid);
  uint16_t* key = reinterpret_cast<uint16_t*>(p);
  uint32_t* out = reinterpret_cast<uint32_t*>(p + arr);
  hipLaunchKernelGGL(k_chain_keys, dim3((unsigned)kgrid), dim3(256), 0, s, len, n,
                     quad_min_lines(n), key, count, hist);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint64_t chunk = (n + kgrid - 1) / kgrid;
  hipLaunchKernelGGL(k_order_place, dim3((unsigned)kgrid), dim3(256), 0, s, key, n, chunk, hist,
                     cursor, out);
  *perm = out;
  return hipGetLastError();
}

}  // namespace dev
}  // namespace cir
