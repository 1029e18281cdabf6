// How much of config 2's kernel time is the slowest XCD's tail?
//
// k_chunks hands workgroups to the eight XCDs round-robin, so each XCD hashes
// the same 1/8 of the blocks; under load the XCD clocks differ by up to ~6 %
// (profiles/r03_s2/xcd_clock_probe.log), so the slowest XCD would set the
// kernel's time while the others idle.  This probe runs the production wave
// body (uniform_glds_wave, k_chunks' hot loop) over 1 M x 32 KiB blocks and
// records, per wave, its XCD and its start and end (s_memrealtime, 100 MHz).
// Per launch it prints each XCD's finish time and the bound of a perfect
// dynamic balance: the harmonic mean of the XCD finish times (every XCD kept
// busy to the end at its own rate), against the kernel's span.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude -Iciruela_amd/csrc \
//     tools/xcd_tail_probe.hip -o build/xcd_tail_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "uniform.hpp"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

using namespace cir::dev;

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xf;
}

__device__ __forceinline__ uint32_t hw_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(x));
  return x;
}

// stamps[wave * 4 + {0, 1, 2, 3}] = xcc, start, end, HW_ID (one lane per wave
// writes)
__global__ __launch_bounds__(kThreads, 4) void k_tail(const uint8_t* __restrict__ data,
                                                      uint64_t bs, uint32_t lines,
                                                      uint8_t* __restrict__ out,
                                                      uint64_t* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWaves * kWaveLds];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wave;
  const uint64_t blk0 = gw * 64u;
  uniform_glds_wave(data + blk0 * bs, bs, lines, out + blk0 * 32u, lds + wave * kWaveLds);
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0) {
    stamps[gw * 4 + 0] = xcc_id();
    stamps[gw * 4 + 1] = t0;
    stamps[gw * 4 + 2] = t1;
    stamps[gw * 4 + 3] = hw_id();
  }
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = (i + 1) * 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    p[i] = z ^ (z >> 31);
  }
}

int main() {
  const uint64_t bs = 32768, nblk = 1u << 20, nbytes = bs * nblk;
  const uint64_t nwaves = nblk / 64, nwg = nwaves / kWaves;
  uint8_t *data, *out;
  uint64_t* stamps;
  CK(hipMalloc(&data, nbytes));
  CK(hipMalloc(&out, nblk * 32));
  CK(hipMalloc(&stamps, nwaves * 4 * 8));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)data, nbytes / 8);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> h(nwaves * 4);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 8; ++rep) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_tail, dim3((unsigned)nwg), dim3(kThreads), 0, 0, data, bs,
                       (uint32_t)(bs / 128), out, stamps);
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
    if (rep < 2) continue;  // warm-up launches
    uint64_t t_first = UINT64_MAX, t_last = 0;
    std::vector<uint64_t> xend(8, 0), xcount(8, 0);
    std::vector<double> xbusy(8, 0);
    for (uint64_t w = 0; w < nwaves; ++w) {
      const uint32_t x = (uint32_t)h[w * 4] & 7u;
      t_first = std::min(t_first, h[w * 4 + 1]);
      t_last = std::max(t_last, h[w * 4 + 2]);
      xend[x] = std::max(xend[x], h[w * 4 + 2]);
      xbusy[x] += (double)(h[w * 4 + 2] - h[w * 4 + 1]);
      ++xcount[x];
    }
    const double span = (t_last - t_first) / 100e3;  // ms (100 MHz)
    double inv = 0;
    printf("launch %d: %.3f ms (events), span %.3f ms | XCD finish ms:", rep, ms, span);
    for (int x = 0; x < 8; ++x) {
      const double t = (xend[x] - t_first) / 100e3;
      inv += 1.0 / t;
      printf(" %.3f", t);
    }
    const double hm = 8.0 / inv;
    printf(" | waves/XCD %llu..%llu | wave avg ms:",
           (unsigned long long)*std::min_element(xcount.begin(), xcount.end()),
           (unsigned long long)*std::max_element(xcount.begin(), xcount.end()));
    for (int x = 0; x < 8; ++x) printf(" %.3f", xbusy[x] / (double)std::max<uint64_t>(1, xcount[x]) / 100e3);
    printf(" | balanced bound %.3f ms (%.2f %% below the span)\n", hm, 100.0 * (1.0 - hm / span));
    // SIMD occupancy over the span: SIMD key = xcc, se, sh, cu, simd (HW_ID
    // bits: simd [5:4], cu [11:8], sh [12], se [15:13]); time in 1 us bins,
    // each bin counted by the number of this SIMD's waves active in it
    std::vector<std::vector<int>> occ;
    std::vector<int> key_of(1 << 16, -1);
    const uint64_t nbins = (t_last - t_first) / 100 + 1;
    std::vector<double> hist(6, 0);
    std::vector<int> per_simd;
    for (uint64_t w = 0; w < nwaves; ++w) {
      const uint32_t id = (uint32_t)h[w * 4 + 3];
      const uint32_t k = ((uint32_t)h[w * 4] & 7u) << 13 | ((id >> 13) & 7u) << 10 |
                         ((id >> 12) & 1u) << 9 | ((id >> 8) & 15u) << 4 | ((id >> 4) & 3u);
      if (key_of[k] < 0) {
        key_of[k] = (int)occ.size();
        occ.emplace_back(nbins, 0);
        per_simd.push_back(0);
      }
      std::vector<int>& o = occ[key_of[k]];
      ++per_simd[key_of[k]];
      for (uint64_t b = (h[w * 4 + 1] - t_first) / 100; b <= (h[w * 4 + 2] - t_first) / 100 && b < nbins; ++b)
        ++o[b];
    }
    for (auto& o : occ)
      for (int v : o) hist[std::min(v, 5)] += 1;
    double tot = 0;
    for (double v : hist) tot += v;
    printf("    %zu SIMDs, waves per SIMD %d..%d; SIMD-time with 0/1/2/3/4/5+ waves: %.1f %.1f %.1f %.1f %.1f %.1f %%\n",
           occ.size(), *std::min_element(per_simd.begin(), per_simd.end()),
           *std::max_element(per_simd.begin(), per_simd.end()), 100 * hist[0] / tot,
           100 * hist[1] / tot, 100 * hist[2] / tot, 100 * hist[3] / tot, 100 * hist[4] / tot,
           100 * hist[5] / tot);
    // dispatch ramp and tail: when the waves start and end
    std::vector<uint64_t> st(nwaves), en(nwaves);
    for (uint64_t w = 0; w < nwaves; ++w) {
      st[w] = h[w * 4 + 1] - t_first;
      en[w] = h[w * 4 + 2] - t_first;
    }
    std::sort(st.begin(), st.end());
    std::sort(en.begin(), en.end());
    printf("    starts (ms): 4096th %.3f, last %.3f; ends: first %.3f, 12288th %.3f, last %.3f\n",
           st[4095] / 100e3, st[nwaves - 1] / 100e3, en[0] / 100e3, en[12287] / 100e3,
           en[nwaves - 1] / 100e3);
  }
  return 0;
}
