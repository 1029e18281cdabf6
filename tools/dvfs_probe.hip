// What lowers the sustained clock of the production kernel?  (diagnostics,
// not part of the product).  Times the LDS-DMA production loop
// (uniform.hpp) on 1 M x 32 KiB blocks streamed from HBM, the same loop
// with every wave re-reading the same 64 blocks (2 MiB, L2-resident: no HBM
// traffic), and the register-only compression, each with per-wave
// s_memtime / s_memrealtime stamps for the in-kernel clock.
//
//   hipcc -O3 --offload-arch=gfx950 -I ciruela_amd/csrc tools/dvfs_probe.hip -o build/dvfs_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "uniform.hpp"

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

using namespace cir::dev;

__device__ __forceinline__ void stamp(uint64_t* st, uint64_t t0, uint64_t r0) {
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    const uint32_t w = blockIdx.x * kWaves + (threadIdx.x >> 6);
    st[2 * w] = t1 - t0;
    st[2 * w + 1] = r1 - r0;
  }
}

// V 0: blocks streamed from HBM; V 1: every wave reads blocks 0..63 (L2)
template <int V>
__global__ __launch_bounds__(256, 5) void k_prod(const uint8_t* __restrict__ data, uint64_t bs,
                                                 uint32_t lines, uint8_t* __restrict__ out,
                                                 uint64_t* st) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWaves * kWaveLds];
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t blk0 = ((uint64_t)blockIdx.x * kWaves + wave) * 64u;
  const uint8_t* src = V == 0 ? data + blk0 * bs : data;
  uniform_glds_wave(src, bs, lines, out + blk0 * 32u, lds + wave * kWaveLds);
  stamp(st, t0, r0);
}

__global__ __launch_bounds__(256, 4) void k_comp(uint8_t* out, uint32_t lines, uint64_t* st) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t h[8], m[16];
  init_state(h);
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = b * 0x9e3779b97f4a7c15ULL + k;
  for (uint32_t i = 0; i < lines; ++i) {
    m[0] ^= i;
    compress(h, m, (uint64_t)(i + 1) * 128u, i + 1 == lines);
  }
  store_digest(out + b * 32u, h);
  stamp(st, t0, r0);
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (i + 1) * 0x9E3779B97F4A7C15ULL ^ (i >> 7);
}

int main() {
  const uint64_t nb = 1 << 20, bs = 32768;
  uint8_t *data, *out;
  uint64_t* st;
  CHECK(hipMalloc(&data, nb * bs));
  CHECK(hipMalloc(&out, nb * 32));
  CHECK(hipMalloc(&st, nb / 64 * 16));
  hipLaunchKernelGGL(k_fill, dim3(65536), dim3(256), 0, 0, (uint64_t*)data, nb * bs / 8);
  CHECK(hipDeviceSynchronize());
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const char* names[] = {"production, blocks streamed from HBM", "production, 64 blocks re-read (L2)",
                         "register-only compression"};
  std::vector<float> t[3];
  std::vector<double> clk[3];
  std::vector<uint64_t> hs(nb / 64 * 2);
  for (int round = 0; round < 6; ++round) {
    for (int v = 0; v < 3; ++v) {
      (void)hipEventRecord(a);
      if (v == 0) hipLaunchKernelGGL(k_prod<0>, dim3(nb / 256), dim3(256), 0, 0, data, bs, 256u, out, st);
      if (v == 1) hipLaunchKernelGGL(k_prod<1>, dim3(nb / 256), dim3(256), 0, 0, data, bs, 256u, out, st);
      if (v == 2) hipLaunchKernelGGL(k_comp, dim3(nb / 256), dim3(256), 0, 0, out, 256u, st);
      (void)hipEventRecord(b);
      CHECK(hipEventSynchronize(b));
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      if (round == 0) continue;
      t[v].push_back(ms);
      CHECK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
      const size_t nw = v == 2 ? nb / 64 : nb / 64;
      for (size_t i = 0; i < nw; i += 97) clk[v].push_back((double)hs[2 * i] / (double)hs[2 * i + 1] * 0.1);
    }
  }
  for (int v = 0; v < 3; ++v) {
    std::sort(t[v].begin(), t[v].end());
    std::sort(clk[v].begin(), clk[v].end());
    printf("%-40s median %.3f ms  in-kernel clock median %.3f GHz (p10 %.3f p90 %.3f)\n", names[v],
           t[v][t[v].size() / 2], clk[v][clk[v].size() / 2], clk[v][clk[v].size() / 10],
           clk[v][9 * clk[v].size() / 10]);
  }
  return 0;
}
