// Does HBM row locality move k_chunks' clock?  The production loop
// (uniform.hpp: 64 blocks per wave, one 128-B line of each per step, LDS-DMA)
// run with the line of block b at step i placed at
//   wsrc + b * bstride + i * lstride
// over the same 32 GiB:
//   strided     bstride 32768, lstride 128   (the real layout: each DMA
//               instruction reads 8 lines 32 KiB apart)
//   interleaved bstride 128,   lstride 8192  (each DMA instruction reads 1 KiB
//               contiguous, a wave's step 8 KiB contiguous)
// Same instructions, same bytes, different DRAM pages per byte.  The digests
// differ between the two (different bytes per block); only the time matters.
//
//   build/locality_probe [reps=5] [constant=0]
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Iciruela_amd/csrc \
//         tools/locality_probe.hip -o build/locality_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "blake2b_dev.hpp"
#include "kernels.hpp"

using namespace cir::dev;

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      return 1;                                                          \
    }                                                                    \
  } while (0)

__global__ __launch_bounds__(256, 4) void k_probe(const uint8_t* __restrict__ src,
                                                  uint64_t bstride, uint64_t lstride,
                                                  uint64_t wave_bytes, uint32_t lines,
                                                  uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 8192];
  const uint32_t wave = threadIdx.x >> 6;
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + wave;
  const uint8_t* wsrc = src + gw * wave_bytes;
  uint8_t* wl = lds + wave * 8192;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t r = lane >> 3;
  uint32_t dma_lane = (uint32_t)(r * bstride) + 16u * ((lane & 7u) ^ r);
  const uint32_t s = (lane ^ (lane >> 3)) & 7u;
  uint32_t rd_base = lane * 128u + 16u * s;
  const uint64_t jstride = 8u * bstride;
  auto issue = [&](uint32_t i) {
    const uint8_t* line = wsrc + (uint64_t)i * lstride;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint8_t* p = line + (uint64_t)j * jstride + (dma_lane ^ (16u * j));
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)p,
                                       (void __attribute__((address_space(3)))*)(wl + j * 1024),
                                       16, 0, 2);
    }
  };
  uint64_t h[8];
  init_state(h);
  uint64_t m[16];
  issue(0);
  for (uint32_t i = 0; i < lines; ++i) {
    asm volatile("" : "+v"(rd_base), "+v"(dma_lane));
    __builtin_amdgcn_s_waitcnt(0x0070);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint4 x = *reinterpret_cast<const uint4*>(wl + (rd_base ^ (16u * c)));
      m[2 * c] = mk64(x.x, x.y);
      m[2 * c + 1] = mk64(x.z, x.w);
    }
    compress_sm(h, m, (uint64_t)(i + 1) * 128u, i + 1 == lines, [&] {
      __builtin_amdgcn_s_waitcnt(0xC07F);
      if (i + 1 < lines) issue(i + 1);
    });
  }
  store_digest(out + (gw * 64 + lane) * 32u, h);
}

// splitmix64 words (the bench's data is random: constant bytes run the
// compression at a higher clock, MI355X_MICROARCH.md DVFS note)
__global__ void k_fill(uint64_t* p, uint64_t n) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = 0x5EED0002ull + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[k] = z ^ (z >> 31);
  }
}

int main(int argc, char** argv) {
  const uint64_t nblk = 1ull << 20, bs = 32768;
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  uint8_t *d = nullptr, *out = nullptr;
  CHECK(hipMalloc(&d, nblk * bs));
  CHECK(hipMalloc(&out, nblk * 32));
  const bool constant = argc > 2 && atoi(argv[2]) == 1;
  if (constant) {
    CHECK(hipMemset(d, 0x5a, nblk * bs));
  } else {
    hipLaunchKernelGGL(k_fill, dim3(65536), dim3(256), 0, 0, (uint64_t*)d, nblk * bs / 8);
    CHECK(hipGetLastError());
  }
  CHECK(hipDeviceSynchronize());
  printf("data: %s\n", constant ? "constant 0x5a bytes" : "splitmix64 words");
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const uint64_t waves = nblk / 64;
  struct V {
    const char* name;
    uint64_t bstride, lstride;
  } vs[2] = {{"strided (real layout)", bs, 128}, {"interleaved (8 KiB contiguous per step)", 128, 8192}};
  double tot[2] = {0, 0};
  for (int rep = 0; rep <= reps; ++rep)
    for (int v = 0; v < 2; ++v) {
      CHECK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(k_probe, dim3((unsigned)(waves / 4)), dim3(256), 0, 0, d, vs[v].bstride,
                         vs[v].lstride, 64 * bs, (uint32_t)(bs / 128), out);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(b, 0));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      if (rep) tot[v] += ms;
      printf("rep %d %-42s %.3f ms\n", rep, vs[v].name, ms);
    }
  for (int v = 0; v < 2; ++v)
    printf("mean %-42s %.3f ms = %.1f GiB/s\n", vs[v].name, tot[v] / reps,
           nblk * bs / (tot[v] / reps / 1e3) / (1 << 30));
  return 0;
}
