// Is the shader clock one domain for the chip or one per XCD?
//
// k_load: an integer G-like loop (64-bit adds, xors, funnel shifts -- the
// blake2b instruction mix) on every workgroup whose XCD is in `mask`; the
// others exit at once.  k_probe: one light wave per workgroup on a
// high-priority stream, concurrently, that records its XCD and the shader
// clock over its loop (delta s_memtime / delta s_memrealtime x 100 MHz).
// Scenarios: probe alone, load on every XCD, load on XCDs 2-7, load on 0-1.
// If the clock is per XCD, an unloaded XCD keeps ~2.4 GHz beside loaded ones
// (config 3: quad chains on their own XCDs would then run at the idle clock).
//
//   hipcc -O3 --offload-arch=gfx950 tools/xcd_clock_probe.hip -o build/xcd_clock_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xf;
}

__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

__global__ __launch_bounds__(256) void k_load(uint32_t mask, int iters, const uint4* buf,
                                              uint64_t buf_mask, uint32_t* sink) {
  if (!((mask >> xcc_id()) & 1u)) return;
  uint64_t a = threadIdx.x * 0x9e3779b97f4a7c15ull, b = blockIdx.x ^ 0x6a09e667f3bcc908ull;
  uint64_t c = 0xbb67ae8584caa73bull + threadIdx.x, d = 0x3c6ef372fe94f82bull ^ blockIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * 256u;
  uint64_t idx = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  for (int i = 0; i < iters; ++i, idx += stride) {
    // 16 B per lane per 12 G (the config-2 kernel's 128 B per 96 G): HBM
    // traffic at about that kernel's rate, coalesced 1 KiB per wave
    const uint4 x = buf[idx & buf_mask];
    uint64_t m = ((uint64_t)x.y << 32 | x.x) ^ a, n = ((uint64_t)x.w << 32 | x.z) ^ b;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      a = a + b + m;
      d = rotr64(d ^ a, 32);
      c = c + d;
      b = rotr64(b ^ c, 24);
      a = a + b + n;
      d = rotr64(d ^ a, 16);
      c = c + d;
      b = rotr64(b ^ c, 63);
      m ^= c;
      n += d;
    }
  }
  if ((a ^ b ^ c ^ d) == 0x123456789ull) sink[0] = 1;  // never true in practice; keeps the loop
}

__global__ void k_fill(uint4* buf, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = i * 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    buf[i] = make_uint4((uint32_t)z, (uint32_t)(z >> 32), (uint32_t)~z, (uint32_t)(z >> 17));
  }
}

// out[blk*4 + {0,1,2,3}] = xcc, d memtime, d memrealtime, cu-ish id
__global__ __launch_bounds__(64) void k_probe(int iters, uint64_t* out) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t v = threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    v = v * 1664525u + 1013904223u;
    __builtin_amdgcn_s_sleep(2);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[blockIdx.x * 4 + 0] = xcc_id();
    out[blockIdx.x * 4 + 1] = t1 - t0;
    out[blockIdx.x * 4 + 2] = r1 - r0;
    out[blockIdx.x * 4 + 3] = v;
  }
}

int main() {
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t sl, sp;
  CK(hipStreamCreateWithFlags(&sl, hipStreamNonBlocking));
  CK(hipStreamCreateWithPriority(&sp, hipStreamNonBlocking, greatest));
  uint32_t* sink;
  uint64_t* out;
  const int nprobe = 256;
  CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&out, nprobe * 4 * 8));
  const uint64_t buf_n = 1ull << 29;  // 8 GiB of uint4
  uint4* buf;
  CK(hipMalloc(&buf, buf_n * 16));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, sl, buf, buf_n);
  // the load runs ~0.3 s per launch; the probe ~25 ms inside it
  const int load_grid = 256 * 3, load_iters = 250000;  // 3 waves/SIMD: room for the probe
  const int probe_iters = 400000;
  struct Sc {
    const char* name;
    uint32_t mask;
  } sc[] = {{"probe alone", 0u}, {"load all XCDs", 0xffu}, {"load XCDs 2-7", 0xfcu},
            {"load XCDs 0-1", 0x03u}, {"load all XCDs (again)", 0xffu}, {"probe alone (again)", 0u}};
  // warm-up: ~1 s of load so the chip is at its steady loaded state
  for (int w = 0; w < 4; ++w) hipLaunchKernelGGL(k_load, dim3(load_grid), dim3(256), 0, sl, 0xffu, load_iters, buf, buf_n - 1, sink);
  CK(hipStreamSynchronize(sl));
  for (const Sc& s : sc) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, sl));
    if (s.mask)
      hipLaunchKernelGGL(k_load, dim3(load_grid), dim3(256), 0, sl, s.mask, load_iters, buf, buf_n - 1, sink);
    hipLaunchKernelGGL(k_probe, dim3(nprobe), dim3(64), 0, sp, probe_iters, out);
    CK(hipStreamSynchronize(sp));
    CK(hipStreamSynchronize(sl));
    CK(hipEventRecord(e1, sl));
    CK(hipEventSynchronize(e1));
    float load_ms = 0;
    CK(hipEventElapsedTime(&load_ms, e0, e1));
    std::vector<uint64_t> h(nprobe * 4);
    CK(hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> per[16];
    for (int b = 0; b < nprobe; ++b) {
      const double ghz = h[b * 4 + 2] ? (double)h[b * 4 + 1] / (double)h[b * 4 + 2] * 0.1 : 0;
      per[h[b * 4] & 15].push_back(ghz);
    }
    printf("%-22s mask 0x%02x (load+probe %.1f ms):", s.name, s.mask, load_ms);
    for (int x = 0; x < 8; ++x) {
      auto& v = per[x];
      if (v.empty()) {
        printf("  x%d  -  ", x);
        continue;
      }
      std::sort(v.begin(), v.end());
      printf("  x%d %.3f", x, v[v.size() / 2]);
    }
    printf("  GHz (median per XCD)\n");
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
  }
  return 0;
}
