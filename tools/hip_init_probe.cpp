// Wall time of HIP runtime start-up in a fresh process (config 1's one-shot
// `ciruela-index sync` pays it before any hashing): hipGetDeviceCount, first
// hipSetDevice + hipFree(0) (context creation), one hipMalloc, one stream.
//   hipcc -O2 tools/hip_init_probe.cpp -o build/hip_init_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>

static double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
  const auto t0 = std::chrono::steady_clock::now();
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 1;
  const double t_count = ms_since(t0);
  if (hipSetDevice(0) != hipSuccess || hipFree(nullptr) != hipSuccess) return 1;
  const double t_ctx = ms_since(t0);
  void* p = nullptr;
  if (hipMalloc(&p, 1 << 20) != hipSuccess) return 1;
  const double t_malloc = ms_since(t0);
  hipStream_t s;
  if (hipStreamCreate(&s) != hipSuccess) return 1;
  const double t_stream = ms_since(t0);
  printf("hip_init_probe: devices %d, hipGetDeviceCount %.1f ms, +context %.1f ms, +hipMalloc %.1f ms, "
         "+stream %.1f ms (cumulative)\n", n, t_count, t_ctx, t_malloc, t_stream);
  (void)hipFree(p);
  (void)hipStreamDestroy(s);
  return 0;
}
