// The HIP runtime's start-up cost apart from the library: the least a
// process that hashes anything on the GPU must do, step by step --
// hipGetDeviceCount (device discovery), hipSetDevice + hipFree(0), the first
// stream, a 4 MiB pinned buffer and device buffer, one 4 MiB upload, one
// kernel launch, and the teardown of those -- printing each step's ms.
// The one-shot CLI's own steps (CIR_TRACE=1 bin/ciruela-index ...) compare
// against these (tools/cli_startup.py).
//   build/hip_start_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>

static std::chrono::steady_clock::time_point t;
static void step(const char* what) {
  const auto now = std::chrono::steady_clock::now();
  printf("%s %.1f ms; ", what, std::chrono::duration<double, std::milli>(now - t).count());
  t = now;
}

__global__ void k_touch(uint32_t* p) { p[threadIdx.x] += 1; }

#define CK(x) \
  if ((x) != hipSuccess) return 1
int main() {
  t = std::chrono::steady_clock::now();
  int n = 0;
  CK(hipGetDeviceCount(&n));
  step("hipGetDeviceCount");
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  step("hipSetDevice+hipFree(0)");
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  step("first stream");
  void *h = nullptr, *d = nullptr;
  CK(hipHostMalloc(&h, 4 << 20, 0));
  CK(hipMalloc(&d, 4 << 20));
  step("4 MiB pinned + device");
  CK(hipMemcpyAsync(d, h, 4 << 20, hipMemcpyHostToDevice, s));
  CK(hipStreamSynchronize(s));
  step("first 4 MiB upload");
  CK(hipMemcpyAsync(d, h, 4 << 20, hipMemcpyHostToDevice, s));
  CK(hipStreamSynchronize(s));
  step("second upload");
  hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, (uint32_t*)d);
  CK(hipStreamSynchronize(s));
  step("first kernel");
  CK(hipHostFree(h));
  CK(hipFree(d));
  CK(hipStreamDestroy(s));
  step("teardown");
  printf("\n");
  return 0;
}
