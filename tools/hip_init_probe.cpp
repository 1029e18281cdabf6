// Where a fresh process's HIP start-up goes, one step at a time (config 1's
// one-shot `ciruela-index sync` pays all of it before hashing 10 MiB):
// hipGetDeviceCount (runtime + device discovery), each of the library's
// streams created one by one (compute, copy, footer chain, two part streams,
// the high-priority quad stream), the three 10 MiB staging slots (pinned host
// + device), the first kernel and the first 4 MiB upload.  One line per run;
// tools/cli_start_env.sh runs it under environment variants.
//   hipcc --offload-arch=gfx950 -O2 tools/hip_init_probe.cpp -o build/hip_init_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <unistd.h>

#include <chrono>

static std::chrono::steady_clock::time_point t;
static void step(const char* what) {
  const auto now = std::chrono::steady_clock::now();
  printf("%s %.1f; ", what, std::chrono::duration<double, std::milli>(now - t).count());
  t = now;
}

__global__ void k_touch(uint32_t* p) { p[threadIdx.x] += 1; }

#define CK(x)                                                   \
  do {                                                          \
    hipError_t e_ = (x);                                        \
    if (e_ != hipSuccess) {                                     \
      printf("\n%s: %s\n", #x, hipGetErrorString(e_));          \
      return 1;                                                 \
    }                                                           \
  } while (0)

int main() {
  t = std::chrono::steady_clock::now();
  int n = 0;
  CK(hipGetDeviceCount(&n));
  step("count");
  CK(hipSetDevice(0));
  step("setdev");
  hipStream_t s[6];
  char name[16];
  for (int i = 0; i < 5; ++i) {
    CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
    snprintf(name, sizeof name, "stream%d", i + 1);
    step(name);
  }
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  CK(hipStreamCreateWithPriority(&s[5], hipStreamNonBlocking, hi));
  step("prio_stream");
  hipEvent_t ev[8];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  step("8 events");
  void *h[3], *d[3];
  for (int i = 0; i < 3; ++i) {
    CK(hipHostMalloc(&h[i], 10 << 20, hipHostMallocDefault));
    CK(hipMalloc(&d[i], 10 << 20));
  }
  step("3x10MiB slots");
  hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s[0], (uint32_t*)d[0]);
  CK(hipStreamSynchronize(s[0]));
  step("first kernel");
  CK(hipMemcpyAsync(d[1], h[1], 4 << 20, hipMemcpyHostToDevice, s[1]));
  CK(hipStreamSynchronize(s[1]));
  step("first upload");
  CK(hipMemcpyAsync(d[1], h[1], 4 << 20, hipMemcpyHostToDevice, s[2]));
  CK(hipStreamSynchronize(s[2]));
  step("upload on stream3");
  printf("devices %d\n", n);
  fflush(stdout);
  _exit(0);  // as the CLI: no teardown
}
