// VALU micro-benchmark for the BLAKE2b roofline on gfx950.
//
// 1. Throughput of the instructions the compression uses, relative to
//    v_xor_b32 (8 independent chains per lane, 8 waves per SIMD).
// 2. The compression function alone on register-resident messages: the same
//    number of compressions as the config-2 bench (1 M lanes x 256), no
//    memory traffic -> the VALU-only time floor of the hot kernel.
// 3. The in-kernel clock (s_memtime / s_memrealtime at 100 MHz).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I ciruela_amd/csrc \
//         tools/valu_ubench.hip -o build/valu_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "blake2b_dev.hpp"

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
      return 1;                                                               \
    }                                                                         \
  } while (0)

// X-macro: name, lane-instructions per asm statement, asm body.  Each body
// updates chain i (a[i] / w[i]) from other chains, 8 independent chains.
#define OPS(X)                                                                                   \
  X(xor_b32, 1, asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i])))                    \
  X(bitop3_b32_xor3, 1,                                                                          \
    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b[i]), "v"(b[j])))  \
  X(alignbit_b32, 1, asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(a[i]) : "v"(b[i])))      \
  X(alignbyte_b32, 1, asm volatile("v_alignbyte_b32 %0, %0, %1, 3" : "+v"(a[i]) : "v"(b[i])))     \
  X(perm_b32, 1, asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b[i]), "v"(sel)))   \
  X(lshl_add_u64, 1, asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(w[i]) : "v"(w[j])))      \
  X(lshl_add_u64_s1, 1, asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(w[i]) : "v"(w[j])))   \
  X(add_co_e64_pair, 2, {                                                                        \
    uint64_t c;                                                                                  \
    asm volatile("v_add_co_u32 %0, %2, %0, %3\n\tv_addc_co_u32 %1, %2, %1, %4, %2"               \
                 : "+v"(a[i]), "+v"(b[i]), "=&s"(c) : "v"(b[j]), "v"(a[k]));                     \
  })                                                                                             \
  X(add_co_e32_vcc_pair, 2,                                                                      \
    asm volatile("v_add_co_u32_e32 %0, vcc, %0, %2\n\tv_addc_co_u32_e32 %1, vcc, %1, %3, vcc"    \
                 : "+v"(a[i]), "+v"(b[i]) : "v"(b[j]), "v"(a[k]) : "vcc"))                       \
  X(add_u32_e32, 1, asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i])))            \
  X(add3_u32, 1, asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b[i]), "v"(b[j])))   \
  X(xad_u32, 1, asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b[i]), "v"(b[j])))     \
  X(lshl_or_b32, 1, asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(a[i]) : "v"(b[i])))         \
  X(or3_b32, 1, asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b[i]), "v"(b[j])))     \
  X(lshrrev_b32, 1, asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a[i])))                        \
  X(lshrrev_b64, 1, asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(w[i])))                        \
  X(xor_sdwa, 1,                                                                                 \
    asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE "          \
                 "src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(a[i]) : "v"(b[i])))                     \
  X(xor_dpp, 1,                                                                                  \
    asm volatile("v_xor_b32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"      \
                 : "+v"(a[i]) : "v"(b[i])))                                                       \
  X(mov_b64, 1, asm volatile("v_mov_b64 %0, %1" : "=v"(w[i]) : "v"(w[j])))                       \
  X(pk_mov_b32, 1, asm volatile("v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]" : "+v"(w[i]) : "v"(w[j])))

#define DEF_KERNEL(NAME, NI, BODY)                                                    \
  __global__ __launch_bounds__(256) void k_##NAME(uint32_t* out, int iters) {        \
    uint32_t a[8], b[8];                                                              \
    uint64_t w[8];                                                                    \
    const uint32_t sel = 0x05040302u;                                                 \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                   \
      a[i] = threadIdx.x * 7 + i;                                                     \
      b[i] = threadIdx.x ^ (i * 0x9e3779b9u);                                         \
      w[i] = ((uint64_t)a[i] << 32) | b[i];                                           \
    }                                                                                 \
    for (int it = 0; it < iters; ++it) {                                              \
      _Pragma("unroll") for (int r = 0; r < 16; ++r) {                                \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) {                               \
          const int j = (i + 1) & 7, k = (i + 3) & 7;                                 \
          (void)j;                                                                    \
          (void)k;                                                                    \
          BODY;                                                                       \
        }                                                                             \
      }                                                                               \
    }                                                                                 \
    uint32_t x = sel;                                                                 \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) x ^= a[i] ^ b[i] ^ (uint32_t)w[i] ^ \
                                                  (uint32_t)(w[i] >> 32);             \
    out[blockIdx.x * 256 + threadIdx.x] = x;                                          \
  }
OPS(DEF_KERNEL)

typedef void (*OpKernel)(uint32_t*, int);
struct OpInfo {
  const char* name;
  int ninst;
  OpKernel k;
};
#define DEF_INFO(NAME, NI, BODY) {#NAME, NI, k_##NAME},
static const OpInfo kOps[] = {OPS(DEF_INFO)};

// compression only: 256 compressions per lane on register messages
template <int R16, int R24, int R63>
__global__ __launch_bounds__(256, 4) void k_compress(uint8_t* out, uint32_t lines) {
  using namespace cir::dev;
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t h[8], m[16];
  init_state(h);
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = b * 0x9e3779b97f4a7c15ULL + k;
  for (uint32_t i = 0; i < lines; ++i) {
    m[i & 15] ^= i;  // keep the message live and varying
    compress_v<R16, R24, R63>(h, m, (uint64_t)(i + 1) * 128u, i + 1 == lines);
  }
  store_digest(out + b * 32, h);
}

__global__ void k_clock(uint64_t* out, int spin) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = threadIdx.x;
  for (int i = 0; i < spin; ++i) asm volatile("v_xor_b32 %0, %0, %0\n\tv_add_u32 %0, 1, %0" : "+v"(x));
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[blockIdx.x * 3 + 0] = t1 - t0;
    out[blockIdx.x * 3 + 1] = r1 - r0;
    out[blockIdx.x * 3 + 2] = x;
  }
}

static float time_kernel(OpKernel k, uint32_t* d, int grid, int iters) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, d, iters);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, d, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

typedef void (*CompKernel)(uint8_t*, uint32_t);
static float time_compress(CompKernel k, uint8_t* dout, uint64_t nlanes) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(nlanes / 256), dim3(256), 0, 0, dout, 256u);
  float best = 1e9;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(nlanes / 256), dim3(256), 0, 0, dout, 256u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device %s, %d CUs, clockRate %d kHz\n", prop.gcnArchName, cus, prop.clockRate);
  // clock
  uint64_t* dclk;
  CHECK(hipMalloc(&dclk, cus * 8 * 3 * 8));
  hipLaunchKernelGGL(k_clock, dim3(cus * 8), dim3(256), 0, 0, dclk, 2000000);
  CHECK(hipDeviceSynchronize());
  uint64_t hclk[3];
  CHECK(hipMemcpy(hclk, dclk, sizeof hclk, hipMemcpyDeviceToHost));
  printf("in-kernel clock (busy VALU loop): %.3f GHz\n", (double)hclk[0] / (double)hclk[1] * 0.1);

  const int grid = cus * 8;  // 8 WGs of 4 waves per CU = 8 waves per SIMD
  const int iters = 2048;
  uint32_t* d;
  CHECK(hipMalloc(&d, (size_t)grid * 256 * 4));
  const double lane_stmts = (double)grid * 256 * iters * 16 * 8;
  const float t_xor = time_kernel(kOps[0].k, d, grid, iters);
  for (const OpInfo& op : kOps) {
    const float t = time_kernel(op.k, d, grid, iters);
    printf("%-22s %8.3f ms  %6.2f T lane-instr/s  cost per instr vs v_xor_b32: %.2f\n", op.name, t,
           lane_stmts * op.ninst / (t * 1e-3) / 1e12, t / t_xor / op.ninst);
  }
  const double peak = (double)cus * 128 * 2.4e9;
  printf("peak at 2.4 GHz: %.2f T lane-instr/s; v_xor achieved %.1f%%\n", peak / 1e12,
         100.0 * lane_stmts / (t_xor * 1e-3) / peak);

  // compression only, config-2 shaped (1M lanes x 256 compressions)
  const uint64_t nlanes = 1 << 20;
  uint8_t* dout;
  CHECK(hipMalloc(&dout, nlanes * 32));
  struct {
    const char* name;
    CompKernel k;
  } comps[] = {
      {"alignbit 16/24/63 (r01 kernel)", k_compress<0, 0, 0>},
      {"perm 16/24, alignbit 63", k_compress<1, 1, 0>},
      {"perm 16/24, shl-add 63", k_compress<1, 1, 1>},
      {"alignbit 16/24, shl-add 63", k_compress<0, 0, 1>},
  };
  for (auto& c : comps) {
    const float t = time_compress(c.k, dout, nlanes);
    printf("compress-only [%s]: %.3f ms = %.1f GB/s equivalent\n", c.name, t,
           (double)nlanes * 32768 / (t * 1e-3) / 1e9);
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
