// Dependent-instruction latency on gfx950, one wave alone on the chip
// (diagnostics for the latency-bound quad-per-chain mode; not part of the
// product).  Each kernel runs a chain of dependent instructions (or K
// interleaved independent chains) and reports shader cycles per
// instruction from s_memtime.
//
//   hipcc -O3 --offload-arch=gfx950 tools/lat_ubench.hip -o build/lat_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

constexpr int kIters = 4096;

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

// 32-bit chains: NI instructions per asm block
#define CHAIN32(NAME, NI, BODY)                                                       \
  __global__ void k_##NAME(uint64_t* out, uint32_t seed) {                            \
    uint32_t x = seed + threadIdx.x, y = seed * 3u + 1u, z = 0x12345u;                \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                       \
    for (int i = 0; i < kIters; ++i) asm volatile(R16(BODY) : "+v"(x) : "v"(y), "v"(z)); \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                       \
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = x; out[2] = NI; }              \
  }

CHAIN32(xor, 16, "v_xor_b32 %0, %0, %1\n")
CHAIN32(add_u32, 16, "v_add_u32 %0, %0, %1\n")
CHAIN32(alignbit, 16, "v_alignbit_b32 %0, %0, %1, 7\n")
CHAIN32(bitop3, 16, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n")
CHAIN32(perm, 16, "v_perm_b32 %0, %0, %1, %2\n")
CHAIN32(xor_dpp_nop, 32, "v_xor_b32_dpp %0, %0, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\ns_nop 1\n")
CHAIN32(mov_dpp_nop, 32, "v_mov_b32_dpp %0, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\ns_nop 1\n")
CHAIN32(xor_then_dpp, 48, "v_xor_b32 %0, %0, %1\ns_nop 1\nv_xor_b32_dpp %0, %0, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n")
CHAIN32(nop1, 16, "s_nop 1\n")

// 64-bit chains
#define CHAIN64(NAME, NI, BODY)                                                       \
  __global__ void k_##NAME(uint64_t* out, uint32_t seed) {                            \
    uint64_t x = seed + threadIdx.x, y = seed * 3ull + 1ull;                          \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                       \
    for (int i = 0; i < kIters; ++i) asm volatile(R16(BODY) : "+v"(x) : "v"(y));      \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                       \
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = x; out[2] = NI; }              \
  }

CHAIN64(lshl_add_u64, 16, "v_lshl_add_u64 %0, %0, 0, %1\n")
CHAIN64(lshl_add_u64_x2ind, 16, "v_lshl_add_u64 %0, %0, 0, %1\n")
CHAIN64(mov_b64, 16, "v_mov_b64 %0, %0\n")

// 64-bit add as add_co / addc on halves (the VCC hazard needs 2 wait states)
__global__ void k_addco_pair(uint64_t* out, uint32_t seed) {
  uint32_t xl = seed + threadIdx.x, xh = seed ^ 77u, yl = seed * 3u, yh = 5u;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i)
    asm volatile(R16("v_add_co_u32 %0, vcc, %0, %2\ns_nop 1\nv_addc_co_u32 %1, vcc, %1, %3, vcc\n")
                 : "+v"(xl), "+v"(xh) : "v"(yl), "v"(yh) : "vcc");
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = xl ^ xh; out[2] = 48; }
}

// K independent 64-bit add chains interleaved: throughput of one wave
template <int K>
__global__ void k_lshl_add_ilp(uint64_t* out, uint32_t seed) {
  uint64_t x[K], y = seed * 3ull + 1ull;
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = seed + threadIdx.x + k;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int k = 0; k < K; ++k) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(x[k]) : "v"(y));
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) s ^= x[k];
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = s; out[2] = 16 * K; }
}

template <int K>
__global__ void k_xor_ilp(uint64_t* out, uint32_t seed) {
  uint32_t x[K], y = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = seed + threadIdx.x + k;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int k = 0; k < K; ++k) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[k]) : "v"(y));
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) s ^= x[k];
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = s; out[2] = 16 * K; }
}

template <int K>
__global__ void k_alignbit_ilp(uint64_t* out, uint32_t seed) {
  uint32_t x[K], y = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = seed + threadIdx.x + k;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int k = 0; k < K; ++k) asm volatile("v_alignbit_b32 %0, %0, %1, 9" : "+v"(x[k]) : "v"(y));
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) s ^= x[k];
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = s; out[2] = 16 * K; }
}

typedef void (*K)(uint64_t*, uint32_t);

int main() {
  uint64_t* d;
  CHECK(hipMalloc(&d, 64));
  struct {
    const char* name;
    K k;
  } ks[] = {
      {"v_xor_b32 chain", k_xor},
      {"v_add_u32 chain", k_add_u32},
      {"v_alignbit_b32 chain", k_alignbit},
      {"v_bitop3_b32 chain", k_bitop3},
      {"v_perm_b32 chain", k_perm},
      {"v_lshl_add_u64 chain", k_lshl_add_u64},
      {"v_mov_b64 chain", k_mov_b64},
      {"v_xor_b32_dpp + s_nop 1 (per 2 instr)", k_xor_dpp_nop},
      {"v_mov_b32_dpp + s_nop 1 (per 2 instr)", k_mov_dpp_nop},
      {"xor; s_nop 1; xor_dpp (per 3 instr)", k_xor_then_dpp},
      {"s_nop 1 alone", k_nop1},
      {"add_co; s_nop 1; addc (per 3 instr)", k_addco_pair},
      {"lshl_add_u64 x1 chain", k_lshl_add_ilp<1>},
      {"lshl_add_u64 x2 chains", k_lshl_add_ilp<2>},
      {"lshl_add_u64 x4 chains", k_lshl_add_ilp<4>},
      {"lshl_add_u64 x8 chains", k_lshl_add_ilp<8>},
      {"xor x1 chain", k_xor_ilp<1>},
      {"xor x2 chains", k_xor_ilp<2>},
      {"xor x4 chains", k_xor_ilp<4>},
      {"xor x8 chains", k_xor_ilp<8>},
      {"alignbit x1 chain", k_alignbit_ilp<1>},
      {"alignbit x2 chains", k_alignbit_ilp<2>},
      {"alignbit x4 chains", k_alignbit_ilp<4>},
      {"alignbit x8 chains", k_alignbit_ilp<8>},
  };
  for (auto& k : ks) {
    uint64_t h[3];
    double best = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, d, 12345u);
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost));
      const double c = (double)h[0] / ((double)kIters * (double)h[2]);
      if (c < best) best = c;
    }
    // s_memtime counts at the shader clock (MI355X_MICROARCH.md cycle constants)
    printf("%-42s %6.2f cycles per instruction (one wave)\n", k.name, best);
  }
  return 0;
}
