// Quad-mode G step issue latency on gfx950 (diagnostics, not part of the
// product).  One quad-mode G step (4 lanes per chain, DPP quad_perm for the
// diagonal layout) in two instruction forms:
//   V0 (production today, 24 VALU): b and c permuted into registers with
//      v_mov_b32_dpp, then 64-bit adds as v_lshl_add_u64;
//   V1 (22 VALU): the permuted b and c feed the adds directly as
//      v_add_co_u32_dpp + v_addc_co_u32_dpp (VOP2 DPP), b's second use as
//      v_xor_b32_dpp.
// One wave alone (s_memtime cycles per step) and one wave per SIMD on the
// whole chip (HIP events, ns per step).
//
//   hipcc -O3 --offload-arch=gfx950 tools/quad_dpp_ubench.hip -o build/quad_dpp_ubench
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

// a v[10:11]  b v[12:13]  c v[14:15]  d v[16:17]  m0 v[18:19]  m1 v[20:21]
// t v[22:23]  u v[24:25]  b' v[26:27]  c' v[28:29]
#define QP "quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf"
#define TAIL                                        \
  "v_lshl_add_u64 v[10:11], v[10:11], 0, v[20:21]\n" \
  "v_lshl_add_u64 v[10:11], v[10:11], 0, v[12:13]\n" \
  "v_xor_b32 v24, v22, v10\n"                       \
  "v_xor_b32 v25, v23, v11\n"                       \
  "v_alignbit_b32 v16, v25, v24, 16\n"              \
  "v_alignbit_b32 v17, v24, v25, 16\n"              \
  "v_lshl_add_u64 v[14:15], v[14:15], 0, v[16:17]\n" \
  "v_xor_b32 v24, v12, v14\n"                       \
  "v_xor_b32 v25, v13, v15\n"                       \
  "v_alignbit_b32 v12, v24, v25, 31\n"              \
  "v_alignbit_b32 v13, v25, v24, 31\n"

#define STEP_V0                                      \
  "v_lshl_add_u64 v[10:11], v[10:11], 0, v[18:19]\n" \
  "v_mov_b32_dpp v28, v14 " QP "\n"                  \
  "v_mov_b32_dpp v29, v15 " QP "\n"                  \
  "v_mov_b32_dpp v26, v12 " QP "\n"                  \
  "v_mov_b32_dpp v27, v13 " QP "\n"                  \
  "v_lshl_add_u64 v[10:11], v[10:11], 0, v[26:27]\n" \
  "v_xor_b32_dpp v22, v17, v11 " QP "\n"             \
  "v_xor_b32_dpp v23, v16, v10 " QP "\n"             \
  "v_lshl_add_u64 v[14:15], v[28:29], 0, v[22:23]\n" \
  "v_xor_b32 v24, v26, v14\n"                        \
  "v_xor_b32 v25, v27, v15\n"                        \
  "v_alignbit_b32 v12, v25, v24, 24\n"               \
  "v_alignbit_b32 v13, v24, v25, 24\n" TAIL

#define STEP_V1                                      \
  "v_lshl_add_u64 v[10:11], v[10:11], 0, v[18:19]\n" \
  "v_add_co_u32_dpp v10, vcc, v12, v10 " QP "\n"     \
  "v_addc_co_u32_dpp v11, vcc, v13, v11, vcc " QP "\n" \
  "v_xor_b32_dpp v22, v17, v11 " QP "\n"             \
  "v_xor_b32_dpp v23, v16, v10 " QP "\n"             \
  "v_add_co_u32_dpp v14, vcc, v14, v22 " QP "\n"     \
  "v_addc_co_u32_dpp v15, vcc, v15, v23, vcc " QP "\n" \
  "v_xor_b32_dpp v24, v12, v14 " QP "\n"             \
  "v_xor_b32_dpp v25, v13, v15 " QP "\n"             \
  "v_alignbit_b32 v12, v25, v24, 24\n"               \
  "v_alignbit_b32 v13, v24, v25, 24\n" TAIL

#define R8(x) x x x x x x x x
#define CLOB "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", \
             "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "vcc"

constexpr int kIters = 2048;  // x 8 steps

template <int V>
__global__ __launch_bounds__(256) void k_step(uint64_t* out, uint32_t seed) {
  extern __shared__ uint8_t pad[];  // dynamic LDS forces one workgroup per CU
  const uint32_t x = seed + threadIdx.x;
  asm volatile(
      "v_mov_b32 v10, %0\n v_mov_b32 v11, %0\n v_mov_b32 v12, %0\n v_mov_b32 v13, %0\n"
      "v_mov_b32 v14, %0\n v_mov_b32 v15, %0\n v_mov_b32 v16, %0\n v_mov_b32 v17, %0\n"
      "v_mov_b32 v18, %0\n v_mov_b32 v19, %0\n v_mov_b32 v20, %0\n v_mov_b32 v21, %0\n"
      "s_nop 4\n" ::"v"(x) : CLOB);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
    if constexpr (V == 0) asm volatile(R8(STEP_V0) ::: CLOB);
    if constexpr (V == 1) asm volatile(R8(STEP_V1) ::: CLOB);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t r;
  asm volatile("s_nop 1\n v_mov_b32 %0, v10" : "=v"(r) :: CLOB);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = r;
  }
  (void)pad;
}

int main() {
  uint64_t* d;
  CHECK(hipMalloc(&d, 1 << 20));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const size_t lds = 96 << 10;
  void (*ks[2])(uint64_t*, uint32_t) = {k_step<0>, k_step<1>};
  const char* names[2] = {"V0 mov_dpp + lshl_add (24 VALU/step)",
                          "V1 add_co_dpp/addc_dpp (22 VALU/step)"};
  const int insts[2] = {24, 22};
  for (int v = 0; v < 2; ++v)
    CHECK(hipFuncSetAttribute((const void*)ks[v], hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds));
  for (int rep = 0; rep < 2; ++rep)
    for (int v = 0; v < 2; ++v) {
      // one wave alone
      hipLaunchKernelGGL(ks[v], dim3(1), dim3(64), lds, 0, d, 1u);
      CHECK(hipDeviceSynchronize());
      uint64_t h[2];
      CHECK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
      const double steps = 8.0 * kIters;
      // s_memtime ticks at the shader clock on gfx950? report raw ticks too
      // whole chip: 256 workgroups x 4 waves = one wave per SIMD
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(ks[v], dim3(256), dim3(256), lds, 0, d, 2u);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("%-40s alone: %.2f ticks/step (%.3f per VALU)  chip 1 wave/SIMD: %.2f ns/step"
             "  -> %.3f us per 24-step compression\n",
             names[v], h[0] / steps, h[0] / steps / insts[v], ms * 1e6 / steps,
             ms * 1e3 / steps * 24);
    }
  return 0;
}
