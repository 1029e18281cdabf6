// Class-mix issue probe (diagnostics, not part of the product): 80-instruction
// bodies of independent 64-bit adds (A: v_lshl_add_u64, As: its SGPR-operand
// form, C: v_add_co/v_addc pair), funnel shifts (L: v_alignbit_b32) and
// xors (X: v_xor_b32) in several mixes, 5 waves per SIMD, 1 M lanes.
//
//   hipcc -O3 --offload-arch=gfx950 -Itools tools/mix_ubench.hip -o build/mix_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "mix_bodies.h"

#define CLOBBERS "v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","s40","s41","vcc"

template <int K>
__global__ __launch_bounds__(256, 5) void k_mix(uint32_t* out, int iters) {
  for (int i = 0; i < iters; ++i) {
    if constexpr (K == 0) asm volatile(MIX_A ::: CLOBBERS);
    if constexpr (K == 1) asm volatile(MIX_L ::: CLOBBERS);
    if constexpr (K == 2) asm volatile(MIX_X ::: CLOBBERS);
    if constexpr (K == 3) asm volatile(MIX_AX ::: CLOBBERS);
    if constexpr (K == 4) asm volatile(MIX_LX ::: CLOBBERS);
    if constexpr (K == 5) asm volatile(MIX_AL ::: CLOBBERS);
    if constexpr (K == 6) asm volatile(MIX_A8X8 ::: CLOBBERS);
    if constexpr (K == 7) asm volatile(MIX_AsX ::: CLOBBERS);
    if constexpr (K == 8) asm volatile(MIX_As ::: CLOBBERS);
    if constexpr (K == 9) asm volatile(MIX_CX ::: CLOBBERS);
    if constexpr (K == 10) asm volatile(MIX_A16X16 ::: CLOBBERS);
    if constexpr (K == 11) asm volatile(MIX_A40X40 ::: CLOBBERS);
    if constexpr (K == 12) asm volatile(MIX_A4X12 ::: CLOBBERS);
  }
  uint32_t v;
  asm volatile("v_mov_b32 %0, v10" : "=v"(v));
  out[blockIdx.x * 256 + threadIdx.x] = v;
}

typedef void (*Kf)(uint32_t*, int);

int main() {
  const int lanes = 1 << 20, iters = 2048;
  uint32_t* d;
  if (hipMalloc(&d, lanes * 4) != hipSuccess) return 1;
  struct { const char* name; Kf k; } ks[] = {
      {"A", k_mix<0>},
      {"L", k_mix<1>},
      {"X", k_mix<2>},
      {"AX", k_mix<3>},
      {"LX", k_mix<4>},
      {"AL", k_mix<5>},
      {"A8X8", k_mix<6>},
      {"AsX", k_mix<7>},
      {"As", k_mix<8>},
      {"CX", k_mix<9>},
      {"A16X16", k_mix<10>},
      {"A40X40", k_mix<11>},
      {"A4X12", k_mix<12>}
  };
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int pass = 0; pass < 2; ++pass)
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.k, dim3(lanes / 256), dim3(256), 0, 0, d, iters);
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(k.k, dim3(lanes / 256), dim3(256), 0, 0, d, iters);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      const double winst = (double)lanes / 64 * iters * 80;
      printf("%-6s %8.3f ms  %.2f cycles per wave instruction per SIMD at 2.37 GHz\n", k.name, ms,
             ms * 1e-3 * 2.37e9 * 1024 / winst);
    }
  return 0;
}
