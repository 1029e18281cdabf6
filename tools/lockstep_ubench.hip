// Lockstep probe (diagnostics, not part of the product): do two waves on one
// SIMD kept in phase by s_barrier (a 512-thread workgroup = 2 waves per
// SIMD, one workgroup per CU) issue their full-rate instructions in pairs?
//
//   hipcc -O3 --offload-arch=gfx950 -Itools tools/lockstep_ubench.hip -o build/lockstep_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "asm_g_bodies.h"
#include "mix_bodies.h"

#define CLOBBERS "v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61"

// K: 0 AX, 1 G half-round (step-major), 2 X only, 3 A only; B: barrier every iteration
template <int K, int B, int WG>
__global__ __launch_bounds__(WG) void k_ls(uint32_t* out, int iters) {
  for (int i = 0; i < iters; ++i) {
    if constexpr (K == 0) asm volatile(MIX_AX ::: CLOBBERS);
    if constexpr (K == 1) asm volatile(ASM_HALF_STEP ::: CLOBBERS);
    if constexpr (K == 2) asm volatile(MIX_X ::: CLOBBERS);
    if constexpr (K == 3) asm volatile(MIX_A ::: CLOBBERS);
    if constexpr (B) __builtin_amdgcn_s_barrier();
  }
  uint32_t v;
  asm volatile("v_mov_b32 %0, v10" : "=v"(v));
  out[blockIdx.x * WG + threadIdx.x] = v;
}

typedef void (*Kf)(uint32_t*, int);

int main() {
  uint32_t* d;
  if (hipMalloc(&d, 1 << 24) != hipSuccess) return 1;
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  struct { const char* name; Kf k; int wg; } ks[] = {
      {"AX  wg512 (2 waves/SIMD) no barrier", k_ls<0, 0, 512>, 512},
      {"AX  wg512 (2 waves/SIMD) barrier/80", k_ls<0, 1, 512>, 512},
      {"G   wg512 (2 waves/SIMD) no barrier", k_ls<1, 0, 512>, 512},
      {"G   wg512 (2 waves/SIMD) barrier/80", k_ls<1, 1, 512>, 512},
      {"X   wg512 (2 waves/SIMD) no barrier", k_ls<2, 0, 512>, 512},
      {"A   wg512 (2 waves/SIMD) no barrier", k_ls<3, 0, 512>, 512},
      {"AX  wg1024 (4 waves/SIMD) barrier/80", k_ls<0, 1, 1024>, 1024},
      {"G   wg1024 (4 waves/SIMD) barrier/80", k_ls<1, 1, 1024>, 1024},
      {"G   wg1024 (4 waves/SIMD) no barrier", k_ls<1, 0, 1024>, 1024},
  };
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int iters = 4096;
  for (int pass = 0; pass < 2; ++pass)
    for (auto& k : ks) {
      const int grid = cus * 4;  // 4 workgroups per CU over time
      hipLaunchKernelGGL(k.k, dim3(grid), dim3(k.wg), 0, 0, d, iters);
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(k.k, dim3(grid), dim3(k.wg), 0, 0, d, iters);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      const double winst = (double)grid * (k.wg / 64) * iters * 80;
      printf("%-40s %8.3f ms  %.2f cycles per wave instruction per SIMD at 2.37 GHz\n", k.name,
             ms, ms * 1e-3 * 2.37e9 * cus * 4 / winst);
    }
  return 0;
}
