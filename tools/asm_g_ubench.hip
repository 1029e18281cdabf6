// Hand-ordered G sequences in inline asm (diagnostics, not part of the
// product): one half-round (4 independent G, 80 VALU instructions) repeated
// 24 x 256 times per lane over 1 M lanes, i.e. the VALU work of the config-2
// compression with no message loads, in three issue orders.  Compare with
// order_ubench's compress-only (12.9 ms).
//
//   hipcc -O3 --offload-arch=gfx950 tools/asm_g_ubench.hip -o build/asm_g_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "asm_g_bodies.h"

#define CLOBBERS "v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61"

template <int K, int OCC>
__global__ __launch_bounds__(256, OCC) void k_asm(uint32_t* out, int iters) {
  for (int i = 0; i < iters; ++i) {
    if constexpr (K == 0) asm volatile(ASM_HALF_GMAJOR ::: CLOBBERS);
    if constexpr (K == 1) asm volatile(ASM_HALF_RR ::: CLOBBERS);
    if constexpr (K == 2) asm volatile(ASM_HALF_STEP ::: CLOBBERS);
    if constexpr (K == 3) asm volatile(ASM_HALF_STEP_SMSG ::: CLOBBERS, "s40", "s41", "s42", "s43");
    if constexpr (K == 4) asm volatile(ASM_HALF_STEP_ALIGNXOR ::: CLOBBERS);
    if constexpr (K == 5) asm volatile(ASM_HALF_STEP_ADDXOR ::: CLOBBERS);
    if constexpr (K == 6) asm volatile(ASM_HALF_INDEP_MIX ::: CLOBBERS);
  }
  uint32_t v;
  asm volatile("v_mov_b32 %0, v10" : "=v"(v));
  out[blockIdx.x * 256 + threadIdx.x] = v;
}

typedef void (*K)(uint32_t*, int);

int main() {
  const int lanes = 1 << 20, iters = 24 * 256;
  uint32_t* d;
  if (hipMalloc(&d, lanes * 4) != hipSuccess) return 1;
  struct {
    const char* name;
    K k;
  } ks[] = {{"G-major (compiler-like)   occ 5", k_asm<0, 5>},
            {"round-robin over 4 G      occ 5", k_asm<1, 5>},
            {"step-major (production)   occ 5", k_asm<2, 5>},
            {"G-major                   occ 8", k_asm<0, 8>},
            {"step-major                occ 8", k_asm<2, 8>},
            {"step-major, messages in SGPRs (probe)    occ 5", k_asm<3, 5>},
            {"step-major, alignbit -> v_xor (probe)    occ 5", k_asm<4, 5>},
            {"step-major, 64-bit add -> v_xor (probe)  occ 5", k_asm<5, 5>},
            {"same class mix, no dependencies (probe)  occ 5", k_asm<6, 5>}};
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
      const double winst = (double)lanes / 64 * iters * 80;  // wave instructions
      printf("%s: %.3f ms  %.2f cycles per wave instruction per SIMD at 2.37 GHz\n", k.name, ms,
             ms * 1e-3 * 2.37e9 * 1024 / winst);
    }
  return 0;
}
