// Does the 8-byte alignment of 8-byte (VOP3 / DPP / DS) instructions change
// their issue rate on gfx950?  (diagnostics, not part of the product)
// Loop bodies of independent instructions, each preceded by one or two
// s_nop 0 after a 16-B alignment, so the body starts 4 mod 8 or 0 mod 8.
// One wave per SIMD and 8 waves per SIMD on the whole chip.
//
//   hipcc -O3 --offload-arch=gfx950 tools/align_ubench.hip -o build/align_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define R8(x) x x x x x x x x
#define ADD8                                           \
  "v_lshl_add_u64 v[10:11], v[10:11], 0, v[26:27]\n"   \
  "v_lshl_add_u64 v[12:13], v[12:13], 0, v[26:27]\n"   \
  "v_lshl_add_u64 v[14:15], v[14:15], 0, v[26:27]\n"   \
  "v_lshl_add_u64 v[16:17], v[16:17], 0, v[26:27]\n"   \
  "v_lshl_add_u64 v[18:19], v[18:19], 0, v[26:27]\n"   \
  "v_lshl_add_u64 v[20:21], v[20:21], 0, v[26:27]\n"   \
  "v_lshl_add_u64 v[22:23], v[22:23], 0, v[26:27]\n"   \
  "v_lshl_add_u64 v[24:25], v[24:25], 0, v[26:27]\n"
#define ALN8                                           \
  "v_alignbit_b32 v30, v30, v27, 24\n v_alignbit_b32 v31, v31, v27, 24\n" \
  "v_alignbit_b32 v32, v32, v27, 24\n v_alignbit_b32 v33, v33, v27, 24\n" \
  "v_alignbit_b32 v34, v34, v27, 24\n v_alignbit_b32 v35, v35, v27, 24\n" \
  "v_alignbit_b32 v36, v36, v27, 24\n v_alignbit_b32 v37, v37, v27, 24\n"
#define XOR8                                           \
  "v_xor_b32 v40, v40, v27\n v_xor_b32 v41, v41, v27\n v_xor_b32 v42, v42, v27\n" \
  "v_xor_b32 v43, v43, v27\n v_xor_b32 v44, v44, v27\n v_xor_b32 v45, v45, v27\n" \
  "v_xor_b32 v46, v46, v27\n v_xor_b32 v47, v47, v27\n"
#define CLOB "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", \
  "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v30", "v31", "v32", "v33", "v34", "v35", \
  "v36", "v37", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "vcc"
#define QP " quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"
#define DPP8                                                             \
  "v_xor_b32_dpp v40, v27, v40" QP "v_xor_b32_dpp v41, v27, v41" QP        \
  "v_xor_b32_dpp v42, v27, v42" QP "v_xor_b32_dpp v43, v27, v43" QP        \
  "v_add_co_u32_dpp v44, vcc, v27, v44" QP "v_addc_co_u32_dpp v45, vcc, v27, v45, vcc" QP \
  "v_xor_b32_dpp v46, v27, v46" QP "v_xor_b32_dpp v47, v27, v47" QP
// the quad-mode G step (tools/quad_dpp_ubench.hip V1), a dependent chain
#define QSTEP                                                           \
  "v_lshl_add_u64 v[10:11], v[10:11], 0, v[18:19]\n"                    \
  "v_add_co_u32_dpp v10, vcc, v12, v10" QP                                \
  "v_addc_co_u32_dpp v11, vcc, v13, v11, vcc" QP                          \
  "v_xor_b32_dpp v22, v17, v11" QP "v_xor_b32_dpp v23, v16, v10" QP       \
  "v_add_co_u32_dpp v14, vcc, v14, v22" QP                                \
  "v_addc_co_u32_dpp v15, vcc, v15, v23, vcc" QP                          \
  "v_xor_b32_dpp v24, v12, v14" QP "v_xor_b32_dpp v25, v13, v15" QP       \
  "v_alignbit_b32 v12, v25, v24, 24\n v_alignbit_b32 v13, v24, v25, 24\n" \
  "v_lshl_add_u64 v[10:11], v[10:11], 0, v[20:21]\n"                    \
  "v_lshl_add_u64 v[10:11], v[10:11], 0, v[12:13]\n"                    \
  "v_xor_b32 v24, v22, v10\n v_xor_b32 v25, v23, v11\n"                 \
  "v_alignbit_b32 v16, v25, v24, 16\n v_alignbit_b32 v17, v24, v25, 16\n" \
  "v_lshl_add_u64 v[14:15], v[14:15], 0, v[16:17]\n"                    \
  "v_xor_b32 v24, v12, v14\n v_xor_b32 v25, v13, v15\n"                 \
  "v_alignbit_b32 v12, v24, v25, 31\n v_alignbit_b32 v13, v25, v24, 31\n"
#define BODY_D R8(DPP8)
#define BODY_Q R8(QSTEP)
#define BODY_A R8(ADD8)                 // 64 x 8-byte
#define BODY_M R4M(ADD8 XOR8 ALN8 XOR8)  // 8-byte runs between even runs of 4-byte
#define R4M(x) x x x x

#define LOOP(PRE, BODY)                                                       \
  asm volatile("s_mov_b32 s40, %0\n"                                           \
               ".p2align 6\n"                                                  \
               "1:\n" PRE BODY                                                 \
               "s_sub_u32 s40, s40, 1\n"                                       \
               "s_cmp_lg_u32 s40, 0\n"                                         \
               "s_cbranch_scc1 1b\n" ::"s"(iters)                              \
               : CLOB, "s40", "scc")

template <int V>
__global__ __launch_bounds__(256) void k_align(uint32_t* out, int iters) {
  asm volatile("v_mov_b32 v26, 1\n v_mov_b32 v27, 3\n" ::: CLOB);
  // aligned: two s_nop 0 then the body (0 mod 8); misaligned: one (4 mod 8)
  if constexpr (V == 0) LOOP("s_nop 0\n s_nop 0\n", BODY_A);
  if constexpr (V == 1) LOOP("s_nop 0\n", BODY_A);
  if constexpr (V == 2) LOOP("s_nop 0\n s_nop 0\n", BODY_M);
  if constexpr (V == 3) LOOP("s_nop 0\n", BODY_M);
  if constexpr (V == 4) LOOP("s_nop 0\n s_nop 0\n", BODY_D);
  if constexpr (V == 5) LOOP("s_nop 0\n", BODY_D);
  if constexpr (V == 6) LOOP("s_nop 0\n s_nop 0\n", BODY_Q);
  if constexpr (V == 7) LOOP("s_nop 0\n", BODY_Q);
  uint32_t r;
  asm volatile("v_mov_b32 %0, v10" : "=v"(r)::CLOB);
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  uint32_t* d;
  if (hipMalloc(&d, 64 << 20) != hipSuccess) return 1;
  void (*ks[])(uint32_t*, int) = {k_align<0>, k_align<1>, k_align<2>, k_align<3>,
                                   k_align<4>, k_align<5>, k_align<6>, k_align<7>};
  const char* names[] = {"64 v_lshl_add_u64, body 0 mod 8 (+2 nop)",
                         "64 v_lshl_add_u64, body 4 mod 8 (+1 nop)",
                         "mixed add/xor/alignbit, 0 mod 8 (+2 nop)",
                         "mixed add/xor/alignbit, 4 mod 8 (+1 nop)",
                         "64 DPP xor/add_co, 0 mod 8 (+2 nop)",
                         "64 DPP xor/add_co, 4 mod 8 (+1 nop)",
                         "8 quad G steps (chain), 0 mod 8 (+2 nop)",
                         "8 quad G steps (chain), 4 mod 8 (+1 nop)"};
  const int insts[] = {69, 68, 133, 132, 69, 68, 181, 180};
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int iters = 4096;
  for (int rep = 0; rep < 2; ++rep)
    for (int wps : {1, 8})
      for (int v = 0; v < 8; ++v) {
        const int wgs = 256 * wps;  // 256 CUs x 4 SIMDs x wps waves, 4 waves per WG
        hipLaunchKernelGGL(ks[v], dim3(wgs), dim3(256), 0, 0, d, 16);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(ks[v], dim3(wgs), dim3(256), 0, 0, d, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        const double winst_per_simd = (double)wps * iters * insts[v];
        printf("waves/SIMD %d  %-42s %8.3f ms  %.2f ns per wave instruction per SIMD\n", wps,
               names[v], ms, ms * 1e6 / winst_per_simd);
      }
  return 0;
}
