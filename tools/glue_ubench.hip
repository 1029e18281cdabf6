// Cost of non-G instructions between quad-mode compressions (diagnostics,
// not part of the product).  One wave runs 24 quad-mode G steps (the V1 form
// of tools/quad_dpp_ubench.hip: one compression) and then 40 "glue"
// instructions of one kind, or the 40 glue instructions spread two after
// each of the first 20 steps.  Cycles per compression for one wave alone and
// time per compression with one wave per SIMD on the whole chip; the
// difference to the no-glue body is the glue's cost.
//
//   hipcc -O3 --offload-arch=gfx950 tools/glue_ubench.hip -o build/glue_ubench
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
#define STEP                                         \
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

#define R4(x) x x x x
#define R20(x) R4(x) R4(x) R4(x) R4(x) R4(x)
#define R24(x) R20(x) R4(x)
#define R40(x) R20(x) R20(x)
// glue kinds
#define G_DS "ds_read_b64 v[30:31], v40\n"
#define G_VA "v_add_u32_e32 v32, v33, v32\n"
#define G_V3 "v_cndmask_b32_e64 v32, v33, v32, s[42:43]\n"
#define G_SA "s_add_u32 s40, s40, 1\n"
#define G_NOP "s_nop 0\n"
#define CLOB "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", \
             "v21", "v22", "v23", "v24", "v25", "v30", "v31", "v32", "v33", "v40", "s40", \
             "s41", "s42", "s43", "vcc", "scc"

constexpr int kIters = 256;  // compressions

template <int G>
__global__ __launch_bounds__(256) void k_glue(uint64_t* out, uint32_t seed) {
  extern __shared__ uint8_t pad[];  // dynamic LDS forces one workgroup per CU
  const uint32_t x = seed + threadIdx.x;
  asm volatile(
      "v_mov_b32 v10, %0\n v_mov_b32 v11, %0\n v_mov_b32 v12, %0\n v_mov_b32 v13, %0\n"
      "v_mov_b32 v14, %0\n v_mov_b32 v15, %0\n v_mov_b32 v16, %0\n v_mov_b32 v17, %0\n"
      "v_mov_b32 v18, %0\n v_mov_b32 v19, %0\n v_mov_b32 v20, %0\n v_mov_b32 v21, %0\n"
      "v_mov_b32 v32, %0\n v_mov_b32 v33, %0\n v_mov_b32 v40, 0\n s_mov_b64 s[42:43], -1\n"
      "s_nop 4\n" ::"v"(x) : CLOB);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < kIters; ++i) {
    if constexpr (G == 0) asm volatile(R24(STEP) ::: CLOB);
    if constexpr (G == 1) asm volatile(R40(G_DS) "s_waitcnt lgkmcnt(0)\n" R24(STEP) ::: CLOB);
    if constexpr (G == 2) asm volatile(R40(G_DS) R24(STEP) "s_waitcnt lgkmcnt(0)\n" ::: CLOB);
    if constexpr (G == 3)
      asm volatile(R20(STEP G_DS G_DS) R4(STEP) "s_waitcnt lgkmcnt(0)\n" ::: CLOB);
    if constexpr (G == 4) asm volatile(R40(G_VA) R24(STEP) ::: CLOB);
    if constexpr (G == 5) asm volatile(R20(STEP G_VA G_VA) R4(STEP) ::: CLOB);
    if constexpr (G == 6) asm volatile(R40(G_V3) R24(STEP) ::: CLOB);
    if constexpr (G == 7) asm volatile(R40(G_SA) R24(STEP) ::: CLOB);
    if constexpr (G == 8) asm volatile(R20(STEP G_SA G_SA) R4(STEP) ::: CLOB);
    if constexpr (G == 9) asm volatile(R40(G_NOP) R24(STEP) ::: CLOB);
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

// Tight quad loop as a hand-scheduled production loop would run it: per
// compression one vmcnt wait, 2 ds_write_b128 (the next line into LDS), 2
// global_load_dwordx4 (a later line, PF lines ahead, from HBM), 40
// ds_read_b64 (the next message set), the 24 G steps, lgkmcnt(0), 4 setup
// moves + 1 bitop3, 8 finalisation xors (6 DPP), one s_add for t; the
// pointer advances once per 2 compressions.
#define RD8(o) "ds_read_b64 v[100:101], v40 offset:" #o "\n"
#define RD40 RD8(0) RD8(8) RD8(16) RD8(24) RD8(32) RD8(40) RD8(48) RD8(56) RD8(64) RD8(72) \
  RD8(80) RD8(88) RD8(96) RD8(104) RD8(112) RD8(120) RD8(0) RD8(8) RD8(16) RD8(24) RD8(32) \
  RD8(40) RD8(48) RD8(56) RD8(64) RD8(72) RD8(80) RD8(88) RD8(96) RD8(104) RD8(112) RD8(120) \
  RD8(0) RD8(8) RD8(16) RD8(24) RD8(32) RD8(40) RD8(48) RD8(56)
#define SETUP_FIN                                                     \
  "v_mov_b64 v[10:11], v[50:51]\n v_mov_b64 v[12:13], v[52:53]\n"     \
  "v_mov_b64 v[14:15], v[54:55]\n v_mov_b32 v17, v57\n"               \
  "v_bitop3_b32 v16, v56, s46, v58 bitop3:0x78\n"                     \
  R24(STEP)                                                           \
  "s_waitcnt lgkmcnt(0)\n"                                            \
  "v_xor_b32_dpp v24, v14, v10 " QP "\n v_xor_b32_dpp v25, v15, v11 " QP "\n" \
  "v_xor_b32 v50, v50, v24\n v_xor_b32 v51, v51, v25\n"             \
  "v_xor_b32_dpp v24, v12, v52 " QP "\n v_xor_b32_dpp v25, v13, v53 " QP "\n" \
  "v_xor_b32_dpp v52, v16, v24 " QP "\n v_xor_b32_dpp v53, v17, v25 " QP "\n" \
  "s_add_u32 s46, s46, 0x80\n"
#define LOOP_A(WAIT, LD)                                              \
  "s_waitcnt vmcnt(" #WAIT ")\n"                                      \
  "ds_write_b128 v41, v[60:63]\n ds_write_b128 v41, v[64:67] offset:16\n" \
  "global_load_dwordx4 v[60:63], v[70:71], off offset:" #LD "\n"      \
  "global_load_dwordx4 v[64:67], v[70:71], off offset:" #LD "+16\n"   \
  RD40 SETUP_FIN
#define LOOP_B(WAIT, LD)                                              \
  "s_waitcnt vmcnt(" #WAIT ")\n"                                      \
  "ds_write_b128 v41, v[80:83]\n ds_write_b128 v41, v[84:87] offset:16\n" \
  "global_load_dwordx4 v[80:83], v[70:71], off offset:" #LD "\n"      \
  "global_load_dwordx4 v[84:87], v[70:71], off offset:" #LD "+16\n"   \
  RD40 SETUP_FIN "v_lshl_add_u64 v[70:71], v[70:71], 0, s[44:45]\n"
#define CLOB2 "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", \
  "v21", "v22", "v23", "v24", "v25", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", \
  "v58", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v80", "v81", "v82", "v83", \
  "v84", "v85", "v86", "v87", "v100", "v101", "s44", "s45", "s46", "vcc", "scc", "memory"

// PF = 2: line j+3 loaded at compression j (two register sets, vmcnt(2));
// PF = 1: line j+2, waited one compression later (vmcnt(0)).
template <int PF>
__global__ __launch_bounds__(256) void k_tight(uint64_t* out, const uint8_t* buf) {
  extern __shared__ uint8_t pad[];
  const uint32_t lane = threadIdx.x & 63u, q = lane >> 2, i = lane & 3u;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint8_t* p = buf + ((wave * 16 + q) << 15) + 32 * i;  // 32 KiB per chain
  const uint32_t lds_line = (threadIdx.x >> 6) * 2048 + q * 128;
  const uint32_t rd = lds_line + i * 8, wr = lds_line + 32 * i;
  const uint32_t m0 = i == 0 ? ~0u : 0u;
  asm volatile(
      "v_mov_b32 v10, %0\n v_mov_b32 v11, %0\n v_mov_b32 v12, %0\n v_mov_b32 v13, %0\n"
      "v_mov_b32 v14, %0\n v_mov_b32 v15, %0\n v_mov_b32 v16, %0\n v_mov_b32 v17, %0\n"
      "v_mov_b32 v18, %0\n v_mov_b32 v19, %0\n v_mov_b32 v20, %0\n v_mov_b32 v21, %0\n"
      "v_mov_b64 v[50:51], v[10:11]\n v_mov_b64 v[52:53], v[10:11]\n v_mov_b64 v[54:55], v[10:11]\n"
      "v_mov_b64 v[56:57], v[10:11]\n v_mov_b32 v58, %4\n"
      "v_mov_b32 v40, %2\n v_mov_b32 v41, %3\n v_mov_b64 v[70:71], %1\n"
      "s_mov_b32 s44, 0x100\n s_mov_b32 s45, 0\n s_mov_b32 s46, 0\n"
      "global_load_dwordx4 v[60:63], v[70:71], off offset:128\n"
      "global_load_dwordx4 v[64:67], v[70:71], off offset:144\n"
      "global_load_dwordx4 v[80:83], v[70:71], off offset:256\n"
      "global_load_dwordx4 v[84:87], v[70:71], off offset:272\n"
      "s_nop 4\n" ::"v"((uint32_t)wave), "v"(p), "v"(rd), "v"(wr), "v"(m0)
      : CLOB2, "v40", "v41", "v70", "v71");
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < 126; it += 2) {  // 252 compressions, every load in bounds
    if constexpr (PF == 2)
      asm volatile(LOOP_A(2, 384) LOOP_B(2, 512) ::: CLOB2, "v70", "v71");
    else
      asm volatile(LOOP_A(0, 384) LOOP_B(0, 512) ::: CLOB2, "v70", "v71");
  }
  asm volatile("s_waitcnt vmcnt(0)\n" ::: "memory");
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t r;
  asm volatile("s_nop 1\n v_mov_b32 %0, v50" : "=v"(r) :: CLOB2);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = r;
  }
  (void)pad;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  uint64_t* d;
  CHECK(hipMalloc(&d, 1 << 20));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const size_t lds = 96 << 10;
  void (*ks[])(uint64_t*, uint32_t) = {k_glue<0>, k_glue<1>, k_glue<2>, k_glue<3>, k_glue<4>,
                                       k_glue<5>, k_glue<6>, k_glue<7>, k_glue<8>, k_glue<9>};
  const char* names[] = {"no glue",
                         "40 ds_read_b64 grouped, wait before",
                         "40 ds_read_b64 grouped, wait after",
                         "40 ds_read_b64 2 per step",
                         "40 v_add_u32 grouped",
                         "40 v_add_u32 2 per step",
                         "40 v_cndmask_b32_e64 grouped",
                         "40 s_add_u32 grouped",
                         "40 s_add_u32 2 per step",
                         "40 s_nop 0 grouped"};
  const int nk = sizeof(ks) / sizeof(ks[0]);
  for (int v = 0; v < nk; ++v)
    CHECK(hipFuncSetAttribute((const void*)ks[v], hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds));
  double base_a = 0, base_c = 0;
  for (int rep = 0; rep < 2; ++rep)
    for (int v = 0; v < nk; ++v) {
      hipLaunchKernelGGL(ks[v], dim3(1), dim3(64), lds, 0, d, 1u);
      CHECK(hipDeviceSynchronize());
      uint64_t h[2];
      CHECK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(ks[v], dim3(256), dim3(256), lds, 0, d, 2u);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double alone = (double)h[0] / kIters, chip = ms * 1e6 / kIters;
      if (v == 0) base_a = alone, base_c = chip;
      printf("%-38s alone %7.1f cycles/compression (%+6.1f, %+5.2f per glue instr)  chip %7.1f ns"
             " (%+6.1f)\n",
             names[v], alone, alone - base_a, (alone - base_a) / 40, chip, chip - base_c);
    }
  uint8_t* buf;
  CHECK(hipMalloc(&buf, (size_t)1024 * 16 << 15));  // 1024 waves x 16 chains x 32 KiB
  CHECK(hipMemset(buf, 1, (size_t)1024 * 16 << 15));
  void (*kt[])(uint64_t*, const uint8_t*) = {k_tight<1>, k_tight<2>};
  for (int rep = 0; rep < 2; ++rep)
    for (int v = 0; v < 2; ++v) {
      CHECK(hipFuncSetAttribute((const void*)kt[v], hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
      hipLaunchKernelGGL(kt[v], dim3(1), dim3(64), lds, 0, d, buf);
      CHECK(hipDeviceSynchronize());
      uint64_t h[2];
      CHECK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(kt[v], dim3(256), dim3(256), lds, 0, d, buf);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("tight loop, global prefetch %d line(s) ahead: alone %7.1f cycles/compression  chip"
             " %7.1f ns/compression\n", v + 1, (double)h[0] / 252, ms * 1e6 / 252);
    }
  return 0;
}
