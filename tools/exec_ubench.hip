// Does a partially filled wave issue VALU faster?  (diagnostics, not part of
// the product).  One wave alone runs a dependent chain of quad-mode G steps
// (the same body as tools/glue_ubench.hip) with 64, 32, 16 or 4 lanes
// launched, and with a full wave whose exec mask is cut to 16 / 4 lanes by a
// branch.  If wave64 VALU always takes 4 passes, cycles per compression do
// not move; if the hardware skips empty 16-lane groups, a 16-lane wave runs
// ~4x faster and long chains could be packed 4 per wave.
//
//   hipcc -O3 --offload-arch=gfx950 tools/exec_ubench.hip -o build/exec_ubench
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
#define STEP                                           \
  "v_lshl_add_u64 v[10:11], v[10:11], 0, v[18:19]\n"   \
  "v_add_co_u32_dpp v10, vcc, v12, v10 " QP "\n"       \
  "v_addc_co_u32_dpp v11, vcc, v13, v11, vcc " QP "\n" \
  "v_xor_b32_dpp v22, v17, v11 " QP "\n"               \
  "v_xor_b32_dpp v23, v16, v10 " QP "\n"               \
  "v_add_co_u32_dpp v14, vcc, v14, v22 " QP "\n"       \
  "v_addc_co_u32_dpp v15, vcc, v15, v23, vcc " QP "\n" \
  "v_xor_b32_dpp v24, v12, v14 " QP "\n"               \
  "v_xor_b32_dpp v25, v13, v15 " QP "\n"               \
  "v_alignbit_b32 v12, v25, v24, 24\n"                 \
  "v_alignbit_b32 v13, v24, v25, 24\n"                 \
  "v_lshl_add_u64 v[10:11], v[10:11], 0, v[20:21]\n"   \
  "v_lshl_add_u64 v[10:11], v[10:11], 0, v[12:13]\n"   \
  "v_xor_b32 v24, v22, v10\n"                          \
  "v_xor_b32 v25, v23, v11\n"                          \
  "v_alignbit_b32 v16, v25, v24, 16\n"                 \
  "v_alignbit_b32 v17, v24, v25, 16\n"                 \
  "v_lshl_add_u64 v[14:15], v[14:15], 0, v[16:17]\n"   \
  "v_xor_b32 v24, v12, v14\n"                          \
  "v_xor_b32 v25, v13, v15\n"                          \
  "v_alignbit_b32 v12, v24, v25, 31\n"                 \
  "v_alignbit_b32 v13, v25, v24, 31\n"
// plain VALU chain without DPP or 64-bit ops: 22 dependent v_xor/v_add
#define PLAIN                                                                   \
  "v_add_u32 v10, v10, v11\n v_xor_b32 v11, v11, v10\n v_add_u32 v10, v10, v11\n" \
  "v_xor_b32 v11, v11, v10\n v_add_u32 v10, v10, v11\n v_xor_b32 v11, v11, v10\n" \
  "v_add_u32 v10, v10, v11\n v_xor_b32 v11, v11, v10\n v_add_u32 v10, v10, v11\n" \
  "v_xor_b32 v11, v11, v10\n v_add_u32 v10, v10, v11\n v_xor_b32 v11, v11, v10\n" \
  "v_add_u32 v10, v10, v11\n v_xor_b32 v11, v11, v10\n v_add_u32 v10, v10, v11\n" \
  "v_xor_b32 v11, v11, v10\n v_add_u32 v10, v10, v11\n v_xor_b32 v11, v11, v10\n" \
  "v_add_u32 v10, v10, v11\n v_xor_b32 v11, v11, v10\n v_add_u32 v10, v10, v11\n" \
  "v_xor_b32 v11, v11, v10\n"
#define R4(x) x x x x
#define R24(x) R4(x) R4(x) R4(x) R4(x) R4(x) R4(x)
#define CLOB "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", \
             "v21", "v22", "v23", "v24", "v25", "vcc", "scc"

constexpr int kIters = 256;  // compressions (24 steps of 22 instructions each)

// body 0: quad G steps, 1: plain VALU chain.  lanes: threads < lanes run the
// loop (the rest of the wave is masked off by the branch).
template <int B>
__global__ __launch_bounds__(64) void k_exec(uint64_t* out, uint32_t seed, uint32_t lanes) {
  const uint32_t x = seed + threadIdx.x;
  uint64_t dt = 0;
  uint32_t r = 0;
  if (threadIdx.x < lanes) {
    asm volatile(
        "v_mov_b32 v10, %0\n v_mov_b32 v11, %0\n v_mov_b32 v12, %0\n v_mov_b32 v13, %0\n"
        "v_mov_b32 v14, %0\n v_mov_b32 v15, %0\n v_mov_b32 v16, %0\n v_mov_b32 v17, %0\n"
        "v_mov_b32 v18, %0\n v_mov_b32 v19, %0\n v_mov_b32 v20, %0\n v_mov_b32 v21, %0\n"
        "s_nop 4\n" ::"v"(x) : CLOB);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < kIters; ++i) {
      if constexpr (B == 0) asm volatile(R24(STEP) ::: CLOB);
      if constexpr (B == 1) asm volatile(R24(PLAIN) ::: CLOB);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_nop 1\n v_mov_b32 %0, v10" : "=v"(r) :: CLOB);
    dt = t1 - t0;
  }
  if (threadIdx.x == 0) {
    out[0] = dt;
    out[1] = r;
  }
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  uint64_t* d;
  CHECK(hipMalloc(&d, 4096));
  const char* bodies[] = {"quad G steps", "plain v_add/v_xor"};
  void (*ks[])(uint64_t*, uint32_t, uint32_t) = {k_exec<0>, k_exec<1>};
  for (int rep = 0; rep < 2; ++rep)
    for (int b = 0; b < 2; ++b) {
      const unsigned launched[] = {64, 32, 16, 4, 64, 64, 64};
      const unsigned active[] = {64, 32, 16, 4, 16, 4, 1};
      for (int v = 0; v < 7; ++v) {
        hipLaunchKernelGGL(ks[b], dim3(1), dim3(launched[v]), 0, 0, d, 1u, active[v]);
        CHECK(hipDeviceSynchronize());
        uint64_t h[2];
        CHECK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
        printf("%-18s launched %2u lanes, %2u active: %7.1f cycles per 528 instructions"
               " (%.2f per instruction)\n",
               bodies[b], launched[v], active[v], (double)h[0] / kIters,
               (double)h[0] / kIters / 528.0);
      }
    }
  return 0;
}
