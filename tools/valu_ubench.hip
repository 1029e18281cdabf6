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

#include <algorithm>
#include <map>
#include <set>
#include <vector>

#include "blake2b_dev.hpp"
#include "blake2b_variants.hpp"
#include "uniform.hpp"

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
  X(mix_3slow_2fast, 5,                                                                          \
    asm volatile("v_alignbit_b32 %0, %0, %2, 24\n\tv_alignbit_b32 %1, %1, %2, 24\n\t"           \
                 "v_lshl_add_u64 %3, %3, 0, %4\n\tv_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %2"   \
                 : "+v"(a[i]), "+v"(b[i]), "+v"(a[k]), "+v"(w[i]) : "v"(w[j])))                  \
  X(alt_slow_fast, 2,                                                                            \
    asm volatile("v_alignbit_b32 %0, %0, %1, 24\n\tv_xor_b32 %1, %1, %2"                         \
                 : "+v"(a[i]), "+v"(b[i]) : "v"(a[k])))                                            \
  X(grp4_slow_4fast, 8,                                                                          \
    asm volatile("v_alignbit_b32 %0, %0, %4, 24\n\tv_alignbit_b32 %1, %1, %4, 24\n\t"           \
                 "v_alignbit_b32 %2, %2, %4, 24\n\tv_alignbit_b32 %3, %3, %4, 24\n\t"           \
                 "v_xor_b32 %0, %0, %4\n\tv_xor_b32 %1, %1, %4\n\t"                             \
                 "v_xor_b32 %2, %2, %4\n\tv_xor_b32 %3, %3, %4"                                   \
                 : "+v"(a[i]), "+v"(b[i]), "+v"(a[j]), "+v"(b[j]) : "v"(a[k])))                    \
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

// Pairing probes: one 512-thread workgroup per CU = 2 waves per SIMD (waves
// w and w+4 share a SIMD).  ROLE_A / ROLE_B: 0 = slow (alignbit), 1 = fast
// (xor), 2 = alternate slow/fast.
template <int ROLE_A, int ROLE_B>
__global__ __launch_bounds__(512) void k_pair(uint32_t* out, int iters) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int role = wave < 4 ? ROLE_A : ROLE_B;
  uint32_t a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 7 + i;
    b[i] = threadIdx.x ^ (i * 0x9e3779b9u);
  }
  if (role == 0) {
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(a[i]) : "v"(b[i]));
  } else if (role == 1) {
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
  } else {
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i)
          asm volatile("v_alignbit_b32 %0, %0, %1, 24\n\tv_xor_b32 %1, %1, %0" : "+v"(a[i]), "+v"(b[i]));
  }
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= a[i] ^ b[i];
  out[blockIdx.x * 512 + threadIdx.x] = x;
}

// Bank probes with hand-assigned VGPRs (bank = register index mod 4 is the
// hypothesis).  8 independent destinations per statement.
#define BANK_KERNEL(NAME, BODY)                                                      \
  __global__ __launch_bounds__(256) void k_bank_##NAME(uint32_t* out, int iters) {  \
    asm volatile("v_mov_b32 v0, %0\n\tv_mov_b32 v1, %0\n\tv_mov_b32 v2, %0\n\t"      \
                 "v_mov_b32 v3, %0\n\tv_mov_b32 v4, %0\n\tv_mov_b32 v5, %0\n\t"       \
                 "v_mov_b32 v6, %0\n\tv_mov_b32 v7, %0\n\tv_mov_b32 v8, %0\n\t"       \
                 "v_mov_b32 v9, %0\n\tv_mov_b32 v10, %0\n\tv_mov_b32 v11, %0\n\t"     \
                 "v_mov_b32 v12, %0\n\tv_mov_b32 v13, %0\n\tv_mov_b32 v14, %0\n\t"    \
                 "v_mov_b32 v15, %0\n\tv_mov_b32 v16, %0\n\tv_mov_b32 v17, %0\n\t"    \
                 "v_mov_b32 v18, %0\n\tv_mov_b32 v19, %0\n\tv_mov_b32 v20, %0\n\t"    \
                 "v_mov_b32 v21, %0\n\tv_mov_b32 v22, %0\n\tv_mov_b32 v23, %0"          \
                 ::"v"(threadIdx.x) : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7",    \
                 "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17",      \
                 "v18", "v19", "v20", "v21", "v22", "v23");                             \
    for (int it = 0; it < iters; ++it) {                                              \
      _Pragma("unroll") for (int r = 0; r < 16; ++r) {                                \
        asm volatile(BODY ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8",   \
                     "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17",     \
                     "v18", "v19", "v20", "v21", "v22", "v23");                       \
      }                                                                               \
    }                                                                                 \
    uint32_t x;                                                                       \
    asm volatile("v_xor_b32 %0, v0, v1" : "=v"(x));                                   \
    out[blockIdx.x * 256 + threadIdx.x] = x;                                          \
  }
// alignbit: dst/src0 in banks 0..3 (v0..v7), src1 in a different bank
BANK_KERNEL(alignbit_nc,
            "v_alignbit_b32 v0, v0, v9, 24\n\tv_alignbit_b32 v1, v1, v10, 24\n\t"
            "v_alignbit_b32 v2, v2, v11, 24\n\tv_alignbit_b32 v3, v3, v8, 24\n\t"
            "v_alignbit_b32 v4, v4, v13, 24\n\tv_alignbit_b32 v5, v5, v14, 24\n\t"
            "v_alignbit_b32 v6, v6, v15, 24\n\tv_alignbit_b32 v7, v7, v12, 24")
// alignbit: src0 and src1 in the same bank
BANK_KERNEL(alignbit_c,
            "v_alignbit_b32 v0, v0, v8, 24\n\tv_alignbit_b32 v1, v1, v9, 24\n\t"
            "v_alignbit_b32 v2, v2, v10, 24\n\tv_alignbit_b32 v3, v3, v11, 24\n\t"
            "v_alignbit_b32 v4, v4, v12, 24\n\tv_alignbit_b32 v5, v5, v13, 24\n\t"
            "v_alignbit_b32 v6, v6, v14, 24\n\tv_alignbit_b32 v7, v7, v15, 24")
BANK_KERNEL(xor_nc,
            "v_xor_b32 v0, v0, v9\n\tv_xor_b32 v1, v1, v10\n\tv_xor_b32 v2, v2, v11\n\t"
            "v_xor_b32 v3, v3, v8\n\tv_xor_b32 v4, v4, v13\n\tv_xor_b32 v5, v5, v14\n\t"
            "v_xor_b32 v6, v6, v15\n\tv_xor_b32 v7, v7, v12")
BANK_KERNEL(xor_c,
            "v_xor_b32 v0, v0, v8\n\tv_xor_b32 v1, v1, v9\n\tv_xor_b32 v2, v2, v10\n\t"
            "v_xor_b32 v3, v3, v11\n\tv_xor_b32 v4, v4, v12\n\tv_xor_b32 v5, v5, v13\n\t"
            "v_xor_b32 v6, v6, v14\n\tv_xor_b32 v7, v7, v15")
// 64-bit adds: operand pairs {0,1}+{2,3} (disjoint banks) vs {0,1}+{0,1}
BANK_KERNEL(lshladd_nc,
            "v_lshl_add_u64 v[0:1], v[0:1], 0, v[10:11]\n\tv_lshl_add_u64 v[4:5], v[4:5], 0, v[14:15]\n\t"
            "v_lshl_add_u64 v[2:3], v[2:3], 0, v[8:9]\n\tv_lshl_add_u64 v[6:7], v[6:7], 0, v[12:13]\n\t"
            "v_lshl_add_u64 v[16:17], v[16:17], 0, v[18:19]\n\tv_lshl_add_u64 v[20:21], v[20:21], 0, v[22:23]\n\t"
            "v_lshl_add_u64 v[18:19], v[18:19], 0, v[16:17]\n\tv_lshl_add_u64 v[22:23], v[22:23], 0, v[20:21]")
BANK_KERNEL(lshladd_c,
            "v_lshl_add_u64 v[0:1], v[0:1], 0, v[8:9]\n\tv_lshl_add_u64 v[4:5], v[4:5], 0, v[12:13]\n\t"
            "v_lshl_add_u64 v[2:3], v[2:3], 0, v[10:11]\n\tv_lshl_add_u64 v[6:7], v[6:7], 0, v[14:15]\n\t"
            "v_lshl_add_u64 v[16:17], v[16:17], 0, v[20:21]\n\tv_lshl_add_u64 v[18:19], v[18:19], 0, v[22:23]\n\t"
            "v_lshl_add_u64 v[20:21], v[20:21], 0, v[16:17]\n\tv_lshl_add_u64 v[22:23], v[22:23], 0, v[18:19]")
// 3-source: bitop3 with all sources in distinct banks vs all in one bank
BANK_KERNEL(bitop3_nc,
            "v_bitop3_b32 v0, v0, v9, v18 bitop3:0x96\n\tv_bitop3_b32 v1, v1, v10, v19 bitop3:0x96\n\t"
            "v_bitop3_b32 v2, v2, v11, v16 bitop3:0x96\n\tv_bitop3_b32 v3, v3, v8, v17 bitop3:0x96\n\t"
            "v_bitop3_b32 v4, v4, v13, v22 bitop3:0x96\n\tv_bitop3_b32 v5, v5, v14, v23 bitop3:0x96\n\t"
            "v_bitop3_b32 v6, v6, v15, v20 bitop3:0x96\n\tv_bitop3_b32 v7, v7, v12, v21 bitop3:0x96")
BANK_KERNEL(bitop3_c,
            "v_bitop3_b32 v0, v0, v8, v16 bitop3:0x96\n\tv_bitop3_b32 v1, v1, v9, v17 bitop3:0x96\n\t"
            "v_bitop3_b32 v2, v2, v10, v18 bitop3:0x96\n\tv_bitop3_b32 v3, v3, v11, v19 bitop3:0x96\n\t"
            "v_bitop3_b32 v4, v4, v12, v20 bitop3:0x96\n\tv_bitop3_b32 v5, v5, v13, v21 bitop3:0x96\n\t"
            "v_bitop3_b32 v6, v6, v14, v22 bitop3:0x96\n\tv_bitop3_b32 v7, v7, v15, v23 bitop3:0x96")

// placement census: per wave, HW_ID (simd/cu/se) and XCC id, plus s_memtime
// around an alignbit stream
template <int WG>
__global__ __launch_bounds__(WG) void k_census(uint32_t* info, uint64_t* cyc, int iters) {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  uint32_t a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 7 + i;
    b[i] = threadIdx.x ^ (i * 0x9e3779b9u);
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(a[i]) : "v"(b[i]));
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= a[i] ^ b[i];
  const uint32_t w = blockIdx.x * (WG / 64) + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) {
    info[2 * w] = hw;
    info[2 * w + 1] = xcc | (x & 0x80000000u);
    cyc[w] = t1 - t0;
  }
}

// compression-only with clock stamps (diagnostic build: the stamps go to a
// buffer of their own)
__global__ __launch_bounds__(256, 4) void k_compress_clk(uint8_t* out, uint32_t lines,
                                                         uint64_t* stamps) {
  using namespace cir::dev;
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint64_t h[8], m[16];
  init_state(h);
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = b * 0x9e3779b97f4a7c15ULL + k;
  for (uint32_t i = 0; i < lines; ++i) {
    m[i & 15] ^= i;
    compress(h, m, (uint64_t)(i + 1) * 128u, i + 1 == lines);
  }
  store_digest(out + b * 32, h);
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t1 - t0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
}

// ---- production-kernel A/B (same process, interleaved rounds) -------------
__global__ void k_fill(uint64_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (i + 1) * 0x9E3779B97F4A7C15ULL ^ (i >> 7);
}

// variant 0: production (uniform.hpp); 1: + stamps (clock); 2: static priority
// for the second half of each workgroup's waves
template <int V>
__global__ __launch_bounds__(256, 5) void k_prod(const uint8_t* __restrict__ data, uint64_t bs,
                                                 uint32_t lines, uint8_t* __restrict__ out,
                                                 uint64_t* stamps) {
  using namespace cir::dev;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWaves * kWaveLds];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t blk0 = ((uint64_t)blockIdx.x * kWaves + wave) * 64u;
  uint64_t t0 = 0, r0 = 0;
  if constexpr (V == 1) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (V == 2) {
    if (wave >= 2) __builtin_amdgcn_s_setprio(1);
  }
  uniform_glds_wave(data + blk0 * bs, bs, lines, out + blk0 * 32u, lds + wave * kWaveLds);
  if constexpr (V == 1) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
      stamps[2 * (blockIdx.x * kWaves + wave)] = t1 - t0;
      stamps[2 * (blockIdx.x * kWaves + wave) + 1] = r1 - r0;
    }
  }
}

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

// workgroup-size variants of the compression-only kernel
template <int WG>
__global__ __launch_bounds__(WG) void k_compress_wg(uint8_t* out, uint32_t lines) {
  using namespace cir::dev;
  const uint64_t b = (uint64_t)blockIdx.x * WG + threadIdx.x;
  uint64_t h[8], m[16];
  init_state(h);
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = b * 0x9e3779b97f4a7c15ULL + k;
  for (uint32_t i = 0; i < lines; ++i) {
    m[i & 15] ^= i;
    compress(h, m, (uint64_t)(i + 1) * 128u, i + 1 == lines);
  }
  store_digest(out + b * 32, h);
}

// same, occupancy limited by dynamic LDS (bytes chosen by the launcher)
__global__ __launch_bounds__(256, 1) void k_compress_occ(uint8_t* out, uint32_t lines) {
  extern __shared__ uint8_t dyn[];
  using namespace cir::dev;
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t h[8], m[16];
  init_state(h);
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = b * 0x9e3779b97f4a7c15ULL + k;
  if (lines == 0xffffffffu) dyn[threadIdx.x] = 1;  // keep the LDS allocation
  for (uint32_t i = 0; i < lines; ++i) {
    m[i & 15] ^= i;
    compress(h, m, (uint64_t)(i + 1) * 128u, i + 1 == lines);
  }
  store_digest(out + b * 32, h);
}

// two independent chains per lane (ILP 8): lane hashes blocks b and b + n/2
__global__ __launch_bounds__(256, 2) void k_compress_x2(uint8_t* out, uint32_t lines) {
  using namespace cir::dev;
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t h[8], g[8], m[16], q[16];
  init_state(h);
  init_state(g);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    m[k] = b * 0x9e3779b97f4a7c15ULL + k;
    q[k] = b * 0x94d049bb133111ebULL + k;
  }
  for (uint32_t i = 0; i < lines; ++i) {
    m[i & 15] ^= i;
    q[i & 15] ^= i;
    compress2(h, m, g, q, (uint64_t)(i + 1) * 128u, i + 1 == lines);
  }
  store_digest(out + b * 64, h);
  store_digest(out + b * 64 + 32, g);
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
  {
    struct {
      const char* name;
      OpKernel k;
    } bk[] = {{"alignbit distinct banks", k_bank_alignbit_nc}, {"alignbit same bank", k_bank_alignbit_c},
              {"xor distinct banks", k_bank_xor_nc}, {"xor same bank", k_bank_xor_c},
              {"lshl_add_u64 {0,1}+{2,3}", k_bank_lshladd_nc}, {"lshl_add_u64 {0,1}+{0,1}", k_bank_lshladd_c},
              {"bitop3 distinct banks", k_bank_bitop3_nc}, {"bitop3 same bank", k_bank_bitop3_c}};
    for (int wps : {2, 8}) {
      const int g = cus * wps;
      const double stm = (double)g * 256 * iters * 16 * 8;
      for (auto& q : bk) {
        const float t = time_kernel(q.k, d, g, iters);
        printf("bank %-28s waves/SIMD %d: %6.2f T lane-instr/s\n", q.name, wps,
               stm / (t * 1e-3) / 1e12);
      }
    }
  }
  {
    uint32_t* dinfo;
    uint64_t* dcyc;
    CHECK(hipMalloc(&dinfo, 65536 * 8));
    CHECK(hipMalloc(&dcyc, 65536 * 8));
    std::vector<uint32_t> info(65536 * 2);
    std::vector<uint64_t> cyc(65536);
    struct Cfg {
      const char* name;
      int wg, grid;
      void (*k)(uint32_t*, uint64_t*, int);
    } cf[] = {{"WG256 x 2/CU", 256, cus * 2, k_census<256>},
              {"WG512 x 1/CU", 512, cus, k_census<512>},
              {"WG256 x 8/CU", 256, cus * 8, k_census<256>}};
    for (auto& c : cf) {
      hipLaunchKernelGGL(c.k, dim3(c.grid), dim3(c.wg), 0, 0, dinfo, dcyc, iters);
      hipEvent_t a, b;
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(c.k, dim3(c.grid), dim3(c.wg), 0, 0, dinfo, dcyc, iters);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      const int nw = c.grid * c.wg / 64;
      CHECK(hipMemcpy(info.data(), dinfo, nw * 8, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(cyc.data(), dcyc, nw * 8, hipMemcpyDeviceToHost));
      std::map<uint64_t, int> per_simd;  // (xcc, se, sh, cu, simd) -> waves
      std::map<uint64_t, std::set<int>> simds_per_cu;
      double csum = 0;
      for (int w = 0; w < nw; ++w) {
        const uint32_t hw = info[2 * w], xcc = info[2 * w + 1] & 0xf;
        const uint32_t simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1,
                       se = (hw >> 13) & 7;
        const uint64_t cukey = ((uint64_t)xcc << 16) | (se << 8) | (sh << 4) | cu;
        per_simd[(cukey << 4) | simd]++;
        simds_per_cu[cukey].insert(simd);
        csum += (double)cyc[w];
      }
      int maxw = 0, minw = 1 << 30;
      size_t s1 = 0;
      for (auto& kv : per_simd) {
        maxw = std::max(maxw, kv.second);
        minw = std::min(minw, kv.second);
      }
      for (auto& kv : simds_per_cu) s1 += kv.second.size();
      const double instr = 16.0 * 8 * iters;
      printf("census %-14s %.3f ms: %zu CUs, %zu SIMDs (%.2f per CU), waves/SIMD %d..%d, "
             "avg wave cycles/instr %.2f (memtime)\n",
             c.name, ms, simds_per_cu.size(), per_simd.size(),
             (double)s1 / simds_per_cu.size(), minw, maxw, csum / nw / instr);
    }
  }
  {
    // every wave issues 16*8*iters instructions; 2 waves per SIMD, 1 WG per CU
    const int g = cus;
    struct {
      const char* name;
      OpKernel k;
    } pk[] = {{"A slow | B slow", k_pair<0, 0>}, {"A fast | B fast", k_pair<1, 1>},
              {"A slow | B fast", k_pair<0, 1>}, {"A alt  | B alt ", k_pair<2, 2>},
              {"A slow | B alt ", k_pair<0, 2>}, {"A fast | B alt ", k_pair<1, 2>}};
    for (auto& q : pk) {
      const float t = time_kernel(q.k, d, g, iters);
      // cycles per SIMD for the pair = t * clk; instructions per SIMD = 2 * 16*8*iters
      const double cyc = t * 1e-3 * 2.38e9;
      printf("pair %-16s %7.3f ms  %.2f cycles per instruction (2 waves/SIMD)\n", q.name, t,
             cyc / (2.0 * 16 * 8 * iters));
    }
  }
  // waves per SIMD sweep (grid = cus * wps WGs of 4 waves; 1 WG per CU per wave/SIMD)
  for (int wps = 1; wps <= 8; wps *= 2) {
    const int g = cus * wps;
    const double stm = (double)g * 256 * iters * 16 * 8;
    const float tx = time_kernel(kOps[0].k, d, g, iters);
    const float ta = time_kernel(kOps[2].k, d, g, iters);
    printf("waves/SIMD %d: xor %.2f T/s, alignbit %.2f T/s\n", wps, stm / (tx * 1e-3) / 1e12,
           stm / (ta * 1e-3) / 1e12);
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
  // occupancy sensitivity: LDS per workgroup limits workgroups (4 waves) per CU
  for (int wgs = 5; wgs >= 1; --wgs) {
    const size_t lds = 163840 / wgs - 64;
    (void)hipFuncSetAttribute((const void*)k_compress_occ,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k_compress_occ, dim3(nlanes / 256), dim3(256), lds, 0, dout, 256u);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_compress_occ, dim3(nlanes / 256), dim3(256), lds, 0, dout, 256u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("compress-only at <= %d waves/SIMD: %.3f ms (%s)\n", wgs, ms,
           hipGetErrorString(hipGetLastError()));
  }
  {
    struct {
      const char* name;
      int wg;
      CompKernel k;
    } wk[] = {{"64", 64, k_compress_wg<64>}, {"128", 128, k_compress_wg<128>},
              {"256", 256, k_compress_wg<256>}, {"512", 512, k_compress_wg<512>},
              {"1024", 1024, k_compress_wg<1024>}};
    for (auto& w : wk) {
      hipEvent_t a, b;
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      hipLaunchKernelGGL(w.k, dim3(nlanes / w.wg), dim3(w.wg), 0, 0, dout, 256u);
      float best = 1e9;
      for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(w.k, dim3(nlanes / w.wg), dim3(w.wg), 0, 0, dout, 256u);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      printf("compress-only, workgroup %s threads: %.3f ms (%s)\n", w.name, best,
             hipGetErrorString(hipGetLastError()));
    }
  }
  {
    uint8_t* d2;
    CHECK(hipMalloc(&d2, nlanes * 32));
    const float t = time_compress(k_compress_x2, d2, nlanes / 2);
    printf("compress-only, 2 chains per lane (ILP 8), same work: %.3f ms\n", t);
  }
  {
    uint64_t* dst;
    const int g = (int)(nlanes / 256);
    CHECK(hipMalloc(&dst, g * 16));
    std::vector<uint64_t> st(2 * g);
    // >= 2 s of back-to-back launches, then stamp the last one
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    int n = 0;
    for (; n < 200; ++n) hipLaunchKernelGGL(k_compress_clk, dim3(g), dim3(256), 0, 0, dout, 256u, dst);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    CHECK(hipMemcpy(st.data(), dst, g * 16, hipMemcpyDeviceToHost));
    std::vector<double> clk;
    for (int i = 0; i < g; ++i) clk.push_back((double)st[2 * i] / (double)st[2 * i + 1] * 0.1);
    std::sort(clk.begin(), clk.end());
    printf("compress-only clock after %d launches (%.1f ms each): median %.3f GHz (p10 %.3f, p90 %.3f)\n",
           n, ms / n, clk[g / 2], clk[g / 10], clk[9 * g / 10]);
  }
  {
    // 1 M x 32 KiB, interleaved rounds: production / priority variant / compress-only
    const uint64_t nb = 1 << 20, bs = 32768, bytes = nb * bs;
    uint8_t *data, *o2;
    uint64_t* st;
    CHECK(hipMalloc(&data, bytes));
    CHECK(hipMalloc(&o2, nb * 32));
    CHECK(hipMalloc(&st, nb / 64 * 16));
    hipLaunchKernelGGL(k_fill, dim3(65536), dim3(256), 0, 0, (uint64_t*)data, bytes / 8);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    auto tp = [&](int v) {
      (void)hipEventRecord(a);
      if (v == 0) hipLaunchKernelGGL(k_prod<0>, dim3(nb / 256), dim3(256), 0, 0, data, bs, 256u, o2, st);
      if (v == 1) hipLaunchKernelGGL(k_prod<1>, dim3(nb / 256), dim3(256), 0, 0, data, bs, 256u, o2, st);
      if (v == 2) hipLaunchKernelGGL(k_prod<2>, dim3(nb / 256), dim3(256), 0, 0, data, bs, 256u, o2, st);
      if (v == 3) hipLaunchKernelGGL(k_compress_wg<256>, dim3(nb / 256), dim3(256), 0, 0, o2, 256u);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      return ms;
    };
    const char* names[] = {"production k_uniform_glds", "production + stamps", "production + setprio(1) waves 2-3",
                           "compress-only (no memory)"};
    std::vector<float> t[4];
    for (int v = 0; v < 4; ++v) tp(v);
    for (int round = 0; round < 7; ++round)
      for (int v = 0; v < 4; ++v) t[v].push_back(tp(v));
    for (int v = 0; v < 4; ++v) {
      std::sort(t[v].begin(), t[v].end());
      printf("AB %-36s median %.3f ms  min %.3f ms\n", names[v], t[v][3], t[v][0]);
    }
    std::vector<uint64_t> hs(nb / 64 * 2);
    CHECK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> clk;
    for (size_t i = 0; i < nb / 64; ++i) clk.push_back((double)hs[2 * i] / (double)hs[2 * i + 1] * 0.1);
    std::sort(clk.begin(), clk.end());
    printf("AB production kernel in-kernel clock: median %.3f GHz (p10 %.3f p90 %.3f)\n",
           clk[clk.size() / 2], clk[clk.size() / 10], clk[9 * clk.size() / 10]);
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
