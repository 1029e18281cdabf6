// Instruction-order micro-benchmark for the lane-per-chain compression
// (diagnostics, not part of the product).  Same 1 M lanes x 256
// compressions on register messages as valu_ubench's compress-only, with the
// rounds written step-major (one G step over the 4 independent columns or
// diagonals at a time) and optional scheduling barriers that keep the slow
// VALU class (64-bit adds, funnel shifts) and the fast class (v_xor_b32)
// in contiguous groups.  Every variant's digests are compared with the
// production compress() on the device.
//
//   hipcc -O3 --offload-arch=gfx950 -I ciruela_amd/csrc tools/order_ubench.hip -o build/order_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "blake2b_dev.hpp"

using namespace cir::dev;

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

// MODE bits: 1 = sched_barrier between steps; 2 = rotl1 as shl-add + lshr;
//            4 = barriers only between class changes (merge adjacent groups)
template <int MODE>
__device__ __forceinline__ void sb() {
  if constexpr ((MODE & 1) != 0) __builtin_amdgcn_sched_barrier(0);
}

template <int N, int MODE>
__device__ __forceinline__ uint64_t rotr_split(uint32_t l, uint32_t h) {
  if constexpr (N == 32) {
    return mk64(h, l);
  } else if constexpr (N == 63 && (MODE & 2) != 0) {
    const uint64_t x = mk64(l, h);
    return (x << 1) + (uint64_t)(h >> 31);
  } else if constexpr (N < 32) {
    return mk64(__builtin_amdgcn_alignbit(h, l, N), __builtin_amdgcn_alignbit(l, h, N));
  } else {
    return mk64(__builtin_amdgcn_alignbit(l, h, N - 32), __builtin_amdgcn_alignbit(h, l, N - 32));
  }
}

// 4 independent G on (A[k], B[k], C[k], D[k]) with messages X[k], Y[k]
template <int MODE>
__device__ __forceinline__ void g4(uint64_t& a0, uint64_t& a1, uint64_t& a2, uint64_t& a3,
                                   uint64_t& b0, uint64_t& b1, uint64_t& b2, uint64_t& b3,
                                   uint64_t& c0, uint64_t& c1, uint64_t& c2, uint64_t& c3,
                                   uint64_t& d0, uint64_t& d1, uint64_t& d2, uint64_t& d3,
                                   uint64_t x0, uint64_t x1, uint64_t x2, uint64_t x3,
                                   uint64_t y0, uint64_t y1, uint64_t y2, uint64_t y3) {
  uint32_t tl0, tl1, tl2, tl3, th0, th1, th2, th3;
#define XOR4(P, Q)                                   \
  tl0 = lo32(P##0) ^ lo32(Q##0); th0 = hi32(P##0) ^ hi32(Q##0); \
  tl1 = lo32(P##1) ^ lo32(Q##1); th1 = hi32(P##1) ^ hi32(Q##1); \
  tl2 = lo32(P##2) ^ lo32(Q##2); th2 = hi32(P##2) ^ hi32(Q##2); \
  tl3 = lo32(P##3) ^ lo32(Q##3); th3 = hi32(P##3) ^ hi32(Q##3);
#define ROT4(P, N)                          \
  P##0 = rotr_split<N, MODE>(tl0, th0);     \
  P##1 = rotr_split<N, MODE>(tl1, th1);     \
  P##2 = rotr_split<N, MODE>(tl2, th2);     \
  P##3 = rotr_split<N, MODE>(tl3, th3);
  // S1: a += x; a += b  (slow)
  a0 = a0 + x0; a1 = a1 + x1; a2 = a2 + x2; a3 = a3 + x3;
  a0 = a0 + b0; a1 = a1 + b1; a2 = a2 + b2; a3 = a3 + b3;
  sb<MODE>();
  // S2: d = rotr32(d ^ a)  (fast)
  XOR4(d, a)
  ROT4(d, 32)
  sb<MODE>();
  // S3: c += d  (slow)
  c0 = c0 + d0; c1 = c1 + d1; c2 = c2 + d2; c3 = c3 + d3;
  sb<MODE>();
  // S4: b = rotr24(b ^ c)
  XOR4(b, c)
  sb<MODE>();
  ROT4(b, 24)
  if constexpr ((MODE & 4) == 0) sb<MODE>();
  // S5
  a0 = a0 + y0; a1 = a1 + y1; a2 = a2 + y2; a3 = a3 + y3;
  a0 = a0 + b0; a1 = a1 + b1; a2 = a2 + b2; a3 = a3 + b3;
  sb<MODE>();
  // S6
  XOR4(d, a)
  sb<MODE>();
  ROT4(d, 16)
  if constexpr ((MODE & 4) == 0) sb<MODE>();
  // S7
  c0 = c0 + d0; c1 = c1 + d1; c2 = c2 + d2; c3 = c3 + d3;
  sb<MODE>();
  // S8
  XOR4(b, c)
  sb<MODE>();
  ROT4(b, 63)
  if constexpr ((MODE & 4) == 0) sb<MODE>();
#undef XOR4
#undef ROT4
}

#define OROUND(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15)             \
  g4<MODE>(v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v15, m[s0], m[s2],   \
           m[s4], m[s6], m[s1], m[s3], m[s5], m[s7]);                                           \
  g4<MODE>(v0, v1, v2, v3, v5, v6, v7, v4, v10, v11, v8, v9, v15, v12, v13, v14, m[s8], m[s10],  \
           m[s12], m[s14], m[s9], m[s11], m[s13], m[s15]);

template <int MODE>
__device__ __forceinline__ void compress_o(uint64_t h[8], const uint64_t m[16], uint64_t t,
                                           bool last) {
  uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3];
  uint64_t v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint64_t v8 = CIR_IV0, v9 = CIR_IV1, v10 = CIR_IV2, v11 = CIR_IV3;
  uint64_t v12 = CIR_IV4 ^ t, v13 = CIR_IV5;
  uint64_t v14 = last ? ~CIR_IV6 : CIR_IV6, v15 = CIR_IV7;
  OROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  OROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  OROUND(11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4)
  OROUND(7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8)
  OROUND(9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13)
  OROUND(2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9)
  OROUND(12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11)
  OROUND(13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10)
  OROUND(6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5)
  OROUND(10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0)
  OROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  OROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  h[0] = xor3(h[0], v0, v8);
  h[1] = xor3(h[1], v1, v9);
  h[2] = xor3(h[2], v2, v10);
  h[3] = xor3(h[3], v3, v11);
  h[4] = xor3(h[4], v4, v12);
  h[5] = xor3(h[5], v5, v13);
  h[6] = xor3(h[6], v6, v14);
  h[7] = xor3(h[7], v7, v15);
}

// Two chains per lane, step-major with class barriers: each group is 8 (or
// 16) independent instructions of one class per chain pair.
__device__ __forceinline__ void g4x2(uint64_t* v, uint64_t* w, const uint64_t* m, const uint64_t* q,
                                     const int* A, const int* B, const int* C, const int* D,
                                     const int* X, const int* Y) {
  uint32_t tl[8], th[8];
  uint64_t* V[8] = {v, v, v, v, w, w, w, w};
  (void)V;
#define EACH(body) _Pragma("unroll") for (int k = 0; k < 4; ++k) { body(v, m, k, 0) body(w, q, k, 4) }
#define S_AX(S, M, k, o) S[A[k]] = S[A[k]] + M[X[k]];
#define S_AB(S, M, k, o) S[A[k]] = S[A[k]] + S[B[k]];
#define S_AY(S, M, k, o) S[A[k]] = S[A[k]] + M[Y[k]];
#define S_CD(S, M, k, o) S[C[k]] = S[C[k]] + S[D[k]];
#define S_XDA(S, M, k, o) tl[k + o] = lo32(S[D[k]]) ^ lo32(S[A[k]]); th[k + o] = hi32(S[D[k]]) ^ hi32(S[A[k]]);
#define S_XBC(S, M, k, o) tl[k + o] = lo32(S[B[k]]) ^ lo32(S[C[k]]); th[k + o] = hi32(S[B[k]]) ^ hi32(S[C[k]]);
#define S_RD32(S, M, k, o) S[D[k]] = rotr_lh<32>(tl[k + o], th[k + o]);
#define S_RD16(S, M, k, o) S[D[k]] = rotr_lh<16>(tl[k + o], th[k + o]);
#define S_RB24(S, M, k, o) S[B[k]] = rotr_lh<24>(tl[k + o], th[k + o]);
#define S_RB63(S, M, k, o) S[B[k]] = rotr_lh<63>(tl[k + o], th[k + o]);
  EACH(S_AX) EACH(S_AB) sched_fence();
  EACH(S_XDA) EACH(S_RD32) sched_fence();
  EACH(S_CD) sched_fence();
  EACH(S_XBC) sched_fence();
  EACH(S_RB24) EACH(S_AY) EACH(S_AB) sched_fence();
  EACH(S_XDA) sched_fence();
  EACH(S_RD16) EACH(S_CD) sched_fence();
  EACH(S_XBC) sched_fence();
  EACH(S_RB63)
}

__device__ __forceinline__ void compress_x2(uint64_t h[8], const uint64_t m[16], uint64_t g[8],
                                            const uint64_t q[16], uint64_t t, bool last) {
  uint64_t v[16], w[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) { v[k] = h[k]; w[k] = g[k]; }
  v[8] = w[8] = CIR_IV0; v[9] = w[9] = CIR_IV1; v[10] = w[10] = CIR_IV2; v[11] = w[11] = CIR_IV3;
  v[12] = w[12] = CIR_IV4 ^ t; v[13] = w[13] = CIR_IV5;
  v[14] = w[14] = last ? ~CIR_IV6 : CIR_IV6; v[15] = w[15] = CIR_IV7;
  constexpr int kS[12][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
      {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
      {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
      {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
      {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
      {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
      {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
      {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
      {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
  constexpr int Ac[4] = {0, 1, 2, 3}, Bc[4] = {4, 5, 6, 7}, Cc[4] = {8, 9, 10, 11}, Dc[4] = {12, 13, 14, 15};
  constexpr int Bd[4] = {5, 6, 7, 4}, Cd[4] = {10, 11, 8, 9}, Dd[4] = {15, 12, 13, 14};
#pragma unroll
  for (int r = 0; r < 12; ++r) {
    const int X0[4] = {kS[r][0], kS[r][2], kS[r][4], kS[r][6]};
    const int Y0[4] = {kS[r][1], kS[r][3], kS[r][5], kS[r][7]};
    const int X1[4] = {kS[r][8], kS[r][10], kS[r][12], kS[r][14]};
    const int Y1[4] = {kS[r][9], kS[r][11], kS[r][13], kS[r][15]};
    g4x2(v, w, m, q, Ac, Bc, Cc, Dc, X0, Y0);
    g4x2(v, w, m, q, Ac, Bd, Cd, Dd, X1, Y1);
  }
  sched_fence();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    h[k] = xor3(h[k], v[k], v[k + 8]);
    g[k] = xor3(g[k], w[k], w[k + 8]);
  }
}

template <int OCC>
__global__ __launch_bounds__(256, OCC) void k_comp_x2(uint8_t* out, uint32_t lines) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;  // lanes = nlanes / 2
  const uint64_t b0 = 2 * b, b1 = 2 * b + 1;
  uint64_t h[8], g[8], m[16], q[16];
  init_state(h);
  init_state(g);
#pragma unroll
  for (int k = 0; k < 16; ++k) { m[k] = b0 * 0x9e3779b97f4a7c15ULL + k; q[k] = b1 * 0x9e3779b97f4a7c15ULL + k; }
  for (uint32_t i = 0; i < lines; ++i) {
    m[0] ^= i;
    q[0] ^= i;
    compress_x2(h, m, g, q, (uint64_t)(i + 1) * 128u, i + 1 == lines);
  }
  store_digest(out + b0 * 32u, h);
  store_digest(out + b1 * 32u, g);
}

template <int OCC>
__global__ __launch_bounds__(256, OCC) void k_comp_sm(uint8_t* out, uint32_t lines) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t h[8], m[16];
  init_state(h);
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = b * 0x9e3779b97f4a7c15ULL + k;
  for (uint32_t i = 0; i < lines; ++i) {
    m[0] ^= i;
    compress_sm(h, m, (uint64_t)(i + 1) * 128u, i + 1 == lines);
  }
  store_digest(out + b * 32u, h);
}

// Instruction-fetch probe: the same instruction mix with the 12 rounds rolled
// into a loop (every round uses sigma_0, so the digests differ from BLAKE2b):
// a ~1.3 KiB loop body instead of ~13 KiB of straight-line code.
__device__ __forceinline__ void compress_rolled(uint64_t h[8], const uint64_t m[16], uint64_t t,
                                                bool last) {
  uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3];
  uint64_t v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint64_t v8 = CIR_IV0, v9 = CIR_IV1, v10 = CIR_IV2, v11 = CIR_IV3;
  uint64_t v12 = CIR_IV4 ^ t, v13 = CIR_IV5;
  uint64_t v14 = last ? ~CIR_IV6 : CIR_IV6, v15 = CIR_IV7;
#pragma unroll 1
  for (int r = 0; r < 12; ++r) {
    CIR_ROUND_SM(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  }
  sched_fence();
  h[0] = xor3(h[0], v0, v8);
  h[1] = xor3(h[1], v1, v9);
  h[2] = xor3(h[2], v2, v10);
  h[3] = xor3(h[3], v3, v11);
  h[4] = xor3(h[4], v4, v12);
  h[5] = xor3(h[5], v5, v13);
  h[6] = xor3(h[6], v6, v14);
  h[7] = xor3(h[7], v7, v15);
}

__global__ __launch_bounds__(256, 4) void k_comp_rolled(uint8_t* out, uint32_t lines) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t h[8], m[16];
  init_state(h);
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = b * 0x9e3779b97f4a7c15ULL + k;
  for (uint32_t i = 0; i < lines; ++i) {
    m[0] ^= i;
    compress_rolled(h, m, (uint64_t)(i + 1) * 128u, i + 1 == lines);
  }
  store_digest(out + b * 32u, h);
}

// same, unrolled (same wrong sigma): isolates the code-size effect
__device__ __forceinline__ void compress_unrolled_s0(uint64_t h[8], const uint64_t m[16], uint64_t t,
                                                     bool last) {
  uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3];
  uint64_t v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint64_t v8 = CIR_IV0, v9 = CIR_IV1, v10 = CIR_IV2, v11 = CIR_IV3;
  uint64_t v12 = CIR_IV4 ^ t, v13 = CIR_IV5;
  uint64_t v14 = last ? ~CIR_IV6 : CIR_IV6, v15 = CIR_IV7;
#pragma unroll
  for (int r = 0; r < 12; ++r) {
    CIR_ROUND_SM(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  }
  sched_fence();
  h[0] = xor3(h[0], v0, v8);
  h[1] = xor3(h[1], v1, v9);
  h[2] = xor3(h[2], v2, v10);
  h[3] = xor3(h[3], v3, v11);
  h[4] = xor3(h[4], v4, v12);
  h[5] = xor3(h[5], v5, v13);
  h[6] = xor3(h[6], v6, v14);
  h[7] = xor3(h[7], v7, v15);
}

__global__ __launch_bounds__(256, 4) void k_comp_unrolled_s0(uint8_t* out, uint32_t lines) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t h[8], m[16];
  init_state(h);
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = b * 0x9e3779b97f4a7c15ULL + k;
  for (uint32_t i = 0; i < lines; ++i) {
    m[0] ^= i;
    compress_unrolled_s0(h, m, (uint64_t)(i + 1) * 128u, i + 1 == lines);
  }
  store_digest(out + b * 32u, h);
}

// MODE < 0: production compress()
template <int MODE>
__global__ __launch_bounds__(256, 4) void k_comp(uint8_t* out, uint32_t lines) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t h[8], m[16];
  init_state(h);
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = b * 0x9e3779b97f4a7c15ULL + k;
  for (uint32_t i = 0; i < lines; ++i) {
    m[0] ^= i;
    if constexpr (MODE < 0)
      compress(h, m, (uint64_t)(i + 1) * 128u, i + 1 == lines);
    else
      compress_o<MODE>(h, m, (uint64_t)(i + 1) * 128u, i + 1 == lines);
  }
  store_digest(out + b * 32u, h);
}

typedef void (*CompKernel)(uint8_t*, uint32_t);

static float time_comp(CompKernel k, uint8_t* dout, uint64_t nlanes, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(nlanes / 256), dim3(256), 0, 0, dout, 256u);
  float best = 1e9;
  for (int rep = 0; rep < reps; ++rep) {
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
  const uint64_t nlanes = 1 << 20;
  uint8_t *dref, *dout;
  CHECK(hipMalloc(&dref, nlanes * 32));
  CHECK(hipMalloc(&dout, nlanes * 32));
  static uint8_t href[(1 << 20) * 32], hout[(1 << 20) * 32];
  struct {
    const char* name;
    CompKernel k;
  } ks[] = {
      {"production compress()", k_comp<-1>},
      {"step-major, compiler scheduled", k_comp<0>},
      {"step-major, barrier every step", k_comp<1>},
      {"step-major, barriers at class changes", k_comp<5>},
      {"step-major, barrier every step, shl-add 63", k_comp<3>},
      {"step-major, class barriers, shl-add 63", k_comp<7>},
      {"step-major, compiler scheduled, shl-add 63", k_comp<2>},
      {"header compress_sm, occupancy >= 5", k_comp_sm<5>},
      {"header compress_sm, occupancy >= 4", k_comp_sm<4>},
      {"header compress_sm, occupancy >= 2", k_comp_sm<2>},
  };
  struct {
    const char* name;
    CompKernel k;
  } k2[] = {
      {"2 chains/lane step-major, occupancy >= 2", k_comp_x2<2>},
  };
  hipLaunchKernelGGL(k_comp<-1>, dim3(nlanes / 256), dim3(256), 0, 0, dref, 256u);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(href, dref, nlanes * 32, hipMemcpyDeviceToHost));
  for (int pass = 0; pass < 2; ++pass) {
    for (auto& k : ks) {
      const float t = time_comp(k.k, dout, nlanes, 5);
      CHECK(hipMemcpy(hout, dout, nlanes * 32, hipMemcpyDeviceToHost));
      const bool ok = memcmp(hout, href, nlanes * 32) == 0;
      printf("pass %d %-45s %8.3f ms  %7.1f GB/s-equivalent  %s\n", pass, k.name, t,
             (double)nlanes * 32768 / (t * 1e-3) / 1e9, ok ? "digests ok" : "DIGEST MISMATCH");
    }
  }
  {
    struct {
      const char* name;
      CompKernel k;
    } kf[] = {{"fetch probe: rounds unrolled, sigma_0 everywhere", k_comp_unrolled_s0},
              {"fetch probe: rounds rolled (1-round loop body)", k_comp_rolled}};
    for (int pass = 0; pass < 2; ++pass)
      for (auto& k : kf) {
        const float t = time_comp(k.k, dout, nlanes, 5);
        printf("%-52s %8.3f ms  (digests are not BLAKE2b)\n", k.name, t);
      }
  }
  for (auto& k : k2) {
    hipLaunchKernelGGL(k.k, dim3(nlanes / 512), dim3(256), 0, 0, dout, 256u);
    CHECK(hipDeviceSynchronize());
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      hipEvent_t a, b;
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(k.k, dim3(nlanes / 512), dim3(256), 0, 0, dout, 256u);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    CHECK(hipMemcpy(hout, dout, nlanes * 32, hipMemcpyDeviceToHost));
    const bool ok = memcmp(hout, href, nlanes * 32) == 0;
    printf("%-52s %8.3f ms  %7.1f GB/s-equivalent  %s\n", k.name, best,
           (double)nlanes * 32768 / (best * 1e-3) / 1e9, ok ? "digests ok" : "DIGEST MISMATCH");
  }
  return 0;
}
