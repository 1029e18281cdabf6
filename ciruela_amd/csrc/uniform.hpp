// The hot loop of the block-hash path: one wave hashes 64 equal blocks with
// message lines streamed HBM -> LDS by LDS-DMA.  Shared by kernels.hip and
// the micro-benchmark (tools/valu_ubench.hip).
#pragma once
#include "blake2b_dev.hpp"
#include "kernels.hpp"

namespace cir {
namespace dev {

constexpr int kWaves = kThreads / 64;

// cache-policy bits of the LDS-DMA loads: 2 = nt (streamed, read once;
// MI355X_MICROARCH.md nt-weights).  A/B in-process: within 1 % of 0
// (profiles/r01/ablib_nt_occ.log).
constexpr int kDmaAux = 2;

// ---------------------------------------------------------------------------
// LDS image of one wave's message lines (8 KiB, no padding).
// DMA instruction j (0..7) fills bytes [1024 j, 1024 j + 1024): lane l
// fetches 16 bytes of block 8j + (l >> 3), chunk (l & 7) ^ (l >> 3) ^ j.
// So chunk c of wave-block b = 8j + r lives at 1024 j + 128 r + 16 (c^r^j)
// = 128 b + 16 (c ^ s_b) with s_b = (b ^ (b >> 3)) & 7.
//   * every DMA instruction reads 8 whole 128-byte lines (coalesced);
//   * ds_read_b128 of chunk c by lanes b = 0..63 hits 16 distinct bank quads
//     in every 16-lane group of the b128 read (checked in DESIGN.md), so the
//     transpose back to one-line-per-lane is conflict free.
// ---------------------------------------------------------------------------
constexpr int kWaveLds = 8192;

// One wave hashes the 64 equal blocks starting at wsrc (bs bytes each,
// `lines` = bs / 128 message lines) into out[0 .. 64*32).
// Register budget: k_chunks runs it at 4 waves per SIMD (107 VGPRs, no spills).
// The per-lane DMA offsets and LDS read addresses are recomputed every line
// from one register each (one full-rate v_xor_b32 apiece) instead of being
// hoisted into 16 + 8 registers; the DMA base address stays scalar.
//
// kPartial: the wave's last block is wsrc block nv - 1 (nv < 64, the file's
// last whole blocks): the DMA rows of blocks >= nv re-read block nv - 1 (in
// bounds; their lanes hash a duplicate) and only lanes < nv store.  A file
// whose whole-block count is not a multiple of 64 then still hashes every
// whole block through the prefetching LDS-DMA body instead of the slower
// general loader.
template <bool kPartial = false>
__device__ __forceinline__ void uniform_glds_wave(const uint8_t* __restrict__ wsrc, uint64_t bs,
                                                  uint32_t lines, uint8_t* __restrict__ out,
                                                  uint8_t* wl, uint32_t nv = 64) {
  const uint32_t lane = threadIdx.x & 63u;
  // DMA lane offset: r*bs + 16*chunk, chunk = (l & 7) ^ r ^ j
  const uint32_t r = lane >> 3;
  uint32_t dma_lane = (uint32_t)(r * bs) + 16u * ((lane & 7u) ^ r);
  // LDS read address of chunk c: rd_base ^ 16c
  const uint32_t s = (lane ^ (lane >> 3)) & 7u;
  uint32_t rd_base = lane * 128u + 16u * s;
  const uint64_t jstride = 8u * bs;

  auto issue = [&](uint32_t i) {
    const uint8_t* line = wsrc + (uint64_t)i * 128u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint8_t* src;
      if constexpr (kPartial) {
        const uint32_t blk = min(8u * j + r, nv - 1u);
        src = line + (uint64_t)blk * bs + ((16u * ((lane & 7u) ^ r)) ^ (16u * j));
      } else {
        src = line + (uint64_t)j * jstride + (dma_lane ^ (16u * j));
      }
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)src,
          (void __attribute__((address_space(3)))*)(wl + j * 1024), 16, 0, kDmaAux);
    }
  };

  uint64_t h[8];
  init_state(h);
  uint64_t m[16];
  issue(0);
  for (uint32_t i = 0; i < lines; ++i) {
    // opaque per iteration: keeps the derived addresses out of registers
    asm volatile("" : "+v"(rd_base), "+v"(dma_lane));
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): line i landed in LDS
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint4 x = *reinterpret_cast<const uint4*>(wl + (rd_base ^ (16u * c)));
      m[2 * c] = mk64(x.x, x.y);
      m[2 * c + 1] = mk64(x.z, x.w);
    }
    const bool last = i + 1 == lines;
    // The next line's DMA goes out after round 0's column step, which needs
    // only chunks 0-3: chunks 4-7 land under it instead of the wave waiting
    // for all eight reads (round 3: config 2 -1.2 to -1.4 % per launch,
    // in-process A/B on two boxes, profiles/r03_s2/ab_overlap.log).
    compress_sm(h, m, (uint64_t)(i + 1) * 128u, last, [&] {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): reads done before the refill
      if (i + 1 < lines) issue(i + 1);
    });
  }
  if (!kPartial || lane < nv) store_digest(out + lane * 32u, h);
}

}  // namespace dev
}  // namespace cir
