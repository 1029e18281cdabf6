// Streaming BLAKE2b-256 on one host thread, for the index footer only.
//
// The footer (ImageId) is H(every byte of the index after its header line):
// dir_signature::get_hash as read back by InMemoryIndexes::register_index
// (src/index.rs:98-105) -> ImageId (src/id.rs:186-196).  It is ONE serial
// chain over ~65 bytes of index text per 32 KiB block (106 MB for the 50 GiB
// tree of config 5), so it has no parallelism for the GPU to use: a lone
// wave's chain runs ~1.2 us per 128-B compression (quad mode, issue-latency
// bound), a host core ~0.1 us.  Every BLOCK digest is still computed by the
// gfx950 kernels; this type is never used for a block.
//
// RFC 7693 BLAKE2b with nn = 32, no key (the parameter block p0 =
// 0x01010000 ^ 32), fed incrementally: the last (possibly partial) 128-B
// block is held back until final(), which compresses it with the final flag.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace cir {
namespace host {

class Blake2b256 {
 public:
  Blake2b256();
  void update(const uint8_t* p, size_t n);
  void final(uint8_t out[32]);  // once; the state is spent afterwards

 private:
  void compress(const uint8_t* block, bool last);
  uint64_t h_[8];
  uint64_t t_ = 0;  // bytes compressed so far (the index stays below 2^64)
  uint8_t buf_[128];
  size_t buflen_ = 0;
};

}  // namespace host
}  // namespace cir
