// Streaming SHA-512/256 on one host thread, for the index footer only:
// the sha512/256 twin of blake2b_host.hpp (dir-signature's second hash type,
// FIPS 180-4; the reference's own fixture index uses it,
// src/cluster/download.rs:357-366).  A footer is one serial chain over the
// index text; every BLOCK digest is still computed by the gfx950 kernels.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace cir {
namespace host {

class Sha512_256 {
 public:
  Sha512_256();
  void update(const uint8_t* p, size_t n);
  void final(uint8_t out[32]);  // once

 private:
  void compress(const uint8_t* block);
  uint64_t h_[8];
  uint64_t len_ = 0;  // bytes fed (the index stays below 2^61)
  uint8_t buf_[128];
  size_t buflen_ = 0;
};

}  // namespace host
}  // namespace cir
