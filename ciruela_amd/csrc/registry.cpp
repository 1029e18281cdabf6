// Host mirrors of the two consumers of the index:
//   InMemoryIndexes   (src/index.rs:53-124)  : ImageId -> index bytes
//   ThreadedBlockReader (src/blocks.rs:85-240): BlockHash -> block pointer
// Plain host bookkeeping (O(#blocks)); the hashing they need goes through the
// GPU entry points (cir_hash_memory).
#include <fcntl.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <memory>
#include <new>
#include <shared_mutex>
#include <unordered_map>

#include "dirsig.hpp"
#include "runtime.hpp"

namespace cir {

struct Key32 {
  uint8_t b[32];
  bool operator==(const Key32& o) const { return memcmp(b, o.b, 32) == 0; }
};
struct Key32Hash {
  size_t operator()(const Key32& k) const {
    size_t h;
    memcpy(&h, k.b, sizeof h);
    return h;
  }
};

struct IndexMap {
  std::shared_mutex mu;
  std::unordered_map<std::string, std::shared_ptr<std::string>> by_id;  // raw id bytes
};

// BlockPointer::{Disk, Mem} (src/blocks.rs:61-72)
struct BlockPtr {
  std::shared_ptr<std::string> path;             // Disk
  std::shared_ptr<std::vector<uint8_t>> data;    // Mem
  uint64_t offset = 0;
  uint64_t size = 0;
};

struct BlockMap {
  std::shared_mutex mu;
  std::unordered_map<Key32, BlockPtr, Key32Hash> blocks;
};

}  // namespace cir

using namespace cir;

extern "C" {


cir_indexes* cir_indexes_new(void) {
  return reinterpret_cast<cir_indexes*>(new (std::nothrow) IndexMap());  // NULL: no memory
}
void cir_indexes_free(cir_indexes* h) { delete reinterpret_cast<IndexMap*>(h); }

// InMemoryIndexes::register_index (src/index.rs:98-105)
int cir_indexes_register(cir_indexes* h, const uint8_t* data, size_t len, uint8_t* id_out,
                         size_t* id_len) try {
  if (!h || !data || !id_out || !id_len) return fail(CIR_EINVAL, "null pointer");
  std::vector<uint8_t> id;
  std::string err;
  if (!dirsig::get_hash(data, len, &id, &err)) return fail(CIR_EPARSE, "error parsing index");
  if (id.size() > 64) return fail(CIR_EPARSE, "error parsing index");
  auto* m = reinterpret_cast<IndexMap*>(h);
  {
    std::unique_lock<std::shared_mutex> lk(m->mu);
    m->by_id[std::string((const char*)id.data(), id.size())] =
        std::make_shared<std::string>((const char*)data, len);
  }
  memcpy(id_out, id.data(), id.size());
  *id_len = id.size();
  return CIR_OK;
} CIR_CATCH_BOUNDARY

// GetIndex::read_index (src/index.rs:106-123)
int cir_indexes_read(cir_indexes* h, const uint8_t* id, size_t id_len, uint8_t** data_out,
                     size_t* len_out) try {
  if (!h || !id || !data_out || !len_out) return fail(CIR_EINVAL, "null pointer");
  auto* m = reinterpret_cast<IndexMap*>(h);
  std::shared_ptr<std::string> v;
  {
    std::shared_lock<std::shared_mutex> lk(m->mu);
    auto it = m->by_id.find(std::string((const char*)id, id_len));
    if (it == m->by_id.end())
      return fail(CIR_ENOTFOUND, "index " + dirsig::to_hex(id, id_len) + " with not found");
    v = it->second;
  }
  *data_out = (uint8_t*)malloc(std::max<size_t>(v->size(), 1));
  if (!*data_out) return fail(CIR_ENOMEM, "malloc");
  memcpy(*data_out, v->data(), v->size());
  *len_out = v->size();
  return CIR_OK;
} CIR_CATCH_BOUNDARY

cir_blocks* cir_blocks_new(void) {
  return reinterpret_cast<cir_blocks*>(new (std::nothrow) BlockMap());  // NULL: no memory
}
void cir_blocks_free(cir_blocks* h) { delete reinterpret_cast<BlockMap*>(h); }

size_t cir_blocks_len(cir_blocks* h) {
  auto* m = reinterpret_cast<BlockMap*>(h);
  std::shared_lock<std::shared_mutex> lk(m->mu);
  return m->blocks.size();
}

// ThreadedBlockReader::register_dir (src/blocks.rs:145-183): every block of
// every file in the index -> Disk{dir + path, idx * bs, min(left, bs)}.
int cir_blocks_register_dir(cir_blocks* h, const char* dir, const uint8_t* index, size_t len) try {
  if (!h || !dir || !index) return fail(CIR_EINVAL, "null pointer");
  dirsig::Index idx;
  std::string err;
  if (!dirsig::parse(index, len, &idx, &err))
    return idx.bad_hash_size ? fail(CIR_EHASHSIZE, "hash size is unsupported: " + err)
                             : fail(CIR_EPARSE, "error parsing index: " + err);
  const uint64_t bs = idx.header.block_size;
  const size_t dl = dirsig::digest_len(idx.header.hash);
  if (dl != 32) return fail(CIR_EHASHSIZE, "hash size is unsupported");
  auto* m = reinterpret_cast<BlockMap*>(h);
  std::unique_lock<std::shared_mutex> lk(m->mu);
  std::string base = dir;
  while (base.size() > 1 && base.back() == '/') base.pop_back();
  for (const dirsig::Entry& e : idx.entries) {
    if (e.kind != dirsig::EntryKind::kFile) continue;
    auto path = std::make_shared<std::string>(base + e.path);  // e.path starts with '/'
    uint64_t left = e.size;
    const size_t n = e.hashes.size() / dl;
    for (size_t i = 0; i < n; ++i) {
      Key32 k;
      memcpy(k.b, e.hashes.data() + i * dl, 32);
      BlockPtr p;
      p.path = path;
      p.offset = (uint64_t)i * bs;
      p.size = std::min(left, bs);
      m->blocks[k] = p;
      left = left > bs ? left - bs : 0;
    }
  }
  return CIR_OK;
} CIR_CATCH_BOUNDARY

// ThreadedBlockReader::register_memory_blocks (src/blocks.rs:187-204): hash
// `data` in block_size blocks (on the GPU) and serve them from memory.
// Quirk of the reference, deliberately not reproduced: it records
// size = min(len, (idx+1)*bs), an end offset used as a length (:201), so its
// reads of blocks 1.. over-read or panic.  Here block idx covers exactly the
// bytes its hash was computed over: [idx*bs, min(len, (idx+1)*bs)).
// The hash type is the index's (put-file passes it through,
// src/client/put_file/network.rs:56): every block id is
// Hashes::hash_file(hash_type, ..)'s digest of the block.
int cir_blocks_register_memory_ht(cir_ctx* ctx, cir_blocks* h, int hash_type, const uint8_t* data,
                                  size_t len, uint64_t block_size) try {
  if (!ctx || !h || (len && !data)) return fail(CIR_EINVAL, "null pointer");
  if (!valid_hash_type(hash_type)) return fail(CIR_EINVAL, "unknown hash type");
  uint8_t* hashes = nullptr;
  size_t n = 0;
  int rc = cir_hash_memory_ht(ctx, hash_type, data, len, block_size, &hashes, &n);
  if (rc) return rc;
  auto buf = std::make_shared<std::vector<uint8_t>>(data, data + len);
  auto* m = reinterpret_cast<BlockMap*>(h);
  std::unique_lock<std::shared_mutex> lk(m->mu);
  for (size_t i = 0; i < n; ++i) {
    Key32 k;
    memcpy(k.b, hashes + 32 * i, 32);
    BlockPtr p;
    p.data = buf;
    p.offset = (uint64_t)i * block_size;
    p.size = std::min<uint64_t>(block_size, len - p.offset);
    m->blocks[k] = p;
  }
  free(hashes);
  return CIR_OK;
} CIR_CATCH_BOUNDARY

int cir_blocks_register_memory(cir_ctx* ctx, cir_blocks* h, const uint8_t* data, size_t len,
                               uint64_t block_size) try {
  return cir_blocks_register_memory_ht(ctx, h, CIR_HASH_BLAKE2B_256, data, len, block_size);
} CIR_CATCH_BOUNDARY

// GetBlock::read_block (src/blocks.rs:207-240).  Unlike the reference's
// single read() + assert_eq! (:227-231), short reads are retried; a file that
// is shorter than recorded is an I/O error, not a panic.
int cir_blocks_read(cir_blocks* h, const uint8_t hash[32], uint8_t** data_out, size_t* len_out) try {
  if (!h || !hash || !data_out || !len_out) return fail(CIR_EINVAL, "null pointer");
  auto* m = reinterpret_cast<BlockMap*>(h);
  BlockPtr p;
  {
    std::shared_lock<std::shared_mutex> lk(m->mu);
    Key32 k;
    memcpy(k.b, hash, 32);
    auto it = m->blocks.find(k);
    if (it == m->blocks.end())
      return fail(CIR_ENOTFOUND, "block " + dirsig::to_hex(hash, 32) + " not found");
    p = it->second;
  }
  uint8_t* out = (uint8_t*)malloc(std::max<uint64_t>(p.size, 1));
  if (!out) return fail(CIR_ENOMEM, "malloc");
  if (p.data) {
    memcpy(out, p.data->data() + p.offset, p.size);
  } else {
    const int fd = ::open(p.path->c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
      free(out);
      return fail(CIR_EIO, "error reading file " + *p.path + ": " + strerror(errno));
    }
    uint64_t got = 0;
    while (got < p.size) {
      const ssize_t r = pread(fd, out + got, p.size - got, (off_t)(p.offset + got));
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) break;
      got += (uint64_t)r;
    }
    ::close(fd);
    if (got != p.size) {
      free(out);
      return fail(CIR_EIO, "error reading file " + *p.path + ": short read");
    }
  }
  *data_out = out;
  *len_out = p.size;
  return CIR_OK;
} CIR_CATCH_BOUNDARY

}  // extern "C"
