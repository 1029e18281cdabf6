// DIRSIGNATURE.v1 index format: emitter and parser (host C++).
//
// Restates what ciruela takes from the external crate dir-signature 0.2.9
// (Cargo.toml:35; not vendored in the reference):
//   * v1::Emitter  — used by MutableIndex::to_raw_data
//                    (src/cluster/download.rs:266-276, dir order :287-319)
//   * v1::Parser   — used by ThreadedBlockReader::register_dir
//                    (src/blocks.rs:150-183) and RawIndex::into_mut
//   * get_hash     — InMemoryIndexes::register_index (src/index.rs:98-105)
// Pinned by the reference's only index fixture (src/cluster/download.rs:
// 357-366): header line, "/dir" lines, "  name f size hex..." entries, an
// empty file carries no hashes, footer = H(every byte after the header line).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace cir {
namespace dirsig {

enum class HashType { kBlake2b256 = 1, kSha512_256 = 2 };

const char* hash_type_name(HashType t);           // "blake2b/256", "sha512/256"
bool parse_hash_type(const std::string& s, HashType* t);

// dir-signature escapes bytes outside printable ASCII, the space and the
// backslash as \xNN (lowercase hex).  Unverified against the crate (see
// DESIGN.md "Index format"); consistent with every fixture in the reference.
std::string escape(const std::string& raw);
bool unescape(const std::string& esc, std::string* raw);

std::string to_hex(const uint8_t* p, size_t n);
bool from_hex(const std::string& s, std::vector<uint8_t>* out);

struct Header {
  HashType hash = HashType::kBlake2b256;
  uint64_t block_size = 32768;
};

// Streaming emitter: header, then for each directory start_dir + entries;
// finish_malloc() needs the footer digest of the body (computed by the
// caller) and appends its hex line.  The index is built in place in one
// malloc'd buffer (header first), so finishing hands that buffer over
// without copying the body.  A caller that writes the index out as it goes
// (cir_scan_v1_write) drops what it has written with consume(), so the
// buffer holds only the unwritten tail; offsets stay absolute (bytes since
// the start of the index, or of the body) across a consume().
class Emitter {
 public:
  explicit Emitter(const Header& h);
  ~Emitter();
  Emitter(const Emitter&) = delete;
  Emitter& operator=(const Emitter&) = delete;
  // room for n more body bytes (an estimate: appends still grow the buffer)
  bool reserve_body(size_t n);
  void start_dir(const std::string& vpath);  // "/" or "/a/b" (raw bytes)
  void add_file(const std::string& name, bool exe, uint64_t size, const uint8_t* hashes,
                size_t nhash);
  void add_symlink(const std::string& name, const std::string& target);
  // Bytes the footer hashes: everything after the header line.  A pointer
  // moves when the buffer grows or is consumed; an offset into the body
  // stays valid.  body_at(off) needs off at or past what consume() dropped.
  const char* body_at(size_t off) const { return (const char*)buf_ + hlen_ + off - drop_; }
  const char* body_data() const { return body_at(0); }  // nothing of the body consumed
  size_t body_size() const { return drop_ + len_ - hlen_; }
  // the whole index so far: bytes [0, index_size()), held from consumed() on
  size_t index_size() const { return drop_ + len_; }
  size_t consumed() const { return drop_; }
  size_t header_size() const { return hlen_; }
  const uint8_t* index_at(size_t off) const { return buf_ + off - drop_; }
  // drop the index bytes before offset `upto` (consumed() <= upto <= index_size())
  void consume(size_t upto);
  // header + body + hex footer + newline in one malloc'd buffer (free()),
  // which the emitter gives up; null if out of memory (or after an append
  // failed to allocate), or if anything was consumed.
  uint8_t* finish_malloc(const uint8_t* footer, size_t footer_len, size_t* len);
  // append the hex footer line only (the streaming form); false if out of memory
  bool finish_footer(const uint8_t* footer, size_t footer_len);
  bool failed() const { return oom_; }
  const std::string& header_line() const { return header_; }

 private:
  char* grow(size_t n);  // n more bytes at the end; null on allocation failure
  void append(const char* p, size_t n);
  void append(const std::string& s) { append(s.data(), s.size()); }
  std::string header_;
  uint8_t* buf_ = nullptr;
  size_t len_ = 0, cap_ = 0, hlen_ = 0;
  size_t drop_ = 0;  // index bytes consumed before buf_[0]
  bool oom_ = false;
};

enum class EntryKind { kDir, kFile, kLink };

struct Entry {
  EntryKind kind;
  std::string path;  // kDir: directory path; kFile/kLink: full path (dir + "/" + name)
  bool exe = false;
  uint64_t size = 0;
  std::vector<uint8_t> hashes;  // nhash x digest_len
  std::string target;           // kLink
};

struct Index {
  Header header;
  std::vector<Entry> entries;
  std::vector<uint8_t> footer;  // decoded last line
  // set (and parse() fails) when a block hash decodes to other than
  // digest_len bytes: register_dir reports it as DirError::HashSize
  // (BlockHash::from_bytes, src/blocks.rs:168-170), other callers as a
  // parse error
  bool bad_hash_size = false;
};

// Parse a whole index.  Returns false with *err set on malformed input
// (the reference's v1::ParseError).
bool parse(const uint8_t* data, size_t len, Index* out, std::string* err);

// dir_signature::get_hash: decode the hex on the last line.
bool get_hash(const uint8_t* data, size_t len, std::vector<uint8_t>* id, std::string* err);

size_t digest_len(HashType t);

}  // namespace dirsig
}  // namespace cir
