// DIRSIGNATURE.v1 emitter / parser.  See dirsig.hpp for the reference
// interfaces this restates.
#include "dirsig.hpp"

#include <stdlib.h>
#include <string.h>

#include <algorithm>

namespace cir {
namespace dirsig {

static const char kHex[] = "0123456789abcdef";

const char* hash_type_name(HashType t) {
  return t == HashType::kSha512_256 ? "sha512/256" : "blake2b/256";
}

bool parse_hash_type(const std::string& s, HashType* t) {
  if (s == "blake2b/256") {
    *t = HashType::kBlake2b256;
    return true;
  }
  if (s == "sha512/256") {
    *t = HashType::kSha512_256;
    return true;
  }
  return false;
}

size_t digest_len(HashType) { return 32; }

static bool needs_escape(unsigned char c) { return c <= 0x20 || c >= 0x7f || c == '\\'; }

std::string escape(const std::string& raw) {
  std::string out;
  out.reserve(raw.size());
  for (unsigned char c : raw) {
    if (needs_escape(c)) {
      out += "\\x";
      out += kHex[c >> 4];
      out += kHex[c & 15];
    } else {
      out += (char)c;
    }
  }
  return out;
}

static int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

bool unescape(const std::string& esc, std::string* raw) {
  raw->clear();
  for (size_t i = 0; i < esc.size(); ++i) {
    if (esc[i] == '\\') {
      if (esc.size() < i + 4 || esc[i + 1] != 'x') return false;
      const int a = hexval(esc[i + 2]), b = hexval(esc[i + 3]);
      if (a < 0 || b < 0) return false;
      *raw += (char)(a * 16 + b);
      i += 3;
    } else {
      *raw += esc[i];
    }
  }
  return true;
}

std::string to_hex(const uint8_t* p, size_t n) {
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) {
    s[2 * i] = kHex[p[i] >> 4];
    s[2 * i + 1] = kHex[p[i] & 15];
  }
  return s;
}

bool from_hex(const std::string& s, std::vector<uint8_t>* out) {
  if (s.size() % 2) return false;
  out->resize(s.size() / 2);
  for (size_t i = 0; i < out->size(); ++i) {
    const int a = hexval(s[2 * i]), b = hexval(s[2 * i + 1]);
    if (a < 0 || b < 0) return false;
    (*out)[i] = (uint8_t)(a * 16 + b);
  }
  return true;
}

Emitter::Emitter(const Header& h) {
  header_ = std::string("DIRSIGNATURE.v1 ") + hash_type_name(h.hash) +
            " block_size=" + std::to_string(h.block_size) + "\n";
  append(header_);
  hlen_ = len_;
}

Emitter::~Emitter() { free(buf_); }

bool Emitter::reserve_body(size_t n) {
  if (len_ + n <= cap_) return true;
  uint8_t* p = (uint8_t*)realloc(buf_, len_ + n);
  if (!p) return false;
  buf_ = p;
  cap_ = len_ + n;
  return true;
}

char* Emitter::grow(size_t n) {
  if (oom_) return nullptr;
  if (len_ + n > cap_) {
    // doubling; realloc of a large block remaps its pages instead of copying
    const size_t cap = std::max(len_ + n, std::max<size_t>(cap_ * 2, 4096));
    uint8_t* p = (uint8_t*)realloc(buf_, cap);
    if (!p) {
      oom_ = true;
      return nullptr;
    }
    buf_ = p;
    cap_ = cap;
  }
  char* at = (char*)buf_ + len_;
  len_ += n;
  return at;
}

void Emitter::append(const char* p, size_t n) {
  if (char* at = grow(n)) memcpy(at, p, n);
}

void Emitter::start_dir(const std::string& vpath) {
  append(escape(vpath));
  append("\n", 1);
}

void Emitter::add_file(const std::string& name, bool exe, uint64_t size, const uint8_t* hashes,
                       size_t nhash) {
  append("  ", 2);
  append(escape(name));
  append(exe ? " x " : " f ", 3);
  append(std::to_string(size));
  // " " + 64 hex digits per digest, written in place
  char* at = grow(65 * nhash + 1);
  if (!at) return;
  for (size_t i = 0; i < nhash; ++i) {
    *at++ = ' ';
    const uint8_t* h = hashes + 32 * i;
    for (int k = 0; k < 32; ++k) {
      *at++ = kHex[h[k] >> 4];
      *at++ = kHex[h[k] & 15];
    }
  }
  *at = '\n';
}

void Emitter::add_symlink(const std::string& name, const std::string& target) {
  append("  ", 2);
  append(escape(name));
  append(" s ", 3);
  append(escape(target));
  append("\n", 1);
}

void Emitter::consume(size_t upto) {
  if (upto <= drop_) return;
  const size_t n = std::min(upto - drop_, len_);
  memmove(buf_, buf_ + n, len_ - n);
  len_ -= n;
  drop_ += n;
}

bool Emitter::finish_footer(const uint8_t* footer, size_t footer_len) {
  append(to_hex(footer, footer_len) + '\n');
  return !oom_;
}

uint8_t* Emitter::finish_malloc(const uint8_t* footer, size_t footer_len, size_t* len) {
  if (drop_) return nullptr;
  append(to_hex(footer, footer_len) + '\n');
  if (oom_) return nullptr;
  uint8_t* out = buf_;
  *len = len_;
  buf_ = nullptr;
  len_ = cap_ = hlen_ = 0;
  return out;
}

static void split_ws(const std::string& s, std::vector<std::string>* parts) {
  parts->clear();
  size_t i = 0;
  while (i < s.size()) {
    while (i < s.size() && s[i] == ' ') ++i;
    if (i >= s.size()) break;
    size_t j = i;
    while (j < s.size() && s[j] != ' ') ++j;
    parts->push_back(s.substr(i, j - i));
    i = j;
  }
}

static bool parse_u64(const std::string& s, uint64_t* v) {
  if (s.empty() || s.size() > 20) return false;
  uint64_t x = 0;
  for (char c : s) {
    if (c < '0' || c > '9') return false;
    const uint64_t nx = x * 10 + (uint64_t)(c - '0');
    if (nx / 10 != x) return false;
    x = nx;
  }
  *v = x;
  return true;
}

// fill_dirs (src/cluster/download.rs:108-167) accepts only RootDir and
// Normal components in a directory line and needs a file_name() for every
// entry: "..", "." and empty names are IndexParseEnum::InvalidPath there.
// Rejecting them here also keeps register_dir (base + path) inside the
// registered directory.
static bool valid_name(const std::string& n) {
  return !n.empty() && n != "." && n != ".." && n.find('/') == std::string::npos &&
         n.find('\0') == std::string::npos;
}

static bool valid_dir_path(const std::string& p) {
  if (p.empty() || p[0] != '/' || p.find('\0') != std::string::npos) return false;
  size_t i = 1;
  while (i < p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    const std::string c = p.substr(i, j - i);
    if (c == "." || c == "..") return false;
    i = j + 1;
  }
  return true;
}

bool parse(const uint8_t* data, size_t len, Index* out, std::string* err) {
  out->entries.clear();
  std::vector<std::string> lines;
  size_t pos = 0;
  while (pos < len) {
    const void* nl = memchr(data + pos, '\n', len - pos);
    if (!nl) {
      *err = "index does not end with a newline";
      return false;
    }
    const size_t e = (const uint8_t*)nl - data;
    lines.emplace_back((const char*)data + pos, e - pos);
    pos = e + 1;
  }
  if (lines.size() < 2) {
    *err = "index too short";
    return false;
  }
  std::vector<std::string> tok;
  split_ws(lines[0], &tok);
  if (tok.size() < 2 || tok[0] != "DIRSIGNATURE.v1") {
    *err = "bad header signature";
    return false;
  }
  if (!parse_hash_type(tok[1], &out->header.hash)) {
    *err = "unknown hash type " + tok[1];
    return false;
  }
  out->header.block_size = 32768;
  for (size_t i = 2; i < tok.size(); ++i) {
    if (tok[i].compare(0, 11, "block_size=") == 0) {
      if (!parse_u64(tok[i].substr(11), &out->header.block_size) || out->header.block_size == 0) {
        *err = "bad block_size";
        return false;
      }
    }
  }
  const size_t dl = digest_len(out->header.hash);
  std::string cur_dir;
  bool have_dir = false;
  for (size_t li = 1; li + 1 < lines.size(); ++li) {
    const std::string& l = lines[li];
    if (!l.empty() && l[0] == '/') {
      if (!unescape(l, &cur_dir)) {
        *err = "bad escape in directory line";
        return false;
      }
      if (!valid_dir_path(cur_dir)) {
        *err = "Invalid path in index: " + l;
        return false;
      }
      have_dir = true;
      Entry e;
      e.kind = EntryKind::kDir;
      e.path = cur_dir;
      out->entries.push_back(std::move(e));
      continue;
    }
    if (l.size() < 3 || l[0] != ' ' || l[1] != ' ' || !have_dir) {
      *err = "unexpected line " + std::to_string(li + 1);
      return false;
    }
    split_ws(l.substr(2), &tok);
    if (tok.size() < 2) {
      *err = "short entry line " + std::to_string(li + 1);
      return false;
    }
    Entry e;
    std::string name;
    if (!unescape(tok[0], &name)) {
      *err = "bad escape in entry name";
      return false;
    }
    if (!valid_name(name)) {
      *err = "Invalid path in index: entry " + tok[0] + " on line " + std::to_string(li + 1);
      return false;
    }
    e.path = cur_dir == "/" ? "/" + name : cur_dir + "/" + name;
    if (tok[1] == "f" || tok[1] == "x") {
      e.kind = EntryKind::kFile;
      e.exe = tok[1] == "x";
      if (tok.size() < 3 || !parse_u64(tok[2], &e.size)) {
        *err = "bad file size on line " + std::to_string(li + 1);
        return false;
      }
      const uint64_t bs = out->header.block_size;
      const uint64_t want = e.size / bs + (e.size % bs != 0);  // no wrap near 2^64
      if (tok.size() - 3 != want) {
        *err = "wrong number of hashes on line " + std::to_string(li + 1);
        return false;
      }
      e.hashes.reserve(want * dl);
      std::vector<uint8_t> one;
      for (size_t k = 3; k < tok.size(); ++k) {
        if (!from_hex(tok[k], &one)) {
          *err = "bad hash hex on line " + std::to_string(li + 1);
          return false;
        }
        if (one.size() != dl) {  // the hashes are stored back to back
          out->bad_hash_size = true;
          *err = "hash of " + std::to_string(one.size()) + " bytes on line " +
                 std::to_string(li + 1);
          return false;
        }
        e.hashes.insert(e.hashes.end(), one.begin(), one.end());
      }
    } else if (tok[1] == "s") {
      e.kind = EntryKind::kLink;
      if (tok.size() != 3 || !unescape(tok[2], &e.target)) {
        *err = "bad symlink on line " + std::to_string(li + 1);
        return false;
      }
    } else {
      *err = "unknown entry type " + tok[1];
      return false;
    }
    out->entries.push_back(std::move(e));
  }
  if (!from_hex(lines.back(), &out->footer) || out->footer.empty()) {
    *err = "bad footer line";
    return false;
  }
  return true;
}

bool get_hash(const uint8_t* data, size_t len, std::vector<uint8_t>* id, std::string* err) {
  size_t end = len;
  if (end > 0 && data[end - 1] == '\n') --end;
  size_t start = end;
  while (start > 0 && data[start - 1] != '\n') --start;
  if (start == end || start == 0) {
    *err = "no footer line";
    return false;
  }
  if (!from_hex(std::string((const char*)data + start, end - start), id) || id->empty()) {
    *err = "footer is not hex";
    return false;
  }
  return true;
}

}  // namespace dirsig
}  // namespace cir
