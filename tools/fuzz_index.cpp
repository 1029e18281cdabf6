// Host-side fuzzing of the DIRSIGNATURE.v1 parser under ASan/UBSan
// (diagnostics, not part of the product).  Index bytes arrive from peers
// (src/daemon/index_cache.rs, src/blocks.rs:145 register_dir), so the parser
// must reject anything malformed without reading out of bounds.
//   * random emitted indexes: parse(emit(tree)) gives the tree back;
//   * byte-level mutations of valid indexes (flips, inserts, deletes,
//     truncations, splices of interesting tokens): parse and get_hash
//     either succeed or fail cleanly;
//   * escape/unescape round trips of random byte strings.
//
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all \
//       -Iciruela_amd/csrc tools/fuzz_index.cpp ciruela_amd/csrc/dirsig.cpp -o build/fuzz_index
//   ./build/fuzz_index [iterations]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "dirsig.hpp"

using namespace cir::dirsig;

namespace {

std::mt19937_64 rng(12345);

uint64_t rnd(uint64_t n) { return n ? rng() % n : 0; }

std::string rand_name() {
  static const char* pool[] = {"a", "b.txt", "...", ".x", "sp ace", "back\\slash", "tab\tx",
                               "\xff\xfe", "name", "nl\nx"};
  std::string s = pool[rnd(10)];
  if (rnd(3) == 0) s += std::to_string(rnd(1000));
  return s;
}

struct File {
  std::string name;
  bool exe;
  uint64_t size;
  std::vector<uint8_t> hashes;
  bool link;
  std::string target;
};

std::string build(const Header& h, const std::vector<std::pair<std::string, std::vector<File>>>& t) {
  Emitter em(h);
  for (const auto& d : t) {
    em.start_dir(d.first);
    for (const File& f : d.second) {
      if (f.link)
        em.add_symlink(f.name, f.target);
      else
        em.add_file(f.name, f.exe, f.size, f.hashes.data(), f.hashes.size() / 32);
    }
  }
  uint8_t footer[32];
  for (auto& b : footer) b = (uint8_t)rng();
  size_t n = 0;
  uint8_t* p = em.finish_malloc(footer, 32, &n);
  std::string out((const char*)p, n);
  free(p);
  return out;
}

int roundtrip_case() {
  Header h;
  h.hash = rnd(2) ? HashType::kBlake2b256 : HashType::kSha512_256;
  h.block_size = 1 + rnd(1 << 16);
  std::vector<std::pair<std::string, std::vector<File>>> t;
  const int nd = 1 + (int)rnd(4);
  for (int d = 0; d < nd; ++d) {
    std::string path = d == 0 ? "/" : "/" + rand_name();
    if (path.find('/', 1) != std::string::npos || path == "/." || path == "/..") path = "/d";
    std::vector<File> fs;
    const int nf = (int)rnd(5);
    for (int i = 0; i < nf; ++i) {
      File f;
      f.name = rand_name();
      f.link = rnd(5) == 0;
      f.exe = rnd(2);
      f.size = rnd(4) == 0 ? 0 : rnd(h.block_size * 5);
      if (!f.link) {
        f.hashes.resize(32 * (f.size / h.block_size + (f.size % h.block_size != 0)));
        for (auto& b : f.hashes) b = (uint8_t)rng();
      } else {
        f.target = rand_name();
      }
      fs.push_back(f);
    }
    t.emplace_back(path, fs);
  }
  const std::string idx = build(h, t);
  Index out;
  std::string err;
  if (!parse((const uint8_t*)idx.data(), idx.size(), &out, &err)) {
    fprintf(stderr, "roundtrip parse failed: %s\n", err.c_str());
    return 1;
  }
  size_t k = 0;
  for (const auto& d : t) {
    if (k >= out.entries.size() || out.entries[k].kind != EntryKind::kDir ||
        out.entries[k].path != d.first) {
      fprintf(stderr, "roundtrip: dir mismatch\n");
      return 1;
    }
    ++k;
    for (const File& f : d.second) {
      const Entry& e = out.entries[k++];
      const std::string want = d.first == "/" ? "/" + f.name : d.first + "/" + f.name;
      if (e.path != want || (f.link ? e.kind != EntryKind::kLink || e.target != f.target
                                    : e.kind != EntryKind::kFile || e.exe != f.exe ||
                                          e.size != f.size || e.hashes != f.hashes)) {
        fprintf(stderr, "roundtrip: entry mismatch at %s\n", want.c_str());
        return 1;
      }
    }
  }
  std::vector<uint8_t> id;
  if (!get_hash((const uint8_t*)idx.data(), idx.size(), &id, &err) || id != out.footer) {
    fprintf(stderr, "roundtrip: footer mismatch\n");
    return 1;
  }
  return 0;
}

void mutate(std::string* s) {
  static const char* tokens[] = {" ", "\n", "/", "..", ".", "\\x", "\\x2f", "\\", "f", "x", "s",
                                 "18446744073709551615", "99999999999999999999", "0",
                                 "block_size=0", "block_size=", "DIRSIGNATURE.v1", "ab", "  "};
  const int n = 1 + (int)rnd(4);
  for (int i = 0; i < n; ++i) {
    const size_t p = rnd(s->size() + 1);
    switch (rnd(5)) {
      case 0:
        if (!s->empty()) (*s)[rnd(s->size())] ^= (char)(1 << rnd(8));
        break;
      case 1:
        s->insert(p, tokens[rnd(sizeof(tokens) / sizeof(tokens[0]))]);
        break;
      case 2:
        s->erase(p, rnd(8));
        break;
      case 3:
        s->resize(p);
        break;
      default:
        s->insert(p, 1, (char)rng());
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  const long iters = argc > 1 ? atol(argv[1]) : 200000;
  long ok = 0, rejected = 0;
  for (long it = 0; it < iters; ++it) {
    if (roundtrip_case()) return 1;
    // a fresh valid index, then mutations of it
    Header h;
    h.block_size = 1 + rnd(100);
    std::vector<std::pair<std::string, std::vector<File>>> t;
    std::vector<File> fs(1);
    fs[0].name = rand_name();
    fs[0].exe = false;
    fs[0].link = false;
    fs[0].size = rnd(300);
    fs[0].hashes.assign(32 * (fs[0].size / h.block_size + (fs[0].size % h.block_size != 0)), 0xab);
    t.emplace_back("/", fs);
    std::string s = build(h, t);
    mutate(&s);
    // parse from a heap copy of exactly s.size() bytes, so ASan sees any
    // read past the end
    std::vector<uint8_t> buf(s.begin(), s.end());
    Index out;
    std::string err;
    const bool good = parse(buf.data(), buf.size(), &out, &err);
    std::vector<uint8_t> id;
    (void)get_hash(buf.data(), buf.size(), &id, &err);
    good ? ++ok : ++rejected;
    // escape / unescape
    std::string raw(rnd(12), '\0');
    for (auto& c : raw) c = (char)rng();
    std::string back;
    if (!unescape(escape(raw), &back) || back != raw) {
      fprintf(stderr, "escape round trip failed\n");
      return 1;
    }
  }
  printf("fuzz_index: %ld iterations, %ld mutated indexes parsed, %ld rejected, no sanitizer "
         "report\n", iters, ok, rejected);
  return 0;
}
