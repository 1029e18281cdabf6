/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by or called
 * from the product (ciruela_amd/); only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, as the checker / CPU baseline.
 *
 * CPU restatement of the reference's block-hash algorithm:
 *   BlockHash::hash_bytes (reference src/block_id.rs:37-43) =
 *     blake2 0.7.1 `Blake2b::VariableOutput::new(32)` + input + variable_result
 *   = BLAKE2b (RFC 7693) with digest length nn = 32, no key, encoded in the
 *     parameter block (p[0] = 0x01010000 ^ (kk << 8) ^ nn, RFC 7693 2.5/3.3).
 *   dir-signature 0.2.9 `Hashes::hash_file(hash, block_size, reader)`
 *   (called at src/blocks.rs:193, src/cluster/download.rs:257) = that hash
 *   over every block_size chunk of the file, last chunk short, no chunk for an
 *   empty file (fixture src/cluster/download.rs:361 "test.txt f 0").
 * The blake2/dir-signature crates are not vendored in the reference and Rust
 * is not installed, so this is a restatement of RFC 7693 (blake2 0.7.1,
 * Cargo.lock:110-117, implements RFC 7693); it is pinned by the RFC's
 * Appendix A vector and by vectors generated with Python hashlib
 * (tests/golden/make_golden.py), see tests/test_oracle.py.
 *
 * Also SHA-512/256 (FIPS 180-4), the second dir-signature hash type, pinned
 * against hashlib.sha512_256 and the reference's index fixture.
 *
 * Build: oracle/Makefile -> oracle/build/liboracle_blake2b.so
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const uint64_t IV[8] = {
    0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
    0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

/* RFC 7693 section 2.7 */
static const uint8_t SIGMA[12][16] = {
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

static inline uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

static inline uint64_t load64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

/* F (RFC 7693 section 3.2) */
static void compress(uint64_t h[8], const uint8_t block[128], uint64_t t0, uint64_t t1, int last) {
  uint64_t v[16], m[16];
  for (int i = 0; i < 16; ++i) m[i] = load64(block + 8 * i);
  for (int i = 0; i < 8; ++i) {
    v[i] = h[i];
    v[i + 8] = IV[i];
  }
  v[12] ^= t0;
  v[13] ^= t1;
  if (last) v[14] = ~v[14];
#define G(a, b, c, d, x, y)          \
  do {                               \
    v[a] = v[a] + v[b] + (x);        \
    v[d] = rotr64(v[d] ^ v[a], 32);  \
    v[c] = v[c] + v[d];              \
    v[b] = rotr64(v[b] ^ v[c], 24);  \
    v[a] = v[a] + v[b] + (y);        \
    v[d] = rotr64(v[d] ^ v[a], 16);  \
    v[c] = v[c] + v[d];              \
    v[b] = rotr64(v[b] ^ v[c], 63);  \
  } while (0)
  for (int r = 0; r < 12; ++r) {
    const uint8_t* s = SIGMA[r];
    G(0, 4, 8, 12, m[s[0]], m[s[1]]);
    G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    G(2, 6, 10, 14, m[s[4]], m[s[5]]);
    G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    G(0, 5, 10, 15, m[s[8]], m[s[9]]);
    G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    G(2, 7, 8, 13, m[s[12]], m[s[13]]);
    G(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
#undef G
  for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

/* BLAKE2b with outlen (1..64) bytes, unkeyed (RFC 7693 section 3.3). */
int oracle_blake2b(uint8_t* out, size_t outlen, const uint8_t* in, size_t inlen) {
  if (outlen == 0 || outlen > 64) return -1;
  uint64_t h[8];
  memcpy(h, IV, sizeof h);
  h[0] ^= 0x01010000ULL ^ (uint64_t)outlen;
  uint64_t t0 = 0, t1 = 0;
  uint8_t buf[128];
  /* all but the last block */
  while (inlen > 128) {
    t0 += 128;
    if (t0 < 128) ++t1;
    compress(h, in, t0, t1, 0);
    in += 128;
    inlen -= 128;
  }
  /* last block (possibly empty), zero padded */
  memset(buf, 0, sizeof buf);
  memcpy(buf, in, inlen);
  t0 += inlen;
  if (t0 < inlen) ++t1;
  compress(h, buf, t0, t1, 1);
  for (size_t i = 0; i < outlen; ++i) out[i] = (uint8_t)(h[i / 8] >> (8 * (i % 8)));
  return 0;
}

/* BlockHash::hash_bytes */
int oracle_blake2b256(uint8_t out[32], const uint8_t* in, size_t inlen) {
  return oracle_blake2b(out, 32, in, inlen);
}

/* ---- batch forms, threaded (CPU baseline: dir-signature hashes on a CPU
 *      pool of `threads` workers; here the unit of work is a block) ---- */

int oracle_sha512_256(uint8_t out[32], const uint8_t* in, size_t inlen);

struct job {
  int sha; /* 1: SHA-512/256 (dir-signature HashType::sha512_256) */
  const uint8_t* arena;
  const uint64_t* off;
  const uint32_t* len;
  uint64_t nbytes, bs; /* chunk form when off == NULL */
  uint8_t* out;
  size_t n;
  size_t next;
  pthread_mutex_t mu;
};

static void* worker(void* arg) {
  struct job* j = (struct job*)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    size_t b0 = j->next;
    j->next += 64;
    pthread_mutex_unlock(&j->mu);
    if (b0 >= j->n) return NULL;
    size_t b1 = b0 + 64 < j->n ? b0 + 64 : j->n;
    for (size_t b = b0; b < b1; ++b) {
      const uint8_t* p;
      uint64_t l;
      if (j->off) {
        p = j->arena + j->off[b];
        l = j->len[b];
      } else {
        uint64_t o = (uint64_t)b * j->bs;
        p = j->arena + o;
        l = j->nbytes - o < j->bs ? j->nbytes - o : j->bs;
      }
      if (j->sha)
        oracle_sha512_256(j->out + 32 * b, p, l);
      else
        oracle_blake2b256(j->out + 32 * b, p, l);
    }
  }
}

static int run(struct job* j, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_mutex_init(&j->mu, NULL);
  j->next = 0;
  pthread_t th[256];
  int started = 0;
  for (int i = 1; i < threads; ++i)
    if (pthread_create(&th[started], NULL, worker, j) == 0) ++started;
  worker(j);
  for (int i = 0; i < started; ++i) pthread_join(th[i], NULL);
  pthread_mutex_destroy(&j->mu);
  return 0;
}

/* block b = arena[off[b] .. off[b] + len[b]) -> out + 32 b */
int oracle_hash_blocks(const uint8_t* arena, const uint64_t* off, const uint32_t* len, size_t n,
                       uint8_t* out, int threads) {
  struct job j;
  memset(&j, 0, sizeof j);
  j.arena = arena;
  j.off = off;
  j.len = len;
  j.out = out;
  j.n = n;
  return run(&j, threads);
}

/* Hashes::hash_file over a memory buffer: ceil(nbytes / bs) digests */
int oracle_hash_chunks(const uint8_t* data, uint64_t nbytes, uint64_t bs, uint8_t* out,
                       int threads) {
  if (bs == 0) return -1;
  struct job j;
  memset(&j, 0, sizeof j);
  j.arena = data;
  j.nbytes = nbytes;
  j.bs = bs;
  j.out = out;
  j.n = (size_t)((nbytes + bs - 1) / bs);
  return run(&j, threads);
}

/* Hashes::hash_file(HashType::sha512_256(), bs, ..) over a memory buffer */
int oracle_sha_chunks(const uint8_t* data, uint64_t nbytes, uint64_t bs, uint8_t* out,
                      int threads) {
  if (bs == 0) return -1;
  struct job j;
  memset(&j, 0, sizeof j);
  j.sha = 1;
  j.arena = data;
  j.nbytes = nbytes;
  j.bs = bs;
  j.out = out;
  j.n = (size_t)((nbytes + bs - 1) / bs);
  return run(&j, threads);
}

/* ---- the reference CPU indexer's hashing loop, restated: v1::scan hashes
 * whole files on a pool of `threads` CPU workers (ScannerConfig::threads,
 * src/client/sync/uploads.rs:50-53; default 4, src/client/global_options.rs:13),
 * each worker reading its file in block_size chunks and hashing every chunk
 * (Hashes::hash_file).  File i's digests go to out + 32 * first[i]; a file
 * must hold exactly ceil(size / bs) blocks of the size the caller planned
 * (returned as -EIO otherwise). ---- */
#include <errno.h>
#include <fcntl.h>
#include <unistd.h>

struct files_job {
  const char* const* paths;
  const uint64_t* first;
  const uint64_t* nblk;
  size_t n, next;
  uint64_t bs;
  uint8_t* out;
  int err;
  int sha; /* 1: SHA-512/256 */
  pthread_mutex_t mu;
};

static void* files_worker(void* arg) {
  struct files_job* j = (struct files_job*)arg;
  uint8_t* buf = (uint8_t*)malloc(j->bs ? j->bs : 1);
  if (!buf) return NULL;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    size_t f = j->next++;
    int stop = j->err != 0;
    pthread_mutex_unlock(&j->mu);
    if (f >= j->n || stop) break;
    int fd = open(j->paths[f], O_RDONLY);
    int e = fd < 0 ? errno : 0;
    uint64_t b = 0;
    while (!e) {
      uint64_t got = 0;
      while (got < j->bs) {
        ssize_t r = read(fd, buf + got, j->bs - got);
        if (r < 0 && errno == EINTR) continue;
        if (r < 0) e = errno;
        if (r <= 0) break;
        got += (uint64_t)r;
      }
      if (e || got == 0) break;
      if (b >= j->nblk[f]) {
        e = EIO;
        break;
      }
      if (j->sha)
        oracle_sha512_256(j->out + 32 * (j->first[f] + b), buf, got);
      else
        oracle_blake2b256(j->out + 32 * (j->first[f] + b), buf, got);
      ++b;
      if (got < j->bs) break;
    }
    if (fd >= 0) close(fd);
    if (!e && b != j->nblk[f]) e = EIO;
    if (e) {
      pthread_mutex_lock(&j->mu);
      if (!j->err) j->err = e;
      pthread_mutex_unlock(&j->mu);
    }
  }
  free(buf);
  return NULL;
}

static int hash_files(const char* const* paths, const uint64_t* first, const uint64_t* nblk,
                      size_t n, uint64_t bs, uint8_t* out, int threads, int sha) {
  if (bs == 0) return -EINVAL;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  struct files_job j;
  memset(&j, 0, sizeof j);
  j.paths = paths;
  j.first = first;
  j.nblk = nblk;
  j.n = n;
  j.bs = bs;
  j.out = out;
  j.sha = sha;
  pthread_mutex_init(&j.mu, NULL);
  pthread_t th[256];
  int started = 0;
  for (int i = 1; i < threads; ++i)
    if (pthread_create(&th[started], NULL, files_worker, &j) == 0) ++started;
  files_worker(&j);
  for (int i = 0; i < started; ++i) pthread_join(th[i], NULL);
  pthread_mutex_destroy(&j.mu);
  return -j.err;
}

int oracle_hash_files(const char* const* paths, const uint64_t* first, const uint64_t* nblk,
                      size_t n, uint64_t bs, uint8_t* out, int threads) {
  return hash_files(paths, first, nblk, n, bs, out, threads, 0);
}

/* the same with HashType::sha512_256() */
int oracle_sha_files(const char* const* paths, const uint64_t* first, const uint64_t* nblk,
                     size_t n, uint64_t bs, uint8_t* out, int threads) {
  return hash_files(paths, first, nblk, n, bs, out, threads, 1);
}

/* ---- SHA-512/256 (FIPS 180-4), dir-signature's HashType::sha512_256();
 * the reference's index fixture (src/cluster/download.rs:357-366) uses it. */
static const uint64_t SHA_K[80] = {
0x428a2f98d728ae22ULL,
0x7137449123ef65cdULL,
0xb5c0fbcfec4d3b2fULL,
0xe9b5dba58189dbbcULL,
0x3956c25bf348b538ULL,
0x59f111f1b605d019ULL,
0x923f82a4af194f9bULL,
0xab1c5ed5da6d8118ULL,
0xd807aa98a3030242ULL,
0x12835b0145706fbeULL,
0x243185be4ee4b28cULL,
0x550c7dc3d5ffb4e2ULL,
0x72be5d74f27b896fULL,
0x80deb1fe3b1696b1ULL,
0x9bdc06a725c71235ULL,
0xc19bf174cf692694ULL,
0xe49b69c19ef14ad2ULL,
0xefbe4786384f25e3ULL,
0x0fc19dc68b8cd5b5ULL,
0x240ca1cc77ac9c65ULL,
0x2de92c6f592b0275ULL,
0x4a7484aa6ea6e483ULL,
0x5cb0a9dcbd41fbd4ULL,
0x76f988da831153b5ULL,
0x983e5152ee66dfabULL,
0xa831c66d2db43210ULL,
0xb00327c898fb213fULL,
0xbf597fc7beef0ee4ULL,
0xc6e00bf33da88fc2ULL,
0xd5a79147930aa725ULL,
0x06ca6351e003826fULL,
0x142929670a0e6e70ULL,
0x27b70a8546d22ffcULL,
0x2e1b21385c26c926ULL,
0x4d2c6dfc5ac42aedULL,
0x53380d139d95b3dfULL,
0x650a73548baf63deULL,
0x766a0abb3c77b2a8ULL,
0x81c2c92e47edaee6ULL,
0x92722c851482353bULL,
0xa2bfe8a14cf10364ULL,
0xa81a664bbc423001ULL,
0xc24b8b70d0f89791ULL,
0xc76c51a30654be30ULL,
0xd192e819d6ef5218ULL,
0xd69906245565a910ULL,
0xf40e35855771202aULL,
0x106aa07032bbd1b8ULL,
0x19a4c116b8d2d0c8ULL,
0x1e376c085141ab53ULL,
0x2748774cdf8eeb99ULL,
0x34b0bcb5e19b48a8ULL,
0x391c0cb3c5c95a63ULL,
0x4ed8aa4ae3418acbULL,
0x5b9cca4f7763e373ULL,
0x682e6ff3d6b2b8a3ULL,
0x748f82ee5defb2fcULL,
0x78a5636f43172f60ULL,
0x84c87814a1f0ab72ULL,
0x8cc702081a6439ecULL,
0x90befffa23631e28ULL,
0xa4506cebde82bde9ULL,
0xbef9a3f7b2c67915ULL,
0xc67178f2e372532bULL,
0xca273eceea26619cULL,
0xd186b8c721c0c207ULL,
0xeada7dd6cde0eb1eULL,
0xf57d4f7fee6ed178ULL,
0x06f067aa72176fbaULL,
0x0a637dc5a2c898a6ULL,
0x113f9804bef90daeULL,
0x1b710b35131c471bULL,
0x28db77f523047d84ULL,
0x32caab7b40c72493ULL,
0x3c9ebe0a15c9bebcULL,
0x431d67c49c100d4cULL,
0x4cc5d4becb3e42b6ULL,
0x597f299cfc657e2aULL,
0x5fcb6fab3ad6faecULL,
0x6c44198c4a475817ULL};
static const uint64_t SHA_IV256[8] = {
0x22312194fc2bf72cULL,
0x9f555fa3c84c64c2ULL,
0x2393b86b6f53b151ULL,
0x963877195940eabdULL,
0x96283ee2a88effe3ULL,
0xbe5e1e2553863992ULL,
0x2b0199fc2c85b8aaULL,
0x0eb72ddc81c52ca2ULL};

static inline uint64_t be64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return v;
}

static void sha_compress(uint64_t h[8], const uint8_t blk[128]) {
  uint64_t w[80];
  for (int t = 0; t < 16; ++t) w[t] = be64(blk + 8 * t);
  for (int t = 16; t < 80; ++t) {
    uint64_t s0 = rotr64(w[t - 15], 1) ^ rotr64(w[t - 15], 8) ^ (w[t - 15] >> 7);
    uint64_t s1 = rotr64(w[t - 2], 19) ^ rotr64(w[t - 2], 61) ^ (w[t - 2] >> 6);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int t = 0; t < 80; ++t) {
    uint64_t S1 = rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41);
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t t1 = hh + S1 + ch + SHA_K[t] + w[t];
    uint64_t S0 = rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39);
    uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

int oracle_sha512_256(uint8_t out[32], const uint8_t* in, size_t inlen) {
  uint64_t h[8];
  memcpy(h, SHA_IV256, sizeof h);
  size_t off = 0;
  while (inlen - off >= 128) {
    sha_compress(h, in + off);
    off += 128;
  }
  uint8_t buf[256];
  memset(buf, 0, sizeof buf);
  size_t rem = inlen - off;
  memcpy(buf, in + off, rem);
  buf[rem] = 0x80;
  size_t nb = rem + 17 > 128 ? 2 : 1;
  uint64_t bits = (uint64_t)inlen << 3;
  for (int i = 0; i < 8; ++i) buf[nb * 128 - 1 - i] = (uint8_t)(bits >> (8 * i));
  buf[nb * 128 - 9] |= (uint8_t)(((uint64_t)inlen >> 61) & 7);
  for (size_t b = 0; b < nb; ++b) sha_compress(h, buf + 128 * b);
  for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(h[i / 8] >> (56 - 8 * (i % 8)));
  return 0;
}

/* Host twin of the product's synthetic-data kernel (k_fill_splitmix64),
 * used to regenerate sampled blocks for checking. */
static inline uint64_t splitmix64_at(uint64_t seed, uint64_t k) {
  uint64_t z = seed + (k + 1) * 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

/* Fill words [word0, word0 + nwords) of the synthetic buffer into dst. */
void oracle_splitmix64_fill(uint64_t* dst, uint64_t word0, uint64_t nwords, uint64_t seed,
                            uint64_t block_words, uint64_t first_block) {
  for (uint64_t i = 0; i < nwords; ++i) {
    uint64_t k = word0 + i, s = seed, w = k;
    if (block_words) {
      s = seed ^ (first_block + k / block_words);
      w = k % block_words;
    }
    dst[i] = splitmix64_at(s, w);
  }
}
