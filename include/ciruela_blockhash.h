/*
 * ciruela_blockhash.h — C ABI of the MI355X (gfx950) block-indexing path.
 *
 * Drop-in boundary for ciruela's indexing loop.  Every entry
 * point names the reference interface it replaces (paths are relative to the
 * tailhook/ciruela v0.6.12 tree).  Every block digest is computed on the GPU
 * (hand-written HIP kernels for gfx950); the host side stages bytes and
 * bookkeeps, and by default hashes the one serial footer chain of a scanned
 * index (cir_set_footer_mode).  There is no CPU fallback for block hashes:
 * without a usable GPU every hashing call returns CIR_ENODEV.
 *
 * Conventions
 *   - return 0 (CIR_OK) on success, a negative CIR_E* code on failure; the
 *     detail of the last failure is in cir_last_error().  No call aborts the
 *     process on bad input it can check (the reference panics only on
 *     impossible states, e.g. src/block_id.rs:38,41 "length is ok").  The
 *     caller's own buffers are trusted, as a slice is in the reference: the
 *     descriptor batches (cir_hash_blocks[_dev][_ht], cir_verify_blocks[_dev])
 *     read arena + off[b] .. + len[b] as given (an out-of-range descriptor is
 *     a memory fault, on the GPU or the host), so descriptors derived from
 *     untrusted data go through the *_bounded entry points, which check
 *     every one against the arena's size (on the device for *_dev_bounded).
 *   - digests are 32 raw bytes (BlockHash([u8; 32]), src/block_id.rs:19),
 *     printed as lowercase hex (src/hexlify.rs:9-13).
 *   - `stream` arguments are hipStream_t passed as void* (NULL = the null
 *     stream of the calling thread's current device).  *_dev calls are
 *     asynchronous on that stream and never synchronise the device (with a
 *     context, a descriptor batch larger than any before grows the device's
 *     ordering or bounds scratch, waiting once for that scratch's previous
 *     user).
 *   - no call changes the calling thread's current HIP device: entry points
 *     that work on other devices restore it before returning.
 *   - buffers returned through `uint8_t**` are released with cir_free().
 *   - environment (read by the library; none is needed):
 *       CIR_STAGE_COPY=direct  host threads fill the pinned staging slots with
 *                              plain pread()/memcpy() instead of streaming
 *                              (non-temporal) stores;
 *       CIR_STAGE_RAMP=0       staged host paths start with whole-slot batches
 *                              (default: the first three batches ramp up from
 *                              1/8 of a slot, so the first upload starts
 *                              sooner);
 *       CIR_FOOTER=gpu         cir_init's contexts start with CIR_FOOTER_GPU;
 *       CIR_TRACE=1            per-batch timings on stderr;
 *       CIR_DEBUG_SPLIT=k      (tests) every opened GPU appears k times.
 *       CIR_DEBUG_STRIPE_BLOCKS=n  (tests) a scan over several devices deals
 *                              stripes of n blocks (default: one staging
 *                              slot of whole blocks) round-robin to them.
 */
#ifndef CIRUELA_BLOCKHASH_H
#define CIRUELA_BLOCKHASH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CIR_DIGEST_BYTES 32
#define CIR_DEFAULT_BLOCK_SIZE 32768 /* src/daemon/disk/public.rs:154 */

/* Every int-returning call returns one of these (the text of the last
 * failure on this thread: cir_last_error).  No C++ exception leaves the
 * library: an allocation that fails inside it is CIR_ENOMEM. */
enum cir_status {
  CIR_OK = 0,
  CIR_EIO = -1,        /* filesystem error: scan's io::Error (src/client/sync/uploads.rs:57) */
  CIR_EINVAL = -2,     /* bad argument, length or shape */
  CIR_EHIP = -3,       /* HIP runtime error (hipError_t text in cir_last_error) */
  CIR_ENOMEM = -4,     /* host or device allocation failed */
  CIR_EPARSE = -5,     /* IndexError::ParseError (src/index.rs:64) / DirError::ParseError (src/blocks.rs:117) */
  CIR_ENOTFOUND = -6,  /* ReadError::NotFound (src/index.rs:78, src/blocks.rs:101) */
  CIR_EHASHSIZE = -7,  /* DirError::HashSize (src/blocks.rs:123) */
  CIR_ENODEV = -8,     /* no usable gfx950 device */
  CIR_EUNSUPPORTED = -9, /* reserved (every dir-signature hash type is implemented) */
  CIR_EAGAIN = -10       /* cir_verify_submit, non-blocking: the verify queue is full */
};

/* dir-signature HashType (external crate 0.2.9; header tokens in the index) */
enum cir_hash_type {
  CIR_HASH_BLAKE2B_256 = 1, /* HashType::blake2b_256()  "blake2b/256" */
  CIR_HASH_SHA512_256 = 2   /* HashType::sha512_256()   "sha512/256" */
};

typedef struct cir_ctx cir_ctx;

/* ---- context --------------------------------------------------------- */

/* Open the devices in device_mask (bit i = HIP device i; 0 = every visible
 * device; the devices are opened in parallel, one host thread each).
 * staging_bytes sizes each device's host->device staging slots for the
 * host-memory entry points (0 = 256 MiB).  What cir_init creates per device:
 * its streams (compute, copy, quad part, footer chain), the relay scratch,
 * the ordering scratch for one full staging batch and -- unless staging_bytes
 * is CIR_STAGING_LAZY -- three staging slots (pinned host + device memory of
 * staging_bytes each, plus descriptor and digest buffers).  A tiny warm-up
 * hash loads the kernels and the first copies on the staging and chain
 * streams are paid here.  Allocated later, on first use: the footer-chain
 * text buffers (cir_scan_v1 with CIR_FOOTER_GPU), the single-launch buffers
 * of cir_blake2b256, timing events, and -- with CIR_STAGING_LAZY -- the
 * staging slots (256 MiB each), so a context used only through the *_dev
 * entry points pins no staging memory.
 *
 * Cost per opened device, staging S (blocks per slot B = max(S / 512, 4096)):
 *   pinned host memory  3 x (S + 44 B)            = 834 MiB at the default
 *   device memory       3 x (S + 44 B) + 8 B + 4 MiB (ordering, relay)
 *                                                 = 842 MiB at the default
 *   with CIR_STAGING_LAZY: ~4.2 MiB of device memory and no pinned memory
 *   until a host path runs; plus, either way, the HIP runtime's own context
 *   on that device and cir_init's 0.1-0.3 s of start-up. */
#define CIR_STAGING_LAZY ((uint64_t)-1)
int cir_init(cir_ctx** ctx, uint32_t device_mask, uint64_t staging_bytes);
/* cir_init with a device-count hint: opens at most max_devices of the
 * devices device_mask selects, the lowest-numbered first (0 = no cap, as
 * cir_init).  With cir_devices_for_bytes a caller that knows how much input
 * it will stage opens only the devices that input can use.  flags: 0 or
 * CIR_INIT_ONE_SHOT. */
int cir_init_n(cir_ctx** ctx, uint32_t device_mask, uint64_t staging_bytes, uint32_t max_devices,
               uint32_t flags);
/* A context for one short job (the CLI's sync of an input that fits one
 * staging slot): each device gets ONE stream for its uploads and kernels and
 * one staging slot.  A HIP stream on a hardware queue of its own costs 8-10
 * ms to create in a fresh process (the first 19 ms; profiles/r05/
 * start_env.log), and the copy, footer-chain and quad-part streams were
 * ~25 ms of a 55 ms cir_init.  Every entry point still works: the other
 * slots are allocated and the footer-chain stream created if a call needs
 * them, uploads wait for the previous batch's kernels, and an ordered
 * batch's quad part runs behind its lane part instead of beside it (config
 * 3's mixed batch takes the sum of the two parts, not the longer). */
#define CIR_INIT_ONE_SHOT 1u
/* The devices worth opening for work_bytes of host-path input (a scan's
 * tree, a hash_file / hash_memory input): ceil(work_bytes / (2 x staging))
 * -- each device gets at least two staging batches, so its start-up and
 * pinned slots are not spent on a fraction of one -- capped at `visible`,
 * at least 1; work_bytes == 0 (unknown) gives `visible`.  staging_bytes as
 * cir_init's (0 / CIR_STAGING_LAZY = 256 MiB).  Pure: no HIP call. */
uint32_t cir_devices_for_bytes(uint64_t work_bytes, uint64_t staging_bytes, uint32_t visible);
void cir_destroy(cir_ctx* ctx);
int cir_device_count(void);
/* devices opened by ctx; ids[i] receives the HIP ordinal of the i-th. */
int cir_ctx_devices(const cir_ctx* ctx, int* ids, int max_ids);
const char* cir_strerror(int status);
const char* cir_last_error(void); /* thread-local detail of the last failure */
void cir_free(void* p);

/* ---- block hashes ---------------------------------------------------- */

/* BlockHash::hash_bytes(&[u8]) -> BlockHash   (src/block_id.rs:37-43).
 * Single host buffer, hashed on the process-default device context. */
int cir_blake2b256(const uint8_t* p, size_t n, uint8_t out[CIR_DIGEST_BYTES]);

/* Device-resident Hashes::hash_file: the bytes [d_data, d_data + nbytes) of
 * one file already in HBM, split into ceil(nbytes / block_size) blocks (the
 * last one short; none when nbytes == 0), digest i -> d_out + 32 i (d_out
 * 16-byte aligned, as hipMalloc returns it).  This is the metric path
 * (BASELINE.json configs 2 and 4).  With a context (ctx != NULL) parts of
 * the file may also run on the device's own quad-part stream (the short last
 * block; the blocks past a whole number of waves per SIMD), forked from and
 * joined back into `stream`, so the call is ordered on `stream` as one
 * launch would be; ctx == NULL: one launch on `stream`, no side streams. */
int cir_hash_chunks_dev(cir_ctx* ctx, const void* d_data, uint64_t nbytes, uint64_t block_size,
                        uint8_t* d_out, void* stream);

/* Device-resident batch of independent blocks: block b = d_arena[d_off[b] ..
 * d_off[b] + d_len[b]) -> d_out + 32 b (d_out 16-byte aligned).  Any order,
 * any mix of lengths (config 3); zero-length blocks hash as the empty input. */
int cir_hash_blocks_dev(cir_ctx* ctx, const void* d_arena, const uint64_t* d_off,
                        const uint32_t* d_len, size_t nblk, uint8_t* d_out, void* stream);

/* cir_hash_blocks_dev_ht for descriptors the caller cannot vouch for (the
 * daemon's received blocks, src/daemon/tracking/fetch_blocks.rs:77,91-103):
 * the arena is [d_arena, d_arena + arena_bytes), and block b is out of range
 * when d_off[b] + d_len[b] wraps around 2^64 or passes arena_bytes.  An
 * out-of-range block is not read (no kernel touches memory outside the
 * arena); its digest is 32 zero bytes and *d_nrange (device u32, may be
 * NULL) = the number of such blocks.  The other blocks' digests are exactly
 * cir_hash_blocks_dev_ht's.  Asynchronous on `stream` like the other *_dev
 * calls: the caller reads *d_nrange after its own synchronisation and treats
 * a non-zero count as CIR_EINVAL for those blocks.  Costs one extra pass
 * over the descriptors (12 B read, 5 B written per block) and, with a
 * context, a device scratch of ~5 B per block kept for the next call. */
int cir_hash_blocks_dev_bounded(cir_ctx* ctx, int hash_type, const void* d_arena,
                                uint64_t arena_bytes, const uint64_t* d_off, const uint32_t* d_len,
                                size_t nblk, uint8_t* d_out, uint32_t* d_nrange, void* stream);

/* Host-memory batch (same meaning as cir_hash_blocks_dev, host pointers);
 * staged through pinned buffers, split across the context's devices. */
int cir_hash_blocks(cir_ctx* ctx, const uint8_t* h_arena, const uint64_t* off,
                    const uint32_t* len, size_t nblk, uint8_t* h_out);

/* cir_hash_blocks_ht over host descriptors the caller cannot vouch for: the
 * arena is [h_arena, h_arena + arena_bytes); block b is out of range when
 * off[b] + len[b] wraps around 2^64 or passes arena_bytes.  Such a block is
 * never read; its digest is 32 zero bytes and *nrange_out (may be NULL) =
 * their number.  The other digests are exactly cir_hash_blocks_ht's; with
 * every block in range nothing is copied (one pass over the descriptors). */
int cir_hash_blocks_bounded(cir_ctx* ctx, int hash_type, const uint8_t* h_arena,
                            uint64_t arena_bytes, const uint64_t* off, const uint32_t* len,
                            size_t nblk, uint8_t* h_out, size_t* nrange_out);

/* dir_signature::v1::Hashes::hash_file(HashType::blake2b_256(), block_size,
 * reader)  (external; call sites src/blocks.rs:193,
 * src/cluster/download.rs:257).  Reads fd from its current offset to EOF.
 * *hashes_out = ceil(size / block_size) x 32 bytes (NULL when size == 0). */
int cir_hash_file(cir_ctx* ctx, int fd, uint64_t block_size, uint64_t* size_out,
                  uint8_t** hashes_out, size_t* nhash_out);

/* Hashes::hash_file over an in-memory reader (register_memory_blocks,
 * src/blocks.rs:187-204). */
int cir_hash_memory(cir_ctx* ctx, const uint8_t* data, uint64_t size, uint64_t block_size,
                    uint8_t** hashes_out, size_t* nhash_out);

/* ---- other hash types (dir-signature HashType) ------------------------ */

/* The entry points above with an explicit HashType (enum cir_hash_type):
 * Hashes::hash_file(hash_type, ...) is generic over the index's hash type
 * (src/cluster/download.rs:257 passes self.hash_type). */
int cir_sha512_256(const uint8_t* p, size_t n, uint8_t out[CIR_DIGEST_BYTES]);
int cir_hash_blocks_dev_ht(cir_ctx* ctx, int hash_type, const void* d_arena,
                           const uint64_t* d_off, const uint32_t* d_len, size_t nblk,
                           uint8_t* d_out, void* stream);
int cir_hash_blocks_ht(cir_ctx* ctx, int hash_type, const uint8_t* h_arena, const uint64_t* off,
                       const uint32_t* len, size_t nblk, uint8_t* h_out);
int cir_hash_file_ht(cir_ctx* ctx, int hash_type, int fd, uint64_t block_size,
                     uint64_t* size_out, uint8_t** hashes_out, size_t* nhash_out);
int cir_hash_memory_ht(cir_ctx* ctx, int hash_type, const uint8_t* data, uint64_t size,
                       uint64_t block_size, uint8_t** hashes_out, size_t* nhash_out);

/* ---- verification (the daemon side of the same hash) ------------------ */

/* FetchBlock::poll's `BlockHash::hash_bytes(&data.data) == blk.hash`
 * (src/daemon/tracking/fetch_blocks.rs:77) over a device-resident batch of
 * received blocks: the blocks are hashed (as cir_hash_blocks_dev_ht) into
 * d_digests (32 x nblk bytes of scratch) and compared with d_expected on the
 * same stream.  d_ok[b] = 1 when block b matches, 0 when it does not (the
 * reference then retries the block elsewhere, :91-103); *d_nbad (device
 * u32) = number of mismatches.  d_ok / d_nbad may be NULL.  d_expected and
 * d_digests must be 16-byte aligned. */
int cir_verify_blocks_dev(cir_ctx* ctx, int hash_type, const void* d_arena, const uint64_t* d_off,
                          const uint32_t* d_len, size_t nblk, const uint8_t* d_expected,
                          uint8_t* d_digests, uint8_t* d_ok, uint32_t* d_nbad, void* stream);

/* cir_verify_blocks_dev over untrusted descriptors, as
 * cir_hash_blocks_dev_bounded checks them: an out-of-range block (d_off[b] +
 * d_len[b] wraps or passes arena_bytes) is never read and counts as a
 * mismatch -- d_ok[b] = 0, included in *d_nbad -- so the caller re-fetches
 * it as it would a corrupted block (fetch_blocks.rs:91-103); its
 * d_digests entry is 32 zero bytes. */
int cir_verify_blocks_dev_bounded(cir_ctx* ctx, int hash_type, const void* d_arena,
                                  uint64_t arena_bytes, const uint64_t* d_off,
                                  const uint32_t* d_len, size_t nblk, const uint8_t* d_expected,
                                  uint8_t* d_digests, uint8_t* d_ok, uint32_t* d_nbad,
                                  void* stream);

/* Host-memory batch of the same check; ok_out (nblk bytes) may be NULL. */
int cir_verify_blocks(cir_ctx* ctx, int hash_type, const uint8_t* h_arena, const uint64_t* off,
                      const uint32_t* len, size_t nblk, const uint8_t* expected, uint8_t* ok_out,
                      size_t* nbad_out);

/* cir_verify_blocks over untrusted host descriptors (checked as
 * cir_hash_blocks_bounded checks them): an out-of-range block is never read
 * and is a mismatch (ok_out[b] = 0, counted in *nbad_out). */
int cir_verify_blocks_bounded(cir_ctx* ctx, int hash_type, const uint8_t* h_arena,
                              uint64_t arena_bytes, const uint64_t* off, const uint32_t* len,
                              size_t nblk, const uint8_t* expected, uint8_t* ok_out,
                              size_t* nbad_out);

/* The same check one block at a time, asynchronously, for a caller that
 * receives blocks one by one (FetchBlock::poll, fetch_blocks.rs:77):
 * cir_verify_submit copies the block (once, into the arena of the batch
 * being formed) with its expected digest and returns a ticket; a worker
 * thread of the context verifies each batch as one host batch once it is full
 * or a short window after its first block (default 200 us, at most 4096
 * blocks, one hash type per batch).  cir_verify_poll: *state = 0 pending,
 * 1 match, 2 mismatch (the outcome is consumed when reported).
 * cir_verify_wait blocks: *ok = 1 match, 0 mismatch.  A failed batch returns
 * its error for each of its tickets.  An unknown, consumed, forgotten or
 * expired ticket is CIR_ENOTFOUND.  cir_verify_window sets the window
 * (microseconds) and the batch cap.
 *
 * Bounds (cir_verify_limits; 0 = the default):
 *   max_bytes    block bytes accepted and not yet verified (default 256 MiB).
 *                It bounds admission only: a batch's arena holds min(half of
 *                it, 128 MiB), so a large bound allocates nothing up front.  A submit that
 *                would pass it waits until the worker has verified enough,
 *                or with flags = CIR_VERIFY_NONBLOCK returns CIR_EAGAIN (the
 *                block is not taken: retry later or elsewhere).  A block
 *                larger than max_bytes is taken once nothing else is held.
 *   max_results  finished outcomes held for tickets not yet polled, waited
 *                or forgotten (default 2^20); beyond it the oldest tickets'
 *                outcomes are dropped (they become CIR_ENOTFOUND, counted as
 *                expired).
 * cir_verify_forget drops a ticket the caller no longer wants (a block the
 * reference would re-fetch elsewhere, :91-103): a pending one is still
 * hashed with its batch but its outcome is never held; a finished one's
 * outcome is released.
 * cir_verify_stats: out[0] bytes held (accepted, not yet verified), [1] the
 * peak of [0], [2] pending tickets, [3] outcomes held, [4] outcomes
 * expired, [5] tickets forgotten, [6] submits refused with CIR_EAGAIN,
 * [7] batches verified. */
#define CIR_VERIFY_NONBLOCK 1
#define CIR_VERIFY_STATS_FIELDS 8
int cir_verify_submit(cir_ctx* ctx, int hash_type, const uint8_t* data, size_t n,
                      const uint8_t expected[CIR_DIGEST_BYTES], uint64_t* ticket);
int cir_verify_poll(cir_ctx* ctx, uint64_t ticket, int* state);
int cir_verify_wait(cir_ctx* ctx, uint64_t ticket, int* ok);
int cir_verify_forget(cir_ctx* ctx, uint64_t ticket);
int cir_verify_window(cir_ctx* ctx, uint32_t window_us, uint32_t max_batch);
int cir_verify_limits(cir_ctx* ctx, uint64_t max_bytes, uint64_t max_results, int flags);
int cir_verify_stats(cir_ctx* ctx, uint64_t out[CIR_VERIFY_STATS_FIELDS]);

/* Hashes::check_file(&mut file) at image commit (src/daemon/disk/commit.rs:
 * 104; false -> Error::Checksum, :110): re-hash fd from its current offset to
 * EOF in block_size blocks; *ok_out = 1 iff the file has exactly nhash
 * blocks and every digest equals expected[32 i .. 32 i + 32]. */
int cir_check_file(cir_ctx* ctx, int hash_type, int fd, uint64_t block_size,
                   const uint8_t* expected, size_t nhash, int* ok_out);

/* ---- index (DIRSIGNATURE.v1) ----------------------------------------- */

/* dir_signature::v1::scan(&ScannerConfig, &mut Vec<u8>)
 * (src/client/sync/uploads.rs:49-59; examples/custom_uploader.rs:59-65):
 * ScannerConfig{threads, hash, add_dir(dirs[i], prefixes[i])}.  threads =
 * host reader threads (gopt.threads, default 4, src/client/global_options.rs:13;
 * 0 = auto_threads).  *index_out receives the index bytes. */
int cir_scan_v1(cir_ctx* ctx, const char* const* dirs, const char* const* prefixes, size_t ndirs,
                uint64_t block_size, int hash_type, uint32_t threads, uint8_t** index_out,
                size_t* len_out);

/* The same scan writing the index out as it goes, as v1::scan writes into
 * the caller's `&mut Vec<u8>` / io::Write (src/client/sync/uploads.rs:55-57):
 * write(user, data, n) receives the index bytes in order -- the header line
 * first, then each stretch of the body as the batches complete files, the
 * footer line last -- from library threads, one call at a time.  The
 * library keeps only the unwritten tail (no whole-index buffer, no copy
 * after the scan).  A non-zero return from write stops the scan with
 * CIR_EIO (the reference's io::Error from the writer); on any error the
 * writer may have received part of an index.  *len_out (may be NULL) = the
 * bytes written. */
typedef int (*cir_write_fn)(void* user, const uint8_t* data, size_t n);
int cir_scan_v1_write(cir_ctx* ctx, const char* const* dirs, const char* const* prefixes,
                      size_t ndirs, uint64_t block_size, int hash_type, uint32_t threads,
                      cir_write_fn write, void* user, size_t* len_out);

/* dir_signature::get_hash via InMemoryIndexes::register_index
 * (src/index.rs:98-105): the image id printed on the index's last line.
 * id_out must hold 64 bytes; *id_len = decoded length (32 for v1 hashes). */
int cir_index_get_hash(const uint8_t* index, size_t len, uint8_t* id_out, size_t* id_len);

/* RawIndex::into_mut + MutableIndex::to_raw_data (src/cluster/download.rs:
 * 171-188, 266-319): parse, rebuild the directory tree and re-emit it in the
 * reference's order (files and links by name, then subdirectories; empty
 * directories dropped) with the footer recomputed in the index's hash type
 * where cir_set_footer_mode says: CIR_FOOTER_HOST (the default, as in
 * cir_scan_v1) hashes it on the calling thread, blake2b/256 and sha512/256
 * alike; CIR_FOOTER_GPU as one descriptor on the GPU. */
int cir_index_rewrite(cir_ctx* ctx, const uint8_t* in, size_t len, uint8_t** out, size_t* out_len);

/* ---- consumers of the index (host bookkeeping) ------------------------ */

/* InMemoryIndexes (src/index.rs:53-124): ImageId -> index bytes. */
typedef struct cir_indexes cir_indexes;
cir_indexes* cir_indexes_new(void); /* NULL if out of memory */
void cir_indexes_free(cir_indexes* h);
/* register_index (src/index.rs:98-105); id_out holds 64 bytes. */
int cir_indexes_register(cir_indexes* h, const uint8_t* data, size_t len, uint8_t* id_out,
                         size_t* id_len);
/* GetIndex::read_index (src/index.rs:106-123); CIR_ENOTFOUND if absent. */
int cir_indexes_read(cir_indexes* h, const uint8_t* id, size_t id_len, uint8_t** data_out,
                     size_t* len_out);

/* ThreadedBlockReader (src/blocks.rs:85-240): BlockHash -> block bytes. */
typedef struct cir_blocks cir_blocks;
cir_blocks* cir_blocks_new(void); /* NULL if out of memory */
void cir_blocks_free(cir_blocks* h);
size_t cir_blocks_len(cir_blocks* h);
/* register_dir (src/blocks.rs:145-183): CIR_EPARSE / CIR_EHASHSIZE. */
int cir_blocks_register_dir(cir_blocks* h, const char* dir, const uint8_t* index, size_t len);
/* register_memory_blocks(HashType::blake2b_256(), ..) (src/blocks.rs:187-204),
 * hashed on the GPU. */
int cir_blocks_register_memory(cir_ctx* ctx, cir_blocks* h, const uint8_t* data, size_t len,
                               uint64_t block_size);
/* register_memory_blocks(hash_type, block_size, data) with the index's own
 * hash type (put-file, src/client/put_file/network.rs:56). */
int cir_blocks_register_memory_ht(cir_ctx* ctx, cir_blocks* h, int hash_type, const uint8_t* data,
                                  size_t len, uint64_t block_size);
/* GetBlock::read_block (src/blocks.rs:207-240); CIR_ENOTFOUND if absent. */
int cir_blocks_read(cir_blocks* h, const uint8_t hash[CIR_DIGEST_BYTES], uint8_t** data_out,
                    size_t* len_out);

/* ---- test data -------------------------------------------------------- */

/* Fill d_ptr with splitmix64 words (bench/tests only).  block_bytes == 0:
 * word k = splitmix64 output k of `seed`; otherwise block i (block_bytes
 * each, a multiple of 8) is its own stream seeded seed ^ (first_block + i). */
int cir_fill_splitmix64_dev(void* d_ptr, uint64_t nbytes, uint64_t seed, uint64_t block_bytes,
                            uint64_t first_block, void* stream);

/* ---- diagnostics (not part of the reference interface) ---------------- */

/* One launch of a uniform-block kernel variant, for A/B measurement:
 * loader 0 = LDS-DMA coalesced lines (the production loader), 1 = per-lane
 * direct loads.  nblk % 256 == 0, block_size % 128 == 0, d_data 16-B aligned. */
int cir_debug_hash_uniform_dev(int loader, const void* d_data, uint64_t block_size, uint64_t nblk,
                               uint8_t* d_out, void* stream);

/* nlanes (% 256 == 0) independent chains of `lines` BLAKE2b compressions on
 * register-resident messages, digest per lane -> d_out + 32 lane: the same
 * compression count as hashing nlanes blocks of 128 x lines bytes, with no
 * memory traffic.  bench.py times it as the measured VALU ceiling. */
int cir_debug_compress_only_dev(uint64_t nlanes, uint32_t lines, uint8_t* d_out, void* stream);

/* Per-part kernel timing of the ordered descriptor batches of ctx's first
 * device (cir_hash_blocks_dev with a context): enable != 0 starts recording
 * HIP events around the ordering, the quad part and the lane part of each
 * batch (at most 256 batches per enable; enabling again restarts), 0 stops.
 * cir_debug_desc_times waits for the recorded events and returns
 * out[0] = batches, out[1..3] = summed ordering / quad-part / lane-part
 * milliseconds, out[4] = summed ordering start -> last part end. */
int cir_debug_desc_timing(cir_ctx* ctx, int enable);
int cir_debug_desc_times(cir_ctx* ctx, double out[5]);

/* Where cir_scan_v1 and cir_index_rewrite hash an index's footer (the
 * ImageId, H(every byte after the header line), src/index.rs:98-105): one
 * serial chain over the index text, ~65 B per 32 KiB block.  CIR_FOOTER_HOST
 * (the default): a host thread hashes the text as the scan emits it
 * (blake2b/256 and sha512/256).  CIR_FOOTER_GPU: the resumable single-chain
 * kernel (quad mode) on device 0's chain stream for blake2b/256, one lane at
 * the end for sha512/256.  Block digests are always computed on the GPU. */
enum cir_footer_mode { CIR_FOOTER_HOST = 0, CIR_FOOTER_GPU = 1 };
int cir_set_footer_mode(cir_ctx* ctx, int mode);

/* Staged-scan timing of ctx (cir_scan_v1): enable != 0 clears the record and
 * starts recording, 0 stops.  While on, every staged batch adds one row of
 * CIR_SCAN_BATCH_FIELDS doubles:
 *   [0] device index in ctx  [1] bytes  [2] blocks
 *   [3] host wait for the slot (ms)
 *   [4] reads start  [5] reads end            (ms since the scan started)
 *   [6] H2D start    [7] H2D end              (HIP events on the copy stream)
 *   [8] hash start   [9] digests back on host (HIP events, compute stream)
 * and every scan sets CIR_SCAN_PHASE_FIELDS doubles:
 *   [0] walk ms  [1] hash loop ms  [2] last emit ms
 *   [3] footer tail ms (hash loop end -> footer digest)  [4] output ms
 *   [5] footer busy ms (host thread hashing, or summed chain-kernel time)
 *   [6] footer mode  [7] batches  [8] index bytes  [9] footer feeds.
 * cir_debug_scan_batches copies at most max_rows rows and sets *nrows to the
 * number recorded. */
#define CIR_SCAN_BATCH_FIELDS 10
#define CIR_SCAN_PHASE_FIELDS 10
int cir_debug_scan_timing(cir_ctx* ctx, int enable);
int cir_debug_scan_batches(cir_ctx* ctx, double* rows, size_t max_rows, size_t* nrows);
int cir_debug_scan_phases(cir_ctx* ctx, double out[CIR_SCAN_PHASE_FIELDS]);

/* The footer's host BLAKE2b-256 / SHA-512/256 fed in `piece`-byte updates
 * (0 = one update): no device involved; the CPU tests check them against
 * the oracle. */
int cir_debug_host_blake2b256(const uint8_t* p, size_t n, size_t piece,
                              uint8_t out[CIR_DIGEST_BYTES]);
int cir_debug_host_sha512_256(const uint8_t* p, size_t n, size_t piece,
                              uint8_t out[CIR_DIGEST_BYTES]);

/* Identity of HIP device `device` as its driver and its own counters see it
 * (the multi-GPU bench puts every rank's into its line): the PCI bus id
 * (hipDeviceGetPCIBusId, into pci_bus_id, len >= 13), the UUID
 * (hipDeviceGetUuid), and one wave's reads of the device's wall clock and
 * shader clock counters ~100 us apart: clocks[0], [1] = wall clock before /
 * after, [2], [3] = shader clock counter before / after, [4] = the wall
 * clock's rate in kHz.  Synchronous; allocates and frees 32 bytes. */
int cir_debug_device_identity(int device, char* pci_bus_id, size_t len, uint8_t uuid[16],
                              uint64_t clocks[5]);

/* How many whole blocks of a file of nfull x block_size bytes (plus any short
 * last block) cir_hash_chunks_dev with a context relays on the calling
 * thread's current device (0: none).  Relayed blocks run in quad mode as
 * segmented chains beside k whole lane (or quad) waves per SIMD. */
uint64_t cir_debug_relay_blocks(uint64_t nfull, uint64_t block_size);

#ifdef __cplusplus
}
#endif

#endif /* CIRUELA_BLOCKHASH_H */
