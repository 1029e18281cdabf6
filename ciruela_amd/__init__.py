"""ciruela_amd — MI355X-native block-indexing path of tailhook/ciruela.

Python mirror of the reference's public interface for the indexing path,
over the C ABI in include/ciruela_blockhash.h (libciruela_amd.so).  Names,
argument meaning and error behaviour follow the reference:

=============================  ==============================================
this module                     reference (tailhook/ciruela v0.6.12)
=============================  ==============================================
BlockHash                       ciruela::blocks::BlockHash (src/block_id.rs:19)
BlockHash.hash_bytes            BlockHash::hash_bytes (src/block_id.rs:37-43)
ImageId                         ciruela::index::ImageId (src/id.rs:142)
HashType                        dir_signature::HashType (external 0.2.9)
Hashes.hash_file                dir_signature::v1::Hashes::hash_file
ScannerConfig, v1.scan          dir_signature::{ScannerConfig, v1::scan}
                                (src/client/sync/uploads.rs:49-59)
get_hash                        dir_signature::get_hash (src/index.rs:99)
InMemoryIndexes                 ciruela::index::InMemoryIndexes (src/index.rs:53)
ThreadedBlockReader             ciruela::blocks::ThreadedBlockReader
                                (src/blocks.rs:85)
Context.verify_blocks[_dev]     FetchBlock::poll's `hash_bytes(..) == blk.hash`
                                (src/daemon/tracking/fetch_blocks.rs:77), batched
Context.verify_submit / poll /  the same check per block, batched by the library,
  wait / forget / limits        bounded (CIR_EAGAIN backpressure, forgotten tickets)
Context.check_file              Hashes::check_file (src/daemon/disk/commit.rs:104)
=============================  ==============================================

All hashing runs on gfx950 through the library; there is no CPU fallback.
"""
import ctypes
import os
import threading

from . import _native as _n
from ._native import CiruelaError, NoDevice  # noqa: F401

__all__ = [
    "BlockHash", "ImageId", "HashType", "Hashes", "ScannerConfig", "v1", "get_hash",
    "InMemoryIndexes", "ThreadedBlockReader", "BlockHint", "Context", "default_context",
    "IndexError_", "DirError", "ReadError", "CiruelaError", "NoDevice", "sha512_256",
]

DEFAULT_BLOCK_SIZE = 32768


def _buf(data):
    """(pointer, keepalive) for any contiguous buffer (bytes, bytearray,
    memoryview, numpy array, mmap), without copying it."""
    import numpy as np
    try:
        mv = memoryview(data)
    except TypeError:
        raise TypeError("expected a bytes-like object, got %r" % type(data)) from None
    if not mv.c_contiguous:
        raise ValueError("buffer must be C-contiguous")
    mv = mv.cast("B")
    if mv.nbytes == 0:
        return None, b""
    arr = np.frombuffer(mv, dtype=np.uint8)
    return ctypes.c_void_p(arr.ctypes.data), (arr, mv)


class Context:
    """A cir_ctx: the devices the host-memory entry points run on."""

    def __init__(self, device_mask=0, staging_bytes=0, max_devices=0, one_shot=False):
        """max_devices: open at most that many of the masked devices (0 = all;
        cir_init_n).  devices_for_bytes() gives the count an input can use.
        one_shot: CIR_INIT_ONE_SHOT -- one stream and one staging slot per
        device, for one short job (the CLI's small inputs)."""
        h = ctypes.c_void_p()
        _n.check(_n.lib.cir_init_n(ctypes.byref(h), device_mask, staging_bytes, max_devices,
                                   _n.CIR_INIT_ONE_SHOT if one_shot else 0))
        self._h = h

    @staticmethod
    def devices_for_bytes(work_bytes, staging_bytes=0, visible=None):
        """cir_devices_for_bytes: ceil(work / (2 x staging)) capped at the
        visible count (no HIP call when `visible` is given)."""
        if visible is None:
            visible = _n.lib.cir_device_count()
        return _n.lib.cir_devices_for_bytes(work_bytes, staging_bytes, visible)

    @property
    def handle(self):
        return self._h

    def devices(self):
        ids = (ctypes.c_int * 64)()
        n = _n.lib.cir_ctx_devices(self._h, ids, 64)
        return list(ids[:n])

    def close(self):
        if self._h:
            _n.lib.cir_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    # ---- device-resident entry points (pointers are device addresses) ----
    def hash_chunks_dev(self, d_data, nbytes, block_size, d_out, stream=0):
        _n.check(_n.lib.cir_hash_chunks_dev(self._h, d_data, nbytes, block_size, d_out, stream))

    def hash_blocks_dev(self, d_arena, d_off, d_len, nblk, d_out, stream=0, hash_type=None):
        ht = (hash_type or HashType.blake2b_256()).code
        _n.check(_n.lib.cir_hash_blocks_dev_ht(self._h, ht, d_arena, d_off, d_len, nblk, d_out,
                                               stream))

    def hash_blocks_dev_bounded(self, d_arena, arena_bytes, d_off, d_len, nblk, d_out,
                                d_nrange=0, stream=0, hash_type=None):
        """hash_blocks_dev over untrusted descriptors: a block past
        arena_bytes is not read, its digest is zeros, *d_nrange counts them."""
        ht = (hash_type or HashType.blake2b_256()).code
        _n.check(_n.lib.cir_hash_blocks_dev_bounded(self._h, ht, d_arena, arena_bytes, d_off,
                                                    d_len, nblk, d_out, d_nrange, stream))

    # ---- host-memory entry points ----------------------------------------
    def hash_blocks(self, arena, offsets, lengths, hash_type=None):
        """Digests (n x 32 bytes) of arena[off[i] : off[i] + len[i]]."""
        ht = (hash_type or HashType.blake2b_256()).code
        n = len(offsets)
        if len(lengths) != n:
            raise ValueError("offsets and lengths differ in length")
        for o, ln in zip(offsets, lengths):
            if o < 0 or ln < 0 or o + ln > len(arena):
                raise ValueError("block outside the arena")
            if ln > 0xFFFFFFFF:
                raise ValueError("block longer than 2^32 - 1 bytes")
        out = ctypes.create_string_buffer(32 * max(n, 1))
        if n == 0:
            return b""
        offs = (ctypes.c_uint64 * n)(*offsets)
        lens = (ctypes.c_uint32 * n)(*lengths)
        ptr, keep = _buf(arena) if len(arena) else (ctypes.c_void_p(0), None)
        if ptr is None:
            one = ctypes.create_string_buffer(1)
            ptr, keep = ctypes.cast(one, ctypes.c_void_p), one
        _n.check(_n.lib.cir_hash_blocks_ht(self._h, ht, ptr, offs, lens, n, out))
        del keep
        return out.raw[:32 * n]

    def hash_file(self, fd, block_size, hash_type=None):
        ht = (hash_type or HashType.blake2b_256()).code
        size = ctypes.c_uint64()
        hp = ctypes.c_void_p()
        nh = ctypes.c_size_t()
        _n.check(_n.lib.cir_hash_file_ht(self._h, ht, fd, block_size, ctypes.byref(size),
                                         ctypes.byref(hp), ctypes.byref(nh)))
        return size.value, _n.take_buffer(hp.value, 32 * nh.value)

    def hash_memory(self, data, block_size, hash_type=None):
        ht = (hash_type or HashType.blake2b_256()).code
        ptr, keep = _buf(data)
        hp = ctypes.c_void_p()
        nh = ctypes.c_size_t()
        _n.check(_n.lib.cir_hash_memory_ht(self._h, ht, ptr, len(data), block_size,
                                           ctypes.byref(hp), ctypes.byref(nh)))
        del keep
        return _n.take_buffer(hp.value, 32 * nh.value)

    # ---- verification (daemon side, fetch_blocks.rs:77 / commit.rs:104) --
    def verify_blocks(self, arena, offsets, lengths, expected, hash_type=None):
        """Per block: does H(arena[off:off+len]) equal expected[32 i:32 i+32]?"""
        ht = (hash_type or HashType.blake2b_256()).code
        n = len(offsets)
        if len(lengths) != n or len(expected) != 32 * n:
            raise ValueError("offsets, lengths and expected digests disagree in length")
        for o, ln in zip(offsets, lengths):
            if o < 0 or ln < 0 or o + ln > len(arena):
                raise ValueError("block outside the arena")
            if ln > 0xFFFFFFFF:
                raise ValueError("block longer than 2^32 - 1 bytes")
        if n == 0:
            return []
        offs = (ctypes.c_uint64 * n)(*offsets)
        lens = (ctypes.c_uint32 * n)(*lengths)
        ptr, keep = _buf(arena) if len(arena) else (None, None)
        if ptr is None:
            one = ctypes.create_string_buffer(1)
            ptr, keep = ctypes.cast(one, ctypes.c_void_p), one
        exp = ctypes.create_string_buffer(bytes(expected), 32 * n)
        ok = ctypes.create_string_buffer(n)
        nbad = ctypes.c_size_t()
        _n.check(_n.lib.cir_verify_blocks(self._h, ht, ptr, offs, lens, n, exp, ok,
                                          ctypes.byref(nbad)))
        del keep
        return [b == 1 for b in ok.raw]

    def verify_blocks_bounded(self, arena, offsets, lengths, expected, hash_type=None):
        """verify_blocks for descriptors from untrusted data: nothing is
        checked here; a block outside the arena is not read and is False."""
        ht = (hash_type or HashType.blake2b_256()).code
        n = len(offsets)
        if len(lengths) != n or len(expected) != 32 * n:
            raise ValueError("offsets, lengths and expected digests disagree in length")
        if n == 0:
            return []
        offs = (ctypes.c_uint64 * n)(*offsets)
        lens = (ctypes.c_uint32 * n)(*lengths)
        ptr, keep = _buf(arena) if len(arena) else (None, None)
        exp = ctypes.create_string_buffer(bytes(expected), 32 * n)
        ok = ctypes.create_string_buffer(n)
        nbad = ctypes.c_size_t()
        _n.check(_n.lib.cir_verify_blocks_bounded(self._h, ht, ptr, len(arena), offs, lens, n, exp,
                                                  ok, ctypes.byref(nbad)))
        del keep
        return [b == 1 for b in ok.raw]

    def verify_blocks_dev(self, d_arena, d_off, d_len, nblk, d_expected, d_digests, d_ok=0,
                          d_nbad=0, stream=0, hash_type=None):
        ht = (hash_type or HashType.blake2b_256()).code
        _n.check(_n.lib.cir_verify_blocks_dev(self._h, ht, d_arena, d_off, d_len, nblk,
                                              d_expected, d_digests, d_ok, d_nbad, stream))

    def verify_blocks_dev_bounded(self, d_arena, arena_bytes, d_off, d_len, nblk, d_expected,
                                  d_digests, d_ok=0, d_nbad=0, stream=0, hash_type=None):
        """verify_blocks_dev over untrusted descriptors: a block past
        arena_bytes is not read and counts as a mismatch."""
        ht = (hash_type or HashType.blake2b_256()).code
        _n.check(_n.lib.cir_verify_blocks_dev_bounded(self._h, ht, d_arena, arena_bytes, d_off,
                                                      d_len, nblk, d_expected, d_digests, d_ok,
                                                      d_nbad, stream))

    # ---- asynchronous per-block verify (FetchBlock::poll, fetch_blocks.rs:77)
    def verify_submit(self, data, expected, hash_type=None):
        """Queue one block with its expected digest; returns a ticket."""
        ht = (hash_type or HashType.blake2b_256()).code
        if len(expected) != 32:
            raise ValueError("expected digest must be 32 bytes")
        ptr, keep = _buf(data) if len(data) else (ctypes.c_void_p(0), None)
        exp = ctypes.create_string_buffer(bytes(expected), 32)
        t = ctypes.c_uint64()
        _n.check(_n.lib.cir_verify_submit(self._h, ht, ptr, len(data), exp, ctypes.byref(t)))
        del keep
        return t.value

    def verify_poll(self, ticket):
        """None while pending, else True (match) / False (mismatch)."""
        st = ctypes.c_int()
        _n.check(_n.lib.cir_verify_poll(self._h, ticket, ctypes.byref(st)))
        return None if st.value == 0 else st.value == 1

    def verify_wait(self, ticket):
        ok = ctypes.c_int()
        _n.check(_n.lib.cir_verify_wait(self._h, ticket, ctypes.byref(ok)))
        return ok.value == 1

    def verify_window(self, window_us, max_batch=4096):
        _n.check(_n.lib.cir_verify_window(self._h, window_us, max_batch))

    def verify_forget(self, ticket):
        """Drop a ticket (pending or finished) whose outcome is not wanted."""
        _n.check(_n.lib.cir_verify_forget(self._h, ticket))

    def verify_limits(self, max_bytes=0, max_results=0, nonblocking=False):
        """Bound the queue (block bytes accepted, not yet verified) and the
        outcomes held; 0 = the library default.  nonblocking: a submit that
        would pass max_bytes raises CiruelaError(CIR_EAGAIN) instead of
        waiting."""
        _n.check(_n.lib.cir_verify_limits(self._h, max_bytes, max_results,
                                          _n.CIR_VERIFY_NONBLOCK if nonblocking else 0))

    VERIFY_STATS_FIELDS = ("bytes_held", "peak_bytes_held", "pending", "outcomes_held",
                           "expired", "forgotten", "refused", "batches")

    def verify_stats(self):
        out = (ctypes.c_uint64 * _n.CIR_VERIFY_STATS_FIELDS)()
        _n.check(_n.lib.cir_verify_stats(self._h, out))
        return dict(zip(self.VERIFY_STATS_FIELDS, list(out)))

    def check_file(self, fd, block_size, expected, hash_type=None):
        ht = (hash_type or HashType.blake2b_256()).code
        if len(expected) % 32:
            raise ValueError("expected digests must be 32 bytes each")
        n = len(expected) // 32
        exp = ctypes.create_string_buffer(bytes(expected), max(len(expected), 1))
        ok = ctypes.c_int()
        _n.check(_n.lib.cir_check_file(self._h, ht, fd, block_size, exp, n, ctypes.byref(ok)))
        return ok.value == 1

    def scan(self, config):
        dirs = [os.fsencode(d) for d, _ in config._dirs]
        pres = [p.encode() for _, p in config._dirs]
        cd = (ctypes.c_char_p * len(dirs))(*dirs)
        cp = (ctypes.c_char_p * len(pres))(*pres)
        out = ctypes.c_void_p()
        ln = ctypes.c_size_t()
        _n.check(_n.lib.cir_scan_v1(self._h, cd, cp, len(dirs), config._block_size,
                                    config._hash.code, config._threads, ctypes.byref(out),
                                    ctypes.byref(ln)))
        return _n.take_buffer(out.value, ln.value)

    def scan_into(self, config, out):
        """cir_scan_v1_write: append the index to `out` (a bytearray) while
        the scan emits it -- header, then each stretch of the body as files
        complete, the footer line last -- as v1::scan writes into the
        caller's Vec (src/client/sync/uploads.rs:55-57).  Returns the number
        of bytes appended.  An exception raised while appending stops the
        scan and is re-raised here."""
        dirs = [os.fsencode(d) for d, _ in config._dirs]
        pres = [p.encode() for _, p in config._dirs]
        cd = (ctypes.c_char_p * len(dirs))(*dirs)
        cp = (ctypes.c_char_p * len(pres))(*pres)
        failed = []

        def write(_user, data, n):
            try:
                out.extend((ctypes.c_char * n).from_address(data))
                return 0
            except BaseException as e:  # noqa: BLE001 - re-raised after the call
                failed.append(e)
                return 1
        cb = _n.WRITE_FN(write)
        ln = ctypes.c_size_t()
        rc = _n.lib.cir_scan_v1_write(self._h, cd, cp, len(dirs), config._block_size,
                                      config._hash.code, config._threads, cb, None,
                                      ctypes.byref(ln))
        if failed:
            raise failed[0]
        _n.check(rc)
        return ln.value

    # ---- footer placement and scan timing (diagnostics) -------------------
    FOOTER_HOST, FOOTER_GPU = 0, 1
    SCAN_BATCH_FIELDS = ("device", "bytes", "blocks", "wait_ms", "read_start_ms", "read_end_ms",
                         "h2d_start_ms", "h2d_end_ms", "hash_start_ms", "done_ms")
    SCAN_PHASE_FIELDS = ("walk_ms", "hash_loop_ms", "last_emit_ms", "footer_tail_ms",
                         "output_ms", "footer_busy_ms", "footer_mode", "batches", "index_bytes",
                         "footer_feeds")

    def set_footer_mode(self, mode):
        """Where cir_scan_v1 and cir_index_rewrite hash an index's footer, in
        either hash type: FOOTER_HOST (a host thread, the default) or
        FOOTER_GPU (blake2b/256: the chain kernel beside the scan;
        sha512/256: one lane at the end)."""
        _n.check(_n.lib.cir_set_footer_mode(self._h, mode))

    def scan_timing(self, enable=True):
        _n.check(_n.lib.cir_debug_scan_timing(self._h, 1 if enable else 0))

    def scan_batches(self):
        """One dict per staged batch of the scans since scan_timing(True)."""
        n = ctypes.c_size_t()
        _n.check(_n.lib.cir_debug_scan_batches(self._h, None, 0, ctypes.byref(n)))
        k = len(self.SCAN_BATCH_FIELDS)
        rows = (ctypes.c_double * (k * max(1, n.value)))()
        _n.check(_n.lib.cir_debug_scan_batches(self._h, rows, n.value, ctypes.byref(n)))
        return [dict(zip(self.SCAN_BATCH_FIELDS, rows[i * k:(i + 1) * k]))
                for i in range(n.value)]

    def scan_phases(self):
        """The phase record of the last scan since scan_timing(True)."""
        out = (ctypes.c_double * len(self.SCAN_PHASE_FIELDS))()
        _n.check(_n.lib.cir_debug_scan_phases(self._h, out))
        return dict(zip(self.SCAN_PHASE_FIELDS, list(out)))

    def index_rewrite(self, data):
        ptr, keep = _buf(data)
        out = ctypes.c_void_p()
        ln = ctypes.c_size_t()
        _n.check(_n.lib.cir_index_rewrite(self._h, ptr, len(data), ctypes.byref(out),
                                          ctypes.byref(ln)))
        del keep
        return _n.take_buffer(out.value, ln.value)


_default = None
_default_lock = threading.Lock()


def default_context():
    """Process-wide context on every visible device (created on first use)."""
    global _default
    with _default_lock:
        if _default is None:
            _default = Context()
        return _default


def _hex(b):
    return b.hex()


class BlockHash:
    """32-byte block id (src/block_id.rs:19); displays as lowercase hex."""

    __slots__ = ("_b",)

    def __init__(self, raw):
        if len(raw) != 32:
            raise ValueError("BlockHash is 32 bytes")
        self._b = bytes(raw)

    @staticmethod
    def from_bytes(raw):
        """Some(BlockHash) for 32 bytes, None otherwise (src/block_id.rs:28-35)."""
        return BlockHash(raw) if len(raw) == 32 else None

    @staticmethod
    def hash_bytes(data):
        """BLAKE2b-256 of data, on the GPU (src/block_id.rs:37-43)."""
        ptr, keep = _buf(bytes(data)) if len(data) else (None, None)
        out = ctypes.create_string_buffer(32)
        _n.check(_n.lib.cir_blake2b256(ptr, len(data), out))
        del keep
        return BlockHash(out.raw)

    def __bytes__(self):
        return self._b

    def __eq__(self, other):
        return isinstance(other, BlockHash) and other._b == self._b

    def __hash__(self):
        return hash(self._b)

    def __str__(self):
        return _hex(self._b)

    def __repr__(self):
        return "BlockHash(%s)" % _hex(self._b)


class ImageId:
    """Image id = the hash on the index's last line (src/id.rs:142-217)."""

    __slots__ = ("_b",)

    def __init__(self, raw):
        self._b = bytes(raw)

    @staticmethod
    def from_str(s):
        try:
            return ImageId(bytes.fromhex(s))
        except ValueError:
            raise ValueError("errors parding hexadecimal image id")

    def __bytes__(self):
        return self._b

    def __eq__(self, other):
        return isinstance(other, ImageId) and other._b == self._b

    def __hash__(self):
        return hash(self._b)

    def __str__(self):
        return _hex(self._b)

    def __repr__(self):
        return "ImageId(%s)" % _hex(self._b)


class HashType:
    """dir_signature::HashType."""

    __slots__ = ("code", "name")

    def __init__(self, code, name):
        self.code = code
        self.name = name

    @staticmethod
    def blake2b_256():
        return HashType(_n.CIR_HASH_BLAKE2B_256, "blake2b/256")

    @staticmethod
    def sha512_256():
        return HashType(_n.CIR_HASH_SHA512_256, "sha512/256")

    def __eq__(self, other):
        return isinstance(other, HashType) and other.code == self.code

    def __repr__(self):
        return "HashType(%s)" % self.name


class Hashes:
    """Per-block hashes of one file (dir_signature::v1::Hashes)."""

    def __init__(self, raw, block_size, hash_type=None):
        self._raw = bytes(raw)
        self._bs = block_size
        self._ht = hash_type or HashType.blake2b_256()

    @staticmethod
    def hash_file(hash_type, block_size, reader, context=None):
        """(size, Hashes) of everything `reader` yields (src/blocks.rs:193).

        reader: an int fd, an object with fileno(), or bytes-like data.
        """
        ctx = context or default_context()
        if isinstance(reader, (bytes, bytearray, memoryview)):
            raw = ctx.hash_memory(reader, block_size, hash_type)
            return len(reader), Hashes(raw, block_size, hash_type)
        fd = reader if isinstance(reader, int) else reader.fileno()
        size, raw = ctx.hash_file(fd, block_size, hash_type)
        return size, Hashes(raw, block_size, hash_type)

    def __len__(self):
        return len(self._raw) // 32

    def get(self, i):
        return self._raw[32 * i:32 * i + 32]

    def __iter__(self):
        return (self.get(i) for i in range(len(self)))

    def block_size(self):
        return self._bs

    def raw(self):
        return self._raw

    def check_file(self, reader, context=None):
        """Hashes::check_file (src/daemon/disk/commit.rs:104): re-hash the file
        on the GPU; True iff it has exactly these blocks."""
        ctx = context or default_context()
        fd = reader if isinstance(reader, int) else reader.fileno()
        return ctx.check_file(fd, self._bs, self._raw, self._ht)


class ScannerConfig:
    """dir_signature::ScannerConfig (used at src/client/sync/uploads.rs:50-54)."""

    def __init__(self):
        self._threads = 4  # GlobalOptions.threads default (src/client/global_options.rs:13)
        self._hash = HashType.blake2b_256()
        self._dirs = []
        self._block_size = DEFAULT_BLOCK_SIZE
        self._progress = False

    @staticmethod
    def new():
        return ScannerConfig()

    def threads(self, n):
        self._threads = int(n)
        return self

    def auto_threads(self):
        self._threads = 0
        return self

    def hash(self, hash_type):
        self._hash = hash_type
        return self

    def block_size(self, n):
        self._block_size = int(n)
        return self

    def add_dir(self, path, prefix="/"):
        self._dirs.append((os.fspath(path), prefix))
        return self

    def print_progress(self):
        self._progress = True
        return self


class v1:  # noqa: N801 - mirrors the `dir_signature::v1` module
    @staticmethod
    def scan(config, out=None, context=None):
        """dir_signature::v1::scan(&cfg, &mut Vec<u8>).

        With `out` (a bytearray), like the reference: the index is appended
        to it as the scan writes it out (cir_scan_v1_write: no whole-index
        copy after the scan) and None is returned.  Without, the index bytes
        are returned (cir_scan_v1)."""
        ctx = context or default_context()
        if out is not None:
            ctx.scan_into(config, out)
            return None
        return ctx.scan(config)


def sha512_256(data):
    """SHA-512/256 of data on the GPU (dir-signature's HashType::sha512_256)."""
    ptr, keep = _buf(bytes(data)) if len(data) else (None, None)
    out = ctypes.create_string_buffer(32)
    _n.check(_n.lib.cir_sha512_256(ptr, len(data), out))
    del keep
    return out.raw


def get_hash(index):
    """dir_signature::get_hash: the id bytes on the index's last line."""
    ptr, keep = _buf(index) if len(index) else (None, None)
    out = ctypes.create_string_buffer(64)
    n = ctypes.c_size_t()
    _n.check(_n.lib.cir_index_get_hash(ptr, len(index), out, ctypes.byref(n)))
    del keep
    return out.raw[:n.value]


class IndexError_(CiruelaError):  # noqa: N801 - ciruela::index::IndexError
    pass


class DirError(CiruelaError):
    """ciruela::blocks::DirError (src/blocks.rs:114-127)."""


class ReadError(CiruelaError):
    """ReadError of src/index.rs:74-85 / src/blocks.rs:95-111."""


def _raise_as(cls, fn):
    try:
        fn()
    except CiruelaError as e:
        raise cls(e.status, e.detail) from None


class InMemoryIndexes:
    """GetIndex implementation serving indexes from memory (src/index.rs:53)."""

    def __init__(self):
        self._h = _n.lib.cir_indexes_new()

    def __del__(self):
        try:
            _n.lib.cir_indexes_free(self._h)
        except Exception:
            pass

    def register_index(self, data):
        """Returns the ImageId (src/index.rs:98-105); IndexError_ on parse failure."""
        ptr, keep = _buf(bytes(data)) if len(data) else (ctypes.c_void_p(1), None)
        out = ctypes.create_string_buffer(64)
        n = ctypes.c_size_t()
        _raise_as(IndexError_, lambda: _n.check(
            _n.lib.cir_indexes_register(self._h, ptr, len(data), out, ctypes.byref(n))))
        del keep
        return ImageId(out.raw[:n.value])

    def read_index(self, image_id):
        raw = bytes(image_id)
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        _raise_as(ReadError, lambda: _n.check(
            _n.lib.cir_indexes_read(self._h, raw, len(raw), ctypes.byref(p), ctypes.byref(n))))
        return _n.take_buffer(p.value, n.value)


class BlockHint:
    """src/blocks.rs:46-48 (currently always empty)."""

    @staticmethod
    def empty():
        return BlockHint()


class ThreadedBlockReader:
    """GetBlock implementation (src/blocks.rs:85-240)."""

    def __init__(self, num_threads=40):
        self._h = _n.lib.cir_blocks_new()
        self._threads = num_threads

    @staticmethod
    def new():
        return ThreadedBlockReader()

    @staticmethod
    def new_num_threads(num):
        return ThreadedBlockReader(num)

    def __del__(self):
        try:
            _n.lib.cir_blocks_free(self._h)
        except Exception:
            pass

    def __len__(self):
        return _n.lib.cir_blocks_len(self._h)

    def register_dir(self, dir, index_data):  # noqa: A002 - reference name
        ptr, keep = _buf(bytes(index_data)) if len(index_data) else (ctypes.c_void_p(1), None)
        _raise_as(DirError, lambda: _n.check(_n.lib.cir_blocks_register_dir(
            self._h, os.fsencode(dir), ptr, len(index_data))))
        del keep

    def register_memory_blocks(self, hash_type, block_size, data, context=None):
        """src/blocks.rs:187-204: block ids are Hashes::hash_file(hash_type, ..)
        digests (put-file passes the index's hash type, put_file/network.rs:56)."""
        ctx = context or default_context()
        ptr, keep = _buf(bytes(data)) if len(data) else (None, None)
        _n.check(_n.lib.cir_blocks_register_memory_ht(ctx.handle, self._h, hash_type.code, ptr,
                                                      len(data), block_size))
        del keep

    def read_block(self, block_hash, hint=None):
        raw = bytes(block_hash)
        if len(raw) != 32:
            raise ValueError("BlockHash is 32 bytes")
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        _raise_as(ReadError, lambda: _n.check(
            _n.lib.cir_blocks_read(self._h, raw, ctypes.byref(p), ctypes.byref(n))))
        return _n.take_buffer(p.value, n.value)
