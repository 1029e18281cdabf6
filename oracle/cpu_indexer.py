"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by ciruela_amd/).

The reference CPU indexer restated for large trees: dir-signature's
v1::scan as `ciruela sync` runs it (src/client/sync/uploads.rs:49-59:
ScannerConfig::threads(gopt.threads), default 4 from
src/client/global_options.rs:13; hash blake2b/256).  The walk and the
DIRSIGNATURE.v1 emission are dirsig_oracle's; the per-file hashing loop
(Hashes::hash_file over block_size chunks, whole files on a pool of
`threads` workers) is oracle_hash_files in blake2b_oracle.c.  The reference
Rust cannot be built here (no toolchain, un-vendored crates), so this is the
CPU baseline bench.py reports (kind "port") and the checker of the scan.
"""
import ctypes
import os

import dirsig_oracle

HERE = os.path.dirname(os.path.abspath(__file__))


def load(path=None):
    lib = ctypes.CDLL(path or os.path.join(HERE, "build", "liboracle_blake2b.so"))
    vp, u64 = ctypes.c_void_p, ctypes.c_uint64
    for f in (lib.oracle_hash_files, lib.oracle_sha_files):
        f.argtypes = [ctypes.POINTER(ctypes.c_char_p), vp, vp, ctypes.c_size_t, u64, vp,
                      ctypes.c_int]
    lib.oracle_hash_chunks.argtypes = [vp, u64, u64, vp, ctypes.c_int]
    lib.oracle_hash_blocks.argtypes = [vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_int]
    lib.oracle_splitmix64_fill.argtypes = [vp, u64, u64, u64, u64, u64]
    return lib


def files_hasher(lib, threads, hash_name="blake2b/256"):
    """files_hasher(paths, sizes, bs) -> per-file digest lists, whole files
    spread over `threads` C workers."""
    import numpy as np
    hash_files = lib.oracle_sha_files if hash_name == "sha512/256" else lib.oracle_hash_files

    def run(paths, sizes, bs):
        n = len(paths)
        nblk = np.array([(s + bs - 1) // bs for s in sizes], dtype=np.uint64)
        first = np.zeros(n, dtype=np.uint64)
        if n:
            first[1:] = np.cumsum(nblk)[:-1]
        total = int(nblk.sum()) if n else 0
        out = np.zeros(32 * max(total, 1), dtype=np.uint8)
        cp = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
        rc = hash_files(cp, first.ctypes.data, nblk.ctypes.data, n, bs, out.ctypes.data,
                        threads)
        if rc:
            raise OSError(-rc, "oracle_hash_files: " + os.strerror(-rc))
        raw = out.tobytes()
        return [[raw[32 * (int(first[i]) + k):32 * (int(first[i]) + k + 1)]
                 for k in range(int(nblk[i]))] for i in range(n)]
    return run


def index(root, block_size=32768, threads=4, lib=None, hash_name="blake2b/256"):
    """Index bytes of the tree at `root`, hashed on `threads` CPU workers."""
    lib = lib or load()
    return dirsig_oracle.scan(root, block_size, hash_name,
                              files_hasher=files_hasher(lib, threads, hash_name))
