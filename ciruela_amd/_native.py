"""ctypes binding of libciruela_amd.so (include/ciruela_blockhash.h).

The library is the product: every hash it returns was computed by the gfx950
kernels.  There is no fallback; a missing library raises ImportError and a
missing GPU makes the hashing calls raise `NoDevice`.

PyTorch, when installed, is imported first so that the library binds to the
HIP runtime PyTorch already carries (same soname, libamdhip64.so.7): device
pointers and streams from torch tensors are then valid in the library.
"""
import ctypes
import os

try:  # share torch's HIP runtime (see module docstring)
    import torch as _torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the library
    _torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# CIRUELA_AMD_LIB: another build of the same library (A/B of build variants)
LIB_PATH = os.environ.get("CIRUELA_AMD_LIB") or os.path.join(_HERE, "libciruela_amd.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "libciruela_amd.so is not built; run `make` or "
        "`python -c 'import __graft_entry__ as g; g.build()'` in the repo root")

lib = ctypes.CDLL(LIB_PATH)

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_sizep = ctypes.POINTER(ctypes.c_size_t)
c_vp = ctypes.c_void_p

CIR_OK = 0
CIR_EIO = -1
CIR_EINVAL = -2
CIR_EHIP = -3
CIR_ENOMEM = -4
CIR_EPARSE = -5
CIR_ENOTFOUND = -6
CIR_EHASHSIZE = -7
CIR_ENODEV = -8
CIR_EUNSUPPORTED = -9
CIR_EAGAIN = -10
CIR_VERIFY_NONBLOCK = 1
CIR_VERIFY_STATS_FIELDS = 8
CIR_INIT_ONE_SHOT = 1  # cir_init_n: one stream and one staging slot per device
CIR_STAGING_LAZY = (1 << 64) - 1  # cir_init: no staging slots until a host path needs them

CIR_HASH_BLAKE2B_256 = 1
CIR_HASH_SHA512_256 = 2

# cir_write_fn: int (*)(void* user, const uint8_t* data, size_t n)
WRITE_FN = ctypes.CFUNCTYPE(ctypes.c_int, c_vp, c_vp, ctypes.c_size_t)

# name -> (restype, argtypes)
_SIGS = {
    "cir_init": (ctypes.c_int, [ctypes.POINTER(c_vp), ctypes.c_uint32, ctypes.c_uint64]),
    "cir_init_n": (ctypes.c_int, [ctypes.POINTER(c_vp), ctypes.c_uint32, ctypes.c_uint64,
                                  ctypes.c_uint32, ctypes.c_uint32]),
    "cir_devices_for_bytes": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]),
    "cir_destroy": (None, [c_vp]),
    "cir_device_count": (ctypes.c_int, []),
    "cir_ctx_devices": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "cir_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "cir_last_error": (ctypes.c_char_p, []),
    "cir_free": (None, [c_vp]),
    "cir_blake2b256": (ctypes.c_int, [c_vp, ctypes.c_size_t, c_vp]),
    "cir_hash_chunks_dev": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, ctypes.c_uint64, c_vp,
                                           c_vp]),
    "cir_hash_blocks_dev": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.c_size_t, c_vp, c_vp]),
    "cir_hash_blocks": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.c_size_t, c_vp]),
    "cir_hash_file": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_uint64, c_u64p,
                                     ctypes.POINTER(c_vp), c_sizep]),
    "cir_hash_memory": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.POINTER(c_vp), c_sizep]),
    "cir_scan_v1": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_char_p),
                                   ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t,
                                   ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32,
                                   ctypes.POINTER(c_vp), c_sizep]),
    "cir_scan_v1_write": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_char_p),
                                         ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t,
                                         ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32,
                                         WRITE_FN, c_vp, c_sizep]),
    "cir_index_get_hash": (ctypes.c_int, [c_vp, ctypes.c_size_t, c_vp, c_sizep]),
    "cir_index_rewrite": (ctypes.c_int, [c_vp, c_vp, ctypes.c_size_t, ctypes.POINTER(c_vp),
                                         c_sizep]),
    "cir_indexes_new": (c_vp, []),
    "cir_indexes_free": (None, [c_vp]),
    "cir_indexes_register": (ctypes.c_int, [c_vp, c_vp, ctypes.c_size_t, c_vp, c_sizep]),
    "cir_indexes_read": (ctypes.c_int, [c_vp, c_vp, ctypes.c_size_t, ctypes.POINTER(c_vp),
                                        c_sizep]),
    "cir_blocks_new": (c_vp, []),
    "cir_blocks_free": (None, [c_vp]),
    "cir_blocks_len": (ctypes.c_size_t, [c_vp]),
    "cir_blocks_register_dir": (ctypes.c_int, [c_vp, ctypes.c_char_p, c_vp, ctypes.c_size_t]),
    "cir_blocks_register_memory": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_size_t,
                                                  ctypes.c_uint64]),
    "cir_blocks_register_memory_ht": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, c_vp,
                                                     ctypes.c_size_t, ctypes.c_uint64]),
    "cir_blocks_read": (ctypes.c_int, [c_vp, c_vp, ctypes.POINTER(c_vp), c_sizep]),
    "cir_sha512_256": (ctypes.c_int, [c_vp, ctypes.c_size_t, c_vp]),
    "cir_hash_blocks_dev_ht": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, c_vp, c_vp, ctypes.c_size_t,
                                              c_vp, c_vp]),
    "cir_hash_blocks_ht": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, c_vp, c_vp, ctypes.c_size_t,
                                          c_vp]),
    "cir_hash_file_ht": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, c_u64p,
                                        ctypes.POINTER(c_vp), c_sizep]),
    "cir_hash_memory_ht": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, ctypes.c_uint64,
                                          ctypes.c_uint64, ctypes.POINTER(c_vp), c_sizep]),
    "cir_verify_blocks_dev": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, c_vp, c_vp, ctypes.c_size_t,
                                             c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cir_verify_blocks": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, c_vp, c_vp, ctypes.c_size_t,
                                         c_vp, c_vp, c_sizep]),
    "cir_hash_blocks_bounded": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, ctypes.c_uint64, c_vp,
                                               c_vp, ctypes.c_size_t, c_vp, c_sizep]),
    "cir_verify_blocks_bounded": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, ctypes.c_uint64, c_vp,
                                                 c_vp, ctypes.c_size_t, c_vp, c_vp, c_sizep]),
    "cir_hash_blocks_dev_bounded": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, ctypes.c_uint64, c_vp,
                                                   c_vp, ctypes.c_size_t, c_vp, c_vp, c_vp]),
    "cir_verify_blocks_dev_bounded": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, ctypes.c_uint64,
                                                     c_vp, c_vp, ctypes.c_size_t, c_vp, c_vp, c_vp,
                                                     c_vp, c_vp]),
    "cir_check_file": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, c_vp,
                                      ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]),
    "cir_debug_compress_only_dev": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, c_vp, c_vp]),
    "cir_debug_relay_blocks": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
    "cir_debug_device_identity": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                                                 c_vp, ctypes.POINTER(ctypes.c_uint64)]),
    "cir_debug_desc_timing": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "cir_debug_desc_times": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double)]),
    "cir_verify_submit": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp, ctypes.c_size_t, c_vp,
                                         ctypes.POINTER(ctypes.c_uint64)]),
    "cir_verify_poll": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int)]),
    "cir_verify_wait": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int)]),
    "cir_verify_window": (ctypes.c_int, [c_vp, ctypes.c_uint32, ctypes.c_uint32]),
    "cir_verify_forget": (ctypes.c_int, [c_vp, ctypes.c_uint64]),
    "cir_verify_limits": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]),
    "cir_verify_stats": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_uint64)]),
    "cir_set_footer_mode": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "cir_debug_scan_timing": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "cir_debug_scan_batches": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double),
                                              ctypes.c_size_t, c_sizep]),
    "cir_debug_scan_phases": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double)]),
    "cir_debug_host_blake2b256": (ctypes.c_int, [c_vp, ctypes.c_size_t, ctypes.c_size_t, c_vp]),
    "cir_debug_host_sha512_256": (ctypes.c_int, [c_vp, ctypes.c_size_t, ctypes.c_size_t, c_vp]),
    "cir_debug_hash_uniform_dev": (ctypes.c_int, [ctypes.c_int, c_vp, ctypes.c_uint64,
                                                  ctypes.c_uint64, c_vp, c_vp]),
    "cir_fill_splitmix64_dev": (ctypes.c_int, [c_vp, ctypes.c_uint64, ctypes.c_uint64,
                                               ctypes.c_uint64, ctypes.c_uint64, c_vp]),
}

for _name, (_res, _args) in _SIGS.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = tuple(_SIGS)


class CiruelaError(Exception):
    """A failing C-ABI call: `.status` is the CIR_E* code."""

    def __init__(self, status, detail=""):
        self.status = status
        self.detail = detail
        msg = lib.cir_strerror(status).decode()
        super().__init__("%s: %s" % (msg, detail) if detail else msg)


class NoDevice(CiruelaError):
    pass


def check(status):
    if status == CIR_OK:
        return
    detail = (lib.cir_last_error() or b"").decode(errors="replace")
    if status == CIR_ENODEV:
        raise NoDevice(status, detail)
    raise CiruelaError(status, detail)


def take_buffer(ptr, n):
    """Copy a library-allocated buffer into bytes and cir_free it."""
    if not ptr:
        return b""
    try:
        return ctypes.string_at(ptr, n)
    finally:
        lib.cir_free(ptr)
