import ctypes
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, GOLDEN, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu)")


@pytest.fixture(scope="session")
def vectors():
    with open(os.path.join(GOLDEN, "blake2b256_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def dirsig_example():
    with open(os.path.join(GOLDEN, "dirsig_v1_example.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    """The C oracle (test infrastructure: oracle/blake2b_oracle.c)."""
    path = os.path.join(ROOT, "oracle", "build", "liboracle_blake2b.so")
    if not os.path.exists(path):
        import subprocess
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
    lib = ctypes.CDLL(path)
    vp, u64 = ctypes.c_void_p, ctypes.c_uint64
    lib.oracle_blake2b.argtypes = [vp, ctypes.c_size_t, vp, ctypes.c_size_t]
    lib.oracle_blake2b256.argtypes = [vp, vp, ctypes.c_size_t]
    lib.oracle_hash_blocks.argtypes = [vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_int]
    lib.oracle_hash_chunks.argtypes = [vp, u64, u64, vp, ctypes.c_int]
    lib.oracle_splitmix64_fill.argtypes = [vp, u64, u64, u64, u64, u64]
    lib.oracle_sha512_256.argtypes = [vp, vp, ctypes.c_size_t]
    return lib


def oracle_digest(lib, data):
    out = ctypes.create_string_buffer(32)
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    lib.oracle_blake2b256(out, buf, len(data))
    return out.raw


def oracle_sha(lib, data):
    out = ctypes.create_string_buffer(32)
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    lib.oracle_sha512_256(out, buf, len(data))
    return out.raw


@pytest.fixture(scope="session")
def gpu():
    """torch + ciruela_amd on cuda:0, or skip/fail when there is no GPU."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a GPU: run `pytest -m 'not gpu'` here")
    import ciruela_amd as ca
    torch.cuda.set_device(0)
    return ca
