"""Pin the oracle before trusting it (CPU only).

The oracle (oracle/blake2b_oracle.c) restates RFC 7693 BLAKE2b-256, the
function behind BlockHash::hash_bytes (reference src/block_id.rs:37-43).
No reference test pins a blake2b value, so it is pinned by
RFC 7693 Appendix A and by the hashlib-generated golden vectors.
"""
import ctypes
import hashlib
import os
import random
import struct

import numpy as np

from conftest import oracle_digest, oracle_sha
from make_golden import RFC7693_ABC_512, gen_bytes, splitmix64_words


def test_rfc7693_appendix_a(oracle):
    out = ctypes.create_string_buffer(64)
    assert oracle.oracle_blake2b(out, 64, b"abc", 3) == 0
    assert out.raw.hex() == RFC7693_ABC_512


def test_every_golden_vector(oracle, vectors):
    for v in vectors["vectors"]:
        assert oracle_digest(oracle, gen_bytes(v)).hex() == v["blake2b256"], (v["gen"], v["n"])


def test_known_answers_from_survey(oracle):
    # SURVEY.md 8c known-answer vectors
    assert oracle_digest(oracle, b"").hex() == \
        "0e5751c026e543b2e8ab2eb06099daa1d1e5df47778f7787faab45cdf12fe3a8"
    assert oracle_digest(oracle, b"abc").hex() == \
        "bddd813c634239723171ef3fee98579b94964e3bb1cb3e427262c8c068d52319"
    assert oracle_digest(oracle, bytes(32768)).hex() == \
        "e9334020344bcb418f16c532a4fad5465ef530cff3eaaee6411bddf59e210e50"
    assert oracle_digest(oracle, bytes(range(256)) * 128).hex() == \
        "c3e6c45e9ba7c00a92593d3c8a4ed297280751fa5c9ff4bdb545d6ef60a41aa6"


def test_random_against_hashlib(oracle):
    rng = random.Random(7)
    for _ in range(200):
        n = rng.choice([rng.randrange(0, 300), rng.randrange(0, 70000)])
        d = os.urandom(n)
        assert oracle_digest(oracle, d) == hashlib.blake2b(d, digest_size=32).digest()


def test_variable_digest_lengths(oracle):
    for outlen in (1, 20, 32, 48, 64):
        out = ctypes.create_string_buffer(outlen)
        oracle.oracle_blake2b(out, outlen, b"ciruela", 7)
        assert out.raw == hashlib.blake2b(b"ciruela", digest_size=outlen).digest()


def test_hash_chunks_split(oracle):
    """Hashes::hash_file split: ceil(n / bs) blocks, last short, none for 0."""
    data = np.frombuffer(os.urandom(100000), dtype=np.uint8).copy()
    for bs, n in [(32768, 100000), (4096, 4096), (4096, 4097), (1000, 1), (128, 100000)]:
        nb = (n + bs - 1) // bs
        out = np.zeros(max(nb, 1) * 32, dtype=np.uint8)
        oracle.oracle_hash_chunks(data.ctypes.data, n, bs, out.ctypes.data, 3)
        raw = data[:n].tobytes()
        for i in range(nb):
            want = hashlib.blake2b(raw[i * bs:(i + 1) * bs], digest_size=32).digest()
            assert out[32 * i:32 * i + 32].tobytes() == want


def test_hash_blocks_threads_agree(oracle):
    rng = random.Random(3)
    arena = np.frombuffer(os.urandom(300000), dtype=np.uint8).copy()
    n = 500
    lens = [rng.randrange(0, 3000) for _ in range(n)]
    offs = [rng.randrange(0, 300000 - 3000) for _ in range(n)]
    ao = np.array(offs, dtype=np.uint64)
    al = np.array(lens, dtype=np.uint32)
    outs = []
    for threads in (1, 4, 7):
        out = np.zeros(n * 32, dtype=np.uint8)
        oracle.oracle_hash_blocks(arena.ctypes.data, ao.ctypes.data, al.ctypes.data, n,
                                  out.ctypes.data, threads)
        outs.append(out)
    assert all(np.array_equal(outs[0], o) for o in outs[1:])
    raw = arena.tobytes()
    for i in range(0, n, 37):
        assert outs[0][32 * i:32 * i + 32].tobytes() == \
            hashlib.blake2b(raw[offs[i]:offs[i] + lens[i]], digest_size=32).digest()


def test_splitmix_host_twin(oracle):
    """oracle_splitmix64_fill == the golden generator (stream and per-block)."""
    buf = np.zeros(64, dtype=np.uint64)
    oracle.oracle_splitmix64_fill(buf.ctypes.data, 10, 64, 0x5EED0002, 0, 0)
    assert list(buf) == splitmix64_words(0x5EED0002, 64, first=10)
    # per-block streams: block words 8, first block 5
    oracle.oracle_splitmix64_fill(buf.ctypes.data, 0, 64, 0x5EED0004, 8, 5)
    for b in range(8):
        assert list(buf[8 * b:8 * b + 8]) == splitmix64_words(0x5EED0004 ^ (5 + b), 8)
    raw = struct.pack("<4Q", *splitmix64_words(7, 4))
    assert gen_bytes({"gen": "splitmix64", "n": 32, "seed": 7}) == raw


def test_sha512_256_oracle(oracle, dirsig_example):
    """Second hash type (FIPS 180-4): hashlib and the reference fixture."""
    for n in list(range(0, 260)) + [1000, 32768, 100000]:
        d = os.urandom(n)
        assert oracle_sha(oracle, d) == hashlib.new("sha512_256", d).digest(), n
    # reference fixture, src/cluster/download.rs:363: ".hidden f 7 6d7f5f98..."
    assert oracle_sha(oracle, b"Hidden\n").hex() == \
        "6d7f5f9804ee4dbc1ff7e12c7665387e0119e8ea629996c52d38b75c12ad0acf"
    idx = dirsig_example["index"].encode()
    body = idx[idx.index(b"\n") + 1:-65]
    assert oracle_sha(oracle, body).hex().encode() == idx[-65:-1]


def test_sha_chunks_threads_agree(oracle):
    """oracle_sha_chunks (threaded SHA-512/256 block split, bench.py's
    config2sha checker / CPU baseline) against hashlib."""
    oracle.oracle_sha_chunks.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_void_p, ctypes.c_int]
    rnd = random.Random(3)
    for n, bs in [(0, 4096), (1, 4096), (111, 128), (112, 128), (5 * 4096 + 17, 4096),
                  (70000, 32768)]:
        data = bytes(rnd.randrange(256) for _ in range(n))
        nb = (n + bs - 1) // bs
        out = ctypes.create_string_buffer(32 * max(nb, 1))
        buf = ctypes.create_string_buffer(data, max(n, 1))
        for threads in (1, 3):
            oracle.oracle_sha_chunks(buf, n, bs, out, threads)
            assert out.raw[:32 * nb] == b"".join(
                hashlib.new("sha512_256", data[i:i + bs]).digest() for i in range(0, n, bs))
