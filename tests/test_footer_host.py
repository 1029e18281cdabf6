"""The index footer's host BLAKE2b-256 (CPU only, no device involved).

cir_scan_v1 hashes a blake2b/256 index's footer -- ImageId = H(every byte
after the header line), dir_signature::get_hash read back by
InMemoryIndexes::register_index (reference src/index.rs:98-105) -- on one host
thread fed in stretches as the index is emitted (scan.cpp HostFooter,
blake2b_host.cpp).  It is product code, not the oracle; here it is checked
against the oracle, the golden vectors and hashlib, over every way a stream
can be cut: piece sizes around the 128-B block edge, single bytes, and the
empty input.  The GPU side of the same footer is test_scan_footer_modes in
tests/test_gpu_parity.py.
"""
import ctypes
import hashlib
import os
import random

from conftest import oracle_digest
from make_golden import gen_bytes

from ciruela_amd import _native


def host_digest(data, piece=0):
    out = ctypes.create_string_buffer(32)
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    _native.check(_native.lib.cir_debug_host_blake2b256(buf, len(data), piece, out))
    return out.raw


def test_golden_vectors_one_update(vectors):
    for v in vectors["vectors"]:
        assert host_digest(gen_bytes(v)).hex() == v["blake2b256"], (v["gen"], v["n"])


def test_pieces_across_block_edges(oracle):
    rng = random.Random(11)
    for n in [0, 1, 127, 128, 129, 255, 256, 257, 1000, 4096, 65 * 1000 + 3]:
        data = os.urandom(n)
        want = oracle_digest(oracle, data)
        for piece in [0, 1, 63, 127, 128, 129, 256, 1000, rng.randrange(1, 600)]:
            assert host_digest(data, piece) == want, (n, piece)


def test_index_sized_text_against_hashlib():
    """A 2.3 MiB index-like body (hex digest lines) fed in 256 KiB stretches,
    the scan's feed size, plus a ragged last stretch."""
    lines = b"".join(b"  f%05d f 32768 %s\n" % (i, os.urandom(32).hex().encode())
                     for i in range(30000))
    assert len(lines) % (256 << 10) != 0
    assert host_digest(lines, 256 << 10) == hashlib.blake2b(lines, digest_size=32).digest()


def test_reference_fixture_rule(dirsig_example):
    """The footer rule of the reference's fixture (src/cluster/download.rs:
    357-366) with this hasher: H(body) as the last line, here for blake2b."""
    idx = dirsig_example["index"].encode()
    body = idx[idx.index(b"\n") + 1:-65]
    assert host_digest(body, 7) == hashlib.blake2b(body, digest_size=32).digest()


def host_sha_digest(data, piece=0):
    out = ctypes.create_string_buffer(32)
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    _native.check(_native.lib.cir_debug_host_sha512_256(buf, len(data), piece, out))
    return out.raw


def test_sha512_256_footer_hasher(oracle):
    """The sha512/256 twin (a sha512/256 index's footer, dir-signature's
    second hash type) over lengths around the 112-byte padding edge and the
    128-byte block, in every feed size, against the oracle and hashlib."""
    from conftest import oracle_sha
    rng = random.Random(12)
    for n in [0, 1, 111, 112, 113, 127, 128, 129, 239, 240, 256, 1000, 70001]:
        data = os.urandom(n)
        want = oracle_sha(oracle, data)
        assert want == hashlib.new("sha512_256", data).digest()
        for piece in [0, 1, 64, 111, 112, 128, 129, rng.randrange(1, 500)]:
            assert host_sha_digest(data, piece) == want, (n, piece)


def test_sha512_256_reference_fixture(dirsig_example):
    """The reference's own sha512/256 index (src/cluster/download.rs:357-366):
    its footer line is this hasher's digest of its body, and its `.hidden`
    line the digest of "Hidden\\n"."""
    idx = dirsig_example["index"].encode()
    body = idx[idx.index(b"\n") + 1:-65]
    assert host_sha_digest(body, 5).hex().encode() == idx[-65:-1]
    assert host_sha_digest(b"Hidden\n").hex() == \
        "6d7f5f9804ee4dbc1ff7e12c7665387e0119e8ea629996c52d38b75c12ad0acf"


def test_footer_hashers_sanitized(tmp_path):
    """Both host hashers under AddressSanitizer + UBSan (g++ on the sources
    alone, no device): random feeds agree with one-shot feeds, and stdin's
    digests equal hashlib's for every piece size."""
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        import pytest
        pytest.skip("needs g++")
    from conftest import ROOT
    csrc = os.path.join(ROOT, "ciruela_amd", "csrc")
    exe = str(tmp_path / "footer_hash_fuzz")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-I" + csrc,
                    os.path.join(ROOT, "tools", "footer_hash_fuzz.cpp"),
                    os.path.join(csrc, "blake2b_host.cpp"), os.path.join(csrc, "sha512_host.cpp"),
                    "-o", exe], check=True)
    rng = random.Random(5)
    for n, piece in [(0, 0), (1, 1), (111, 7), (112, 0), (128, 128), (129, 64), (4096, 1000),
                     (200000, 256 << 10), (70001, rng.randrange(1, 5000))]:
        data = os.urandom(n)
        p = subprocess.run([exe, "300", str(piece)], input=data, capture_output=True,
                           timeout=120)
        assert p.returncode == 0, p.stderr[-3000:]
        out = p.stdout.decode().split("\n")
        b2, sh = out[0].split()
        assert b2 == hashlib.blake2b(data, digest_size=32).hexdigest(), n
        assert sh == hashlib.new("sha512_256", data).hexdigest(), n
        assert "no sanitizer report" in p.stdout.decode()
