"""Pin the DIRSIGNATURE.v1 oracle with the reference's own fixture (CPU).

Fixture: src/cluster/download.rs:357-366 (test `roundtrip`), the only index
in the reference.  It is sha512/256, so it pins the format and the footer
rule, not the blake2b hash (that is pinned in test_oracle.py).
"""
import hashlib
import os
import random

import dirsig_oracle
import ciruela_amd as ca


def test_fixture_facts(dirsig_example):
    idx = dirsig_example["index"].encode()
    header_end = idx.index(b"\n") + 1
    body = idx[header_end:-65]
    # footer = H(every byte after the header line), newline included
    assert hashlib.new("sha512_256", body).hexdigest().encode() == idx[-65:-1]
    # per-block hash = H(block bytes)
    assert hashlib.new("sha512_256", b"Hidden\n").hexdigest() == \
        "6d7f5f9804ee4dbc1ff7e12c7665387e0119e8ea629996c52d38b75c12ad0acf"


def test_oracle_emitter_reproduces_fixture(dirsig_example):
    idx = dirsig_example["index"].encode()
    hash_name, bs, dirs, footer = dirsig_oracle.parse(idx)
    assert (hash_name, bs) == ("sha512/256", 32768)
    assert dirsig_oracle.emit(hash_name, bs, dirs) == idx


def test_oracle_block_split():
    data = os.urandom(70000)
    hs = dirsig_oracle.block_hashes(data, 32768)
    assert len(hs) == 3
    assert hs[2] == hashlib.blake2b(data[65536:], digest_size=32).digest()
    assert dirsig_oracle.block_hashes(b"", 32768) == []


def test_oracle_scan_small_tree(tmp_path):
    (tmp_path / "b").mkdir()
    (tmp_path / "a.txt").write_bytes(b"hello\n")
    (tmp_path / "b" / ".hidden").write_bytes(b"Hidden\n")
    (tmp_path / "b" / "empty").write_bytes(b"")
    idx = dirsig_oracle.scan(str(tmp_path))
    lines = idx.split(b"\n")
    assert lines[0] == b"DIRSIGNATURE.v1 blake2b/256 block_size=32768"
    assert lines[1] == b"/"
    assert lines[2].startswith(b"  a.txt f 6 ")
    assert lines[3] == b"/b"
    assert lines[4].startswith(b"  .hidden f 7 ")
    assert lines[5] == b"  empty f 0"
    assert lines[6] == hashlib.blake2b(b"\n".join(lines[1:6]) + b"\n",
                                       digest_size=32).hexdigest().encode()


def test_escape():
    assert dirsig_oracle.escape(b"a b\\c\x7f\xff") == b"a\\x20b\\x5cc\\x7f\\xff"


def test_library_parser_on_fixture(dirsig_example, tmp_path):
    """The product's parser accepts the fixture (a sha512/256 index) and
    maps every block (register_dir); re-hashing it on the GPU is covered by
    the -m gpu tests."""
    idx = dirsig_example["index"].encode()
    assert ca.get_hash(idx) == bytes.fromhex(
        "552ca5730ee95727e890a2155c88609d244624034ff70de264cf88220d11d6df")
    r = ca.ThreadedBlockReader()
    r.register_dir(str(tmp_path), idx)
    assert len(r) == 3


def test_cpu_indexer_matches_scan_oracle(tmp_path):
    """oracle/cpu_indexer.py (the threaded C restatement of the reference CPU
    indexer: whole files on `threads` workers, block_size chunks) emits the
    same index as the pure-Python scan oracle, at 1 and 4 threads."""
    import cpu_indexer
    rnd = random.Random(7)
    for i, size in enumerate([0, 1, 127, 128, 129, 4096, 4097, 3 * 4096, 70000]):
        d = tmp_path / ("d%d" % (i % 3))
        d.mkdir(exist_ok=True)
        (d / ("f%d" % i)).write_bytes(bytes(rnd.randrange(256) for _ in range(size)))
    (tmp_path / "d0" / "exe").write_bytes(b"#!/bin/sh\n")
    (tmp_path / "d0" / "exe").chmod(0o755)
    (tmp_path / "empty").mkdir()
    os.symlink("d0/f0", tmp_path / "link")
    want = dirsig_oracle.scan(str(tmp_path), 4096)
    for threads in (1, 4):
        assert cpu_indexer.index(str(tmp_path), 4096, threads) == want
    # and with dir-signature's other hash type (bench.py config 5 --hash sha512)
    want = dirsig_oracle.scan(str(tmp_path), 4096, "sha512/256")
    assert cpu_indexer.index(str(tmp_path), 4096, 3, hash_name="sha512/256") == want


def test_emitter_streaming_sanitized(tmp_path):
    """The emitter's streaming form (Emitter::consume, as cir_scan_v1_write
    drives it) under AddressSanitizer + UBSan, g++ on dirsig.cpp alone: random
    entries written out in random pieces, with the written and footer-fed
    prefix dropped, give exactly the whole index, and the footer feed exactly
    its body (tools/emitter_stream_fuzz.cpp)."""
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        import pytest
        pytest.skip("needs g++")
    from conftest import ROOT
    csrc = os.path.join(ROOT, "ciruela_amd", "csrc")
    exe = str(tmp_path / "emitter_stream_fuzz")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-I" + csrc,
                    os.path.join(ROOT, "tools", "emitter_stream_fuzz.cpp"),
                    os.path.join(csrc, "dirsig.cpp"), "-o", exe], check=True)
    for seed in (1, 2):
        p = subprocess.run([exe, "80", str(seed)], capture_output=True, timeout=300)
        assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
        assert b"no sanitizer report" in p.stdout
