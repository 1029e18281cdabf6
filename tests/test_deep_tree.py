"""A tree nested past PATH_MAX (4096 bytes of path).

dir-signature 0.2.9 walks with openat (Cargo.lock:323), so the reference
indexes such a tree; the scan here opens every directory relative to its
parent's fd and lists, lstats and read-links through it (scan.cpp read_dir),
and opens files for reading piecewise (open_long).  The oracle walks the
same way (oracle/dirsig_oracle.py walk, open_rel).  The CPU test pins the
oracle on such a tree; the GPU tests compare the scan with it.  (Parity
unpinned: the reference holds no such tree among its fixtures.)
"""
import errno
import os
import random
import stat

import pytest

import dirsig_oracle

LEVELS = 20
NAME = 240  # bytes per directory name: 20 levels = ~4.8 KB of path


def _level_name(i):
    return ("L%02d_" % i + "d" * NAME)[:NAME]


def make_deep_tree(root, seed=7):
    """root/L00_ddd.../L01_ddd.../... LEVELS deep (created through dir fds:
    no call below takes the full path), with files of several block counts
    along the way, an executable, a symlink and an empty directory at the
    bottom, and a short sibling subtree.  Returns the deepest path."""
    rng = random.Random(seed)
    os.makedirs(root, exist_ok=True)
    fd = os.open(root, os.O_RDONLY | os.O_DIRECTORY)
    path = root
    try:
        for i in range(LEVELS):
            if i in (0, 3, 11, LEVELS - 1):
                for k, size in enumerate((0, 1000, 70000, 3 * 32768 + 17)):
                    f = os.open("f%d_%d" % (i, k), os.O_WRONLY | os.O_CREAT, 0o644, dir_fd=fd)
                    os.write(f, rng.randbytes(size))
                    os.close(f)
            if i == LEVELS - 1:
                f = os.open("run.sh", os.O_WRONLY | os.O_CREAT, 0o755, dir_fd=fd)
                os.write(f, b"#!/bin/sh\necho deep\n")
                os.close(f)
                os.symlink("../" + _level_name(i - 1), "up", dir_fd=fd)
                os.mkdir("empty", dir_fd=fd)
                break
            name = _level_name(i)
            os.mkdir(name, dir_fd=fd)
            nfd = os.open(name, os.O_RDONLY | os.O_DIRECTORY, dir_fd=fd)
            os.close(fd)
            fd = nfd
            path = os.path.join(path, name)
    finally:
        os.close(fd)
    side = os.path.join(root, "side")
    os.mkdir(side)
    with open(os.path.join(side, "s.bin"), "wb") as f:
        f.write(rng.randbytes(5000))
    return path


def test_oracle_walks_past_path_max(tmp_path):
    root = str(tmp_path / "deep")
    deepest = make_deep_tree(root)
    assert len(os.fsencode(deepest)) > 4096
    # the tree really is beyond what a path-based walk can open
    with pytest.raises(OSError) as e:
        os.listdir(deepest)
    assert e.value.errno == errno.ENAMETOOLONG
    idx = dirsig_oracle.scan(root, 32768)
    text = idx.decode("latin-1")
    # every level's directory line, the deepest one's files, link and exe
    assert text.count("\n/L") == LEVELS  # LEVELS - 1 level dirs and the empty one
    assert " up s ../" + _level_name(LEVELS - 2) in text
    assert "  run.sh x 20 " in text
    assert "  f19_3 f 98321 " in text
    # the deepest file reads back through open_rel
    parts = tuple(os.fsencode(_level_name(i)) for i in range(LEVELS - 1)) + (b"f19_2",)
    fd = dirsig_oracle.open_rel(root, parts)
    try:
        assert stat.S_ISREG(os.fstat(fd).st_mode) and os.fstat(fd).st_size == 70000
    finally:
        os.close(fd)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["whole", "written", "split"])
@pytest.mark.parametrize("hash_name", ["blake2b/256", "sha512/256"])
def test_scan_past_path_max_matches_oracle(gpu, tmp_path, monkeypatch, mode, hash_name):
    root = str(tmp_path / "deep")
    make_deep_tree(root, seed=len(mode) + len(hash_name))
    if mode == "split":  # two device states on the one GPU, stripes of 1 block
        monkeypatch.setenv("CIR_DEBUG_SPLIT", "2")
        monkeypatch.setenv("CIR_DEBUG_STRIPE_BLOCKS", "1")
    ctx = gpu.Context(device_mask=1, staging_bytes=1 << 20)
    monkeypatch.delenv("CIR_DEBUG_SPLIT", raising=False)
    ht = gpu.HashType.sha512_256() if hash_name == "sha512/256" else gpu.HashType.blake2b_256()
    cfg = gpu.ScannerConfig.new().block_size(32768).threads(3).hash(ht)
    cfg.add_dir(root, "/")
    if mode == "written":
        out = bytearray()
        gpu.v1.scan(cfg, out=out, context=ctx)
        got = bytes(out)
    else:
        got = gpu.v1.scan(cfg, context=ctx)
    want = dirsig_oracle.scan(root, 32768, hash_name)
    assert got == want
    ctx.close()


@pytest.mark.gpu
def test_cli_sync_past_path_max(gpu, tmp_path):
    """`ciruela-index sync` of the deep tree: the same index as the oracle."""
    import subprocess
    from conftest import ROOT
    root = str(tmp_path / "deep")
    make_deep_tree(root, seed=3)
    exe = os.path.join(ROOT, "bin", "ciruela-index")
    p = subprocess.run([exe, "sync", "--append", root + ":/dest", "--index-dir", str(tmp_path)],
                       capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    image_id = p.stdout.decode().split()[0]
    assert (tmp_path / (image_id + ".ds1")).read_bytes() == dirsig_oracle.scan(root, 32768)
