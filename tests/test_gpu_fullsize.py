"""Parity at BASELINE.json's full sizes on one MI355X.

Config 2 (1 M x 32 KiB = 32 GiB) and config 3 (10 GiB of mixed 4 KiB /
32 KiB / 1 MiB blocks, 10 % ragged, shuffled), SURVEY.md 8d:
  * golden digests of the special config-2 blocks (0-15 zero, 16-31 range);
  * EVERY digest against the oracle: the splitmix64 data is regenerated on
    the host (counter-based, so in parallel chunks) and hashed by the
    threaded C oracle (16 threads, the box's CPU share per GPU);
  * determinism: a second launch gives the identical digest array, and the
    per-lane direct loader gives the same array as the LDS-DMA loader.
"""
import ctypes
import os
import random
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BS = 32768
SEED_C2 = 0x5EED0002


THREADS = 16


def host_fill(oracle, buf, word0, seed):
    """buf (uint64) = splitmix64 words word0.. of `seed`, filled in parallel."""
    n = buf.size
    step = max(1, (n + THREADS - 1) // THREADS)

    def part(k):
        a, b = k * step, min(n, (k + 1) * step)
        if a < b:
            oracle.oracle_splitmix64_fill(buf.ctypes.data + 8 * a, word0 + a, b - a, seed, 0, 0)

    with ThreadPoolExecutor(THREADS) as ex:
        list(ex.map(part, range(THREADS)))


def test_config2_full(gpu, oracle, vectors):
    import torch
    nblk = 1 << 20
    nbytes = nblk * BS
    data = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    gpu._n.check(gpu._n.lib.cir_fill_splitmix64_dev(data.data_ptr(), nbytes, SEED_C2, 0, 0, 0))
    data[:16 * BS].zero_()
    data[16 * BS:32 * BS].copy_(torch.arange(256, device="cuda:0").to(torch.uint8).repeat(16 * 128))
    ctx = gpu.Context(device_mask=1)
    out = torch.empty(nblk * 32, dtype=torch.uint8, device="cuda:0")
    ctx.hash_chunks_dev(data.data_ptr(), nbytes, BS, out.data_ptr(), 0)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(nblk, 32)
    gold = vectors["config2"]
    for i in range(16):
        assert got[i].tobytes().hex() == gold["zero_block"]
    for i in range(16, 32):
        assert got[i].tobytes().hex() == gold["range_block"]
    # every other block, 1 GiB of host data at a time
    per = 32768
    words = np.empty(per * BS // 8, dtype=np.uint64)
    want = np.zeros((per, 32), dtype=np.uint8)
    for b0 in range(0, nblk, per):
        host_fill(oracle, words, b0 * BS // 8, SEED_C2)
        oracle.oracle_hash_chunks(words.ctypes.data, per * BS, BS, want.ctypes.data, THREADS)
        lo = 32 if b0 == 0 else 0
        bad = np.nonzero((got[b0 + lo:b0 + per] != want[lo:]).any(axis=1))[0]
        assert bad.size == 0, "blocks %s differ" % (bad[:8] + b0 + lo)
    # determinism + loader A/B at full size
    out2 = torch.empty_like(out)
    gpu._n.check(gpu._n.lib.cir_debug_hash_uniform_dev(1, data.data_ptr(), BS, nblk,
                                                       out2.data_ptr(), 0))
    ctx.hash_chunks_dev(data.data_ptr(), nbytes, BS, out.data_ptr(), 0)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    assert np.array_equal(out.cpu().numpy().reshape(nblk, 32), got)
    del data


def test_config3_full(gpu, oracle):
    """10 GiB: equal bytes per class, 10% ragged U[1, size-1], shuffled."""
    import torch
    total = 10 << 30
    rng = random.Random(0x5EED0003)
    lens = []
    for size in (4096, 32768, 1 << 20):
        count = (total // 3) // size
        lens += [rng.randrange(1, size) if rng.random() < 0.1 else size for _ in range(count)]
    order = list(range(len(lens)))
    rng.shuffle(order)
    lens = [lens[i] for i in order]
    # arena: blocks back to back at 128-B aligned offsets in descriptor order
    l64 = np.array(lens, dtype=np.uint64)
    padded = (l64 + 127) // 128 * 128
    offs = np.zeros(len(lens), dtype=np.uint64)
    offs[1:] = np.cumsum(padded)[:-1]
    nbytes = int(offs[-1] + padded[-1])
    data = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    seed = 0x5EED0003
    gpu._n.check(gpu._n.lib.cir_fill_splitmix64_dev(data.data_ptr(), nbytes, seed, 0, 0, 0))
    d_off = torch.from_numpy(offs.view(np.int64)).to("cuda:0")
    d_len = torch.from_numpy(np.array(lens, dtype=np.int32)).to("cuda:0")
    out = torch.empty(32 * len(lens), dtype=torch.uint8, device="cuda:0")
    ctx = gpu.Context(device_mask=1)
    ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                        out.data_ptr(), 0)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(-1, 32)
    del data
    # every digest: regenerate the whole arena on the host, threaded oracle
    host = np.empty(nbytes // 8, dtype=np.uint64)
    host_fill(oracle, host, 0, seed)
    want = np.zeros((len(lens), 32), dtype=np.uint8)
    al = np.array(lens, dtype=np.uint32)
    oracle.oracle_hash_blocks(host.ctypes.data, offs.ctypes.data, al.ctypes.data, len(lens),
                              want.ctypes.data, THREADS)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, "blocks %s differ" % bad[:8]


def test_quad_file_above_4gib(gpu, oracle):
    """A device-resident file of 600 blocks of 8 MiB + 128 B (~5 GiB, a small
    batch: quad mode) with a short last block: 64-bit offsets in the quad
    path, every digest against the threaded oracle."""
    import torch
    bs = (8 << 20) + 128
    nbytes = 600 * bs - 4321
    seed = 0x5EED0006
    data = torch.empty(nbytes + 8, dtype=torch.uint8, device="cuda:0")
    gpu._n.check(gpu._n.lib.cir_fill_splitmix64_dev(data.data_ptr(), (nbytes + 7) // 8 * 8, seed,
                                                    0, 0, 0))
    nb = (nbytes + bs - 1) // bs
    out = torch.empty(32 * nb, dtype=torch.uint8, device="cuda:0")
    ctx = gpu.Context(device_mask=1)
    ctx.hash_chunks_dev(data.data_ptr(), nbytes, bs, out.data_ptr(), 0)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(-1, 32)
    del data
    host = np.empty((nbytes + 7) // 8, dtype=np.uint64)
    host_fill(oracle, host, 0, seed)
    want = np.zeros(32 * nb, dtype=np.uint8)
    oracle.oracle_hash_chunks(host.ctypes.data, nbytes, bs, want.ctypes.data, THREADS)
    bad = np.nonzero((got != want.reshape(-1, 32)).any(axis=1))[0]
    assert bad.size == 0, "blocks %s differ" % bad[:8]


SEED_C4 = 0x5EED0004


def host_fill_blocks(oracle, buf, word0, seed, block_words, first_block):
    """buf (uint64) = words word0.. of the per-block splitmix64 streams
    (block i seeded seed ^ (first_block + i)), filled in parallel."""
    n = buf.size
    step = max(1, (n + THREADS - 1) // THREADS)

    def part(k):
        a, b = k * step, min(n, (k + 1) * step)
        if a < b:
            oracle.oracle_splitmix64_fill(buf.ctypes.data + 8 * a, word0 + a, b - a, seed,
                                          block_words, first_block)

    with ThreadPoolExecutor(THREADS) as ex:
        list(ex.map(part, range(THREADS)))


@pytest.mark.parametrize("rank", range(8))
def test_config4_shard_full(gpu, oracle, rank):
    """Config 4 (BASELINE.json configs[3]): 256 GiB of 32 KiB
    blocks range-split over 8 GPUs, rank g owning global blocks
    [g*2^20, (g+1)*2^20), block i filled with splitmix64 seeded
    0x5EED0004 ^ i -- exactly as bench.py's N>1 path fills HBM
    (bench.shard + cir_fill_splitmix64_dev).  Each rank's full 32 GiB shard
    is hashed here, one after another on the one GPU, through
    cir_hash_chunks_dev, and EVERY digest is checked against the threaded
    oracle, which regenerates each block from its global index alone: the
    eight cases together check all 8,388,608 digests of config 4."""
    import sys
    import torch
    from conftest import ROOT
    sys.path.insert(0, ROOT)
    import bench
    nblk, world = 1 << 20, 8
    first, count = bench.shard(rank, world, nblk)
    assert (first, count) == (rank << 20, 1 << 20)
    nbytes = count * BS
    data = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    gpu._n.check(gpu._n.lib.cir_fill_splitmix64_dev(data.data_ptr(), nbytes, SEED_C4, BS, first,
                                                    0))
    ctx = gpu.Context(device_mask=1)
    out = torch.empty(count * 32, dtype=torch.uint8, device="cuda:0")
    ctx.hash_chunks_dev(data.data_ptr(), nbytes, BS, out.data_ptr(), 0)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(count, 32)
    del data
    per = 32768  # 1 GiB of host data at a time
    words = np.empty(per * BS // 8, dtype=np.uint64)
    want = np.zeros((per, 32), dtype=np.uint8)
    for b0 in range(0, count, per):
        host_fill_blocks(oracle, words, b0 * BS // 8, SEED_C4, BS // 8, first)
        oracle.oracle_hash_chunks(words.ctypes.data, per * BS, BS, want.ctypes.data, THREADS)
        bad = np.nonzero((got[b0:b0 + per] != want).any(axis=1))[0]
        assert bad.size == 0, "global blocks %s differ" % (bad[:8] + first + b0)
    # bench.py's own N>1 parity check agrees (the range boundaries + a spread)
    nbad, checked = bench.config4_check(bench.load_oracle(), out.cpu().numpy(), nbytes, BS, first)
    assert nbad == 0 and checked >= 128


def test_scan_tree_above_2gib(gpu, oracle, tmp_path):
    """cir_scan_v1 through the 3-slot staging pipeline on a 2.3 GiB tree (9+
    full 256 MiB batches, files straddling batches, ragged tails, an empty
    file, nested dirs), index byte for byte against the CPU indexer
    restatement (every block digest by the threaded C oracle, emitter and
    footer by dirsig_oracle)."""
    import cpu_indexer
    root = "/dev/shm" if os.path.isdir("/dev/shm") else str(tmp_path)
    import tempfile
    import shutil
    top = tempfile.mkdtemp(prefix="cir_scan2g_", dir=root)
    try:
        rng = np.random.default_rng(0x5EED2)
        sizes = [(40 << 20) + 12345, 0, 1, 32767, 32768, 32769, (300 << 20) - 7]
        sizes += [int(x) for x in rng.integers(1 << 20, 60 << 20, size=72)]
        total = 0
        for i, sz in enumerate(sizes):
            d = os.path.join(top, "d%d" % (i % 5), "e%d" % (i % 3))
            os.makedirs(d, exist_ok=True)
            blob = rng.integers(0, 1 << 63, size=(sz + 7) // 8, dtype=np.uint64).tobytes()[:sz]
            with open(os.path.join(d, "f%03d.bin" % i), "wb") as f:
                f.write(blob)
            total += sz
        assert total > (2 << 30)
        ctx = gpu.Context(device_mask=1)  # default 256 MiB staging
        cfg = gpu.ScannerConfig.new().threads(16).add_dir(top, "/")
        got = gpu.v1.scan(cfg, context=ctx)
        want = cpu_indexer.index(top, 32768, THREADS)
        assert got == want
        assert gpu.get_hash(got) == bytes.fromhex(want.rstrip(b"\n").split(b"\n")[-1].decode())
    finally:
        shutil.rmtree(top, ignore_errors=True)


def test_config1_cli_sync_append(gpu, tmp_path):
    """Config 1 at its stated size (BASELINE.json configs[0]):
    the 100-file / 10 MiB tree of 10 subdirectories that bench.py builds
    (make_config1_tree, default_rng(1)), indexed by one `ciruela-index sync
    --append SRC:/bench` process (the indexing half of `ciruela sync`,
    src/client/sync/uploads.rs:49-59, 4 disk threads).  The .ds1 it writes
    equals the scan oracle's index byte for byte, its name and the printed
    image id are the footer hash, and every block hash in it equals
    hash_bytes(block) (src/daemon/tracking/fetch_blocks.rs:77)."""
    import subprocess
    import sys
    from conftest import ROOT, oracle_digest
    import dirsig_oracle
    sys.path.insert(0, ROOT)
    import bench
    src = tmp_path / "tree"
    total = bench.make_config1_tree(str(src))
    assert total == 10 << 20
    assert sum(len(fs) for _, _, fs in os.walk(src)) == 100
    idx_dir = tmp_path / "idx"
    idx_dir.mkdir()
    out = subprocess.check_output([os.path.join(ROOT, "bin", "ciruela-index"), "sync",
                                   "--index-dir", str(idx_dir), "--append", "%s:/bench" % src],
                                  timeout=120)
    image_id, kind, dest, srcp = out.decode().split()
    assert (kind, dest, srcp) == ("append", "/bench", str(src))
    written = (idx_dir / (image_id + ".ds1")).read_bytes()
    want = dirsig_oracle.scan(str(src))
    assert written == want
    assert want.rstrip(b"\n").split(b"\n")[-1].decode() == image_id
    assert gpu.get_hash(written).hex() == image_id
    # per-block invariant on a sample of files, through the oracle's own hash
    oracle = bench.load_oracle()
    oracle.oracle_blake2b256.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    checked = 0
    for line in written.split(b"\n"):
        parts = line.split()
        if len(parts) >= 4 and parts[1] == b"f" and line.startswith(b"  "):
            name, size, hashes = parts[0].decode(), int(parts[2]), parts[3:]
            path = next(os.path.join(dp, name) for dp, _, fs in os.walk(src) if name in fs)
            blob = open(path, "rb").read()
            assert len(blob) == size and len(hashes) == (size + 32767) // 32768
            for k in (0, len(hashes) - 1):
                assert oracle_digest(oracle, blob[32768 * k:32768 * (k + 1)]).hex() == \
                    hashes[k].decode()
            checked += 1
    assert checked == 100


def test_config5_full_tree(gpu):
    """Config 5 at its stated size (BASELINE.json configs[4]): the 50 GiB
    tmpfs tree bench.py indexes (make_tree: 1600 files x 32 MiB in 40
    directories), scanned once through cir_scan_v1 with the default staging
    (3 x 256 MiB pinned slots) in a fresh context, and the index checked byte
    for byte against the CPU indexer restatement (oracle/cpu_indexer.py:
    every block by the threaded C oracle, emitter and footer by
    dirsig_oracle).  Skipped when /dev/shm cannot hold the tree."""
    import shutil
    import sys
    import tempfile
    from conftest import ROOT
    import cpu_indexer
    sys.path.insert(0, ROOT)
    import bench
    if not os.path.isdir("/dev/shm"):
        pytest.skip("no /dev/shm")
    st = os.statvfs("/dev/shm")
    if st.f_bavail * st.f_frsize < (55 << 30):
        pytest.skip("/dev/shm has %.1f GiB free, config 5 needs 55"
                    % (st.f_bavail * st.f_frsize / (1 << 30)))
    top = tempfile.mkdtemp(prefix="cir_cfg5_", dir="/dev/shm")
    try:
        nfiles = bench.make_tree(top, 50.0)
        assert nfiles == 1600
        ctx = gpu.Context(device_mask=1)
        cfg = gpu.ScannerConfig.new().threads(16).add_dir(top, "/")
        got = gpu.v1.scan(cfg, context=ctx)
        want = cpu_indexer.index(top, 32768, THREADS)
        assert len(got) == len(want)
        assert got == want
        ndirs = sum(len(ds) for _, ds, _ in os.walk(top))
        nfiles = sum(len(fs) for _, _, fs in os.walk(top))
        assert ndirs == 40 and nfiles >= 1600
        # header, "/", one line per directory and per file, footer
        assert got.count(b"\n") == 3 + ndirs + nfiles
    finally:
        shutil.rmtree(top, ignore_errors=True)
