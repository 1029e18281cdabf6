"""GPU parity: every digest from the gfx950 kernels equals the oracle's.

Bit-exact (byte work).  Sizes small enough for the oracle to finish in
seconds; the full BASELINE sizes are in test_gpu_fullsize.py.  All calls go
through the C ABI (libciruela_amd.so).
"""
import ctypes
import os
import random
import zlib

import numpy as np
import pytest

from conftest import oracle_digest, oracle_sha
from make_golden import gen_bytes

import dirsig_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(gpu):
    return gpu.Context(device_mask=1, staging_bytes=8 << 20)


@pytest.fixture(scope="module")
def small_ctx(gpu):
    # tiny staging buffers: forces many double-buffered batches
    return gpu.Context(device_mask=1, staging_bytes=1 << 20)


def dev_random(gpu, nbytes, seed, pad=64):
    import torch
    n = (nbytes + pad + 7) // 8 * 8
    t = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    gpu._n.check(gpu._n.lib.cir_fill_splitmix64_dev(t.data_ptr(), n, seed, 0, 0, 0))
    torch.cuda.synchronize()
    return t


def oracle_chunks(oracle, host, nbytes, bs):
    nb = (nbytes + bs - 1) // bs
    out = np.zeros(max(nb, 1) * 32, dtype=np.uint8)
    oracle.oracle_hash_chunks(host.ctypes.data, nbytes, bs, out.ctypes.data, 8)
    return out[:nb * 32]


def first_bad(a, b):
    d = (a.reshape(-1, 32) != b.reshape(-1, 32)).any(1)
    return int(np.nonzero(d)[0][0]) if d.any() else None


def test_golden_vectors_host_entry(ctx, vectors):
    vecs = vectors["vectors"]
    arena = b"".join(gen_bytes(v) for v in vecs)
    offs, pos = [], 0
    for v in vecs:
        offs.append(pos)
        pos += v["n"]
    got = ctx.hash_blocks(arena, offs, [v["n"] for v in vecs])
    for i, v in enumerate(vecs):
        assert got[32 * i:32 * i + 32].hex() == v["blake2b256"], (i, v["gen"], v["n"])


def test_golden_vectors_device_entry(gpu, ctx, vectors):
    import torch
    vecs = vectors["vectors"]
    # place every vector at a 128-B aligned offset, plus misaligned copies
    chunks, offs, lens, pos = [], [], [], 0
    for k, v in enumerate(vecs):
        data = gen_bytes(v)
        skew = (k * 5) % 16 if k % 3 == 0 else 0
        pad = (-pos) % 128 + skew
        chunks.append(bytes(pad) + data)
        pos += pad
        offs.append(pos)
        lens.append(len(data))
        pos += len(data)
    arena = torch.tensor(bytearray(b"".join(chunks) + bytes(16)), dtype=torch.uint8,
                         device="cuda:0")
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * len(vecs), dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev(arena.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(vecs),
                        out.data_ptr(), 0)
    torch.cuda.synchronize()
    got = out.cpu().numpy().tobytes()
    for i, v in enumerate(vecs):
        assert got[32 * i:32 * i + 32].hex() == v["blake2b256"], (i, v["gen"], v["n"])


def test_hash_bytes(gpu, oracle):
    for data in [b"", b"abc", b"Hidden\n", bytes(128), bytes(129), os.urandom(100000)]:
        assert bytes(gpu.BlockHash.hash_bytes(data)) == oracle_digest(oracle, data)


def test_hash_bytes_from_many_threads(gpu, oracle):
    """BlockHash::hash_bytes is called per received block by the daemon's
    fetch futures (src/daemon/tracking/fetch_blocks.rs:77): eight host
    threads hashing at once through the one default context (callers that
    arrive while a launch runs are coalesced into the next one; ctypes drops
    the GIL) all get their own block's digest, sizes 0 .. 40 KiB across the
    single-shot buffers' growth."""
    from concurrent.futures import ThreadPoolExecutor
    rng = random.Random(77)
    blocks = [os.urandom(rng.choice([0, 1, 127, 128, 129, 4096, 32768, 40000]))
              for _ in range(160)]
    with ThreadPoolExecutor(8) as ex:
        got = list(ex.map(lambda b: bytes(gpu.BlockHash.hash_bytes(b)), blocks))
    for b, g in zip(blocks, got):
        assert g == oracle_digest(oracle, b), len(b)


def test_hash_bytes_concurrent_callers_share_launches(gpu, oracle):
    """32 threads each hashing 32 KiB blocks through the drop-in: coalesced,
    they finish in far less than 32 x one call's time (one chain's latency
    serves the callers that queued meanwhile), every digest correct."""
    import time
    from concurrent.futures import ThreadPoolExecutor
    blk = [os.urandom(32768) for _ in range(32)]
    want = [oracle_digest(oracle, b) for b in blk]
    for _ in range(3):
        bytes(gpu.BlockHash.hash_bytes(blk[0]))
    t0 = time.perf_counter()
    for b in blk[:8]:
        gpu.BlockHash.hash_bytes(b)
    one = (time.perf_counter() - t0) / 8
    with ThreadPoolExecutor(32) as ex:
        for _ in range(2):  # warm the batch buffers
            list(ex.map(lambda b: bytes(gpu.BlockHash.hash_bytes(b)), blk))
        t0 = time.perf_counter()
        got = list(ex.map(lambda b: bytes(gpu.BlockHash.hash_bytes(b)), blk * 4))
        both = time.perf_counter() - t0
    assert got == want * 4
    print("hash_bytes 32 KiB: one call %.0f us; 128 calls from 32 threads %.0f us (%.1f us/call)"
          % (one * 1e6, both * 1e6, both * 1e6 / 128))
    assert both < 0.5 * 128 * one, (both, one)


@pytest.mark.parametrize("bs,nbytes", [
    # < kQuadSmallBatch blocks of >= 8 lines: quad mode (k_quad_chunks)
    (32768, 256 * 32768),
    (32768, 512 * 32768 + 1000),     # + a short tail
    (32768, 300 * 32768 + 5),
    (32768, 100 * 32768),
    (32768, 1), (32768, 127), (32768, 128), (32768, 129), (32768, 32768),
    (4096, 1000 * 4096),
    (128, 1024 * 128 + 64),          # 1-line blocks: lane mode at any count
    (1 << 20, 3 * (1 << 20) + 7),
    (1000, 50000),                   # bs not a multiple of 128: unaligned blocks
    (4097, 300001),
    (65536, 512 * 65536),
    # >= kQuadSmallBatch blocks: the lane-mode launch (LDS-DMA body + fused
    # ragged rest, or the general loader when bs % 128 != 0)
    (4096, 70000 * 4096 + 1234),
    (1000, 70000 * 1000 + 7),
    (128, 65536 * 128),
    (32768, 49152 * 32768 + 99),   # one block past the quad-mode batch limit
    # with a context the ragged rest runs in quad mode beside the uniform
    # part (launch_chunks_split): 255 whole blocks, and whole + short ones
    (32768, 65535 * 32768),
    (1024, 65535 * 1024 + 3),
    # 1 < lane waves per SIMD <= 1.625 (65537..106496 blocks on 1024 SIMDs):
    # quad mode again (chunks_in_quad), whole and with a short tail
    (1024, 81920 * 1024),
    (1024, 81921 * 1024 + 500),
    (2048, 106496 * 2048),
    (1024, 106497 * 1024),           # just past the band: lane mode
])
def test_chunks_dev_vs_oracle(gpu, ctx, oracle, bs, nbytes):
    import torch
    data = dev_random(gpu, nbytes, seed=bs * 31 + nbytes)
    nb = (nbytes + bs - 1) // bs
    out = torch.zeros(nb * 32, dtype=torch.uint8, device="cuda:0")
    ctx.hash_chunks_dev(data.data_ptr(), nbytes, bs, out.data_ptr(), 0)
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    want = oracle_chunks(oracle, host, nbytes, bs)
    got = out.cpu().numpy()
    assert first_bad(got, want) is None, "block %s" % first_bad(got, want)


@pytest.mark.parametrize("skew,nfull", [(1, 300), (4, 300), (8, 300), (15, 300), (4, 50000)])
def test_chunks_dev_misaligned_base(gpu, ctx, oracle, skew, nfull):
    """Quad mode (300 blocks) and lane mode (50000: the general loader, since
    a misaligned base rules out the LDS-DMA body) on a misaligned file."""
    import torch
    bs = 32768 if nfull < 1000 else 4096
    nbytes = nfull * bs + 77
    data = dev_random(gpu, nbytes + skew, seed=skew)
    nb = (nbytes + bs - 1) // bs
    out = torch.zeros(nb * 32, dtype=torch.uint8, device="cuda:0")
    ctx.hash_chunks_dev(data.data_ptr() + skew, nbytes, bs, out.data_ptr(), 0)
    torch.cuda.synchronize()
    host = data.cpu().numpy()[skew:].copy()
    want = oracle_chunks(oracle, host, nbytes, bs)
    assert first_bad(out.cpu().numpy(), want) is None


def test_uniform_loaders_agree(gpu, oracle):
    """The two uniform-kernel loaders (LDS-DMA and direct) vs the oracle."""
    import torch
    bs, nblk = 32768, 1024
    data = dev_random(gpu, bs * nblk, seed=99)
    outs = []
    for loader in (0, 1):
        out = torch.zeros(nblk * 32, dtype=torch.uint8, device="cuda:0")
        gpu._n.check(gpu._n.lib.cir_debug_hash_uniform_dev(loader, data.data_ptr(), bs, nblk,
                                                           out.data_ptr(), 0))
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
    want = oracle_chunks(oracle, data.cpu().numpy(), bs * nblk, bs)
    assert first_bad(outs[0], want) is None
    assert first_bad(outs[1], want) is None


def test_desc_mixed_ragged_shuffled(gpu, ctx, oracle):
    """Config-3 shape at small scale: 4 KiB / 32 KiB / 1 MiB classes, 10%
    ragged, empty and boundary lengths, shuffled, some misaligned offsets."""
    import torch
    rng = random.Random(0x5EED0003)
    lens = []
    for size, count in [(4096, 3000), (32768, 400), (1 << 20, 6)]:
        for _ in range(count):
            lens.append(rng.randrange(1, size) if rng.random() < 0.1 else size)
    lens += [0, 1, 127, 128, 129, 255, 256, 257, 0]
    rng.shuffle(lens)
    offs, pos = [], 0
    for i, ln in enumerate(lens):
        pos += (-pos) % 128 + (i % 7 if i % 5 == 0 else 0)
        offs.append(pos)
        pos += ln
    data = dev_random(gpu, pos, seed=3)
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * len(lens), dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                        out.data_ptr(), 0)
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    ao = np.array(offs, dtype=np.uint64)
    al = np.array(lens, dtype=np.uint32)
    want = np.zeros(32 * len(lens), dtype=np.uint8)
    oracle.oracle_hash_blocks(host.ctypes.data, ao.ctypes.data, al.ctypes.data, len(lens),
                              want.ctypes.data, 8)
    assert first_bad(out.cpu().numpy(), want) is None


def test_desc_large_batch_exclusive_quad(gpu, ctx, oracle):
    """A batch above the small-batch limit (>= 49153 descriptors) with long
    chains: the quad part runs SIMD-exclusive (k_quad_long<_, true>, launched
    before a delayed lane part), the rest in lane mode; chain lengths on both
    sides of the 1024-line threshold, odd and even line counts, ragged
    tails, 16-B aligned and misaligned starts."""
    import torch
    rng = random.Random(0xE5C1)
    q = 1024 * 128
    lens = [rng.choice([q - 128, q - 1, q, q + 1, q + 128, 2 * q + 77, 3 * q]) for _ in range(150)]
    lens += [rng.randrange(0, 8192) for _ in range(50000)]
    rng.shuffle(lens)
    offs, pos = [], 0
    for i, ln in enumerate(lens):
        pos += (-pos) % 16 + (3 if i % 11 == 0 else 0)
        offs.append(pos)
        pos += ln
    data = dev_random(gpu, pos, seed=41)
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * len(lens), dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                        out.data_ptr(), 0)
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    ao = np.array(offs, dtype=np.uint64)
    al = np.array(lens, dtype=np.uint32)
    want = np.zeros(32 * len(lens), dtype=np.uint8)
    oracle.oracle_hash_blocks(host.ctypes.data, ao.ctypes.data, al.ctypes.data, len(lens),
                              want.ctypes.data, 8)
    assert first_bad(out.cpu().numpy(), want) is None


def test_desc_paced_lane_part_single_workgroup(gpu, ctx, oracle):
    """Lane pacing at its extreme: 64 chains of 1 MiB (quad part) beside
    60000 chains of 0..200 bytes, so the paced lane part runs ~1 workgroup
    that strides over every short chain (k_lane_rest, count[2], count[4..5])."""
    import torch
    rng = random.Random(0x9ACE)
    lens = [1 << 20] * 64 + [rng.randrange(0, 201) for _ in range(60000)]
    rng.shuffle(lens)
    offs, pos = [], 0
    for i, ln in enumerate(lens):
        pos += (-pos) % 16 + (5 if i % 13 == 0 else 0)
        offs.append(pos)
        pos += ln
    data = dev_random(gpu, pos, seed=47)
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * len(lens), dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                        out.data_ptr(), 0)
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    ao = np.array(offs, dtype=np.uint64)
    al = np.array(lens, dtype=np.uint32)
    want = np.zeros(32 * len(lens), dtype=np.uint8)
    oracle.oracle_hash_blocks(host.ctypes.data, ao.ctypes.data, al.ctypes.data, len(lens),
                              want.ctypes.data, 8)
    assert first_bad(out.cpu().numpy(), want) is None


def test_desc_paced_lane_part_with_leftover(gpu, ctx, oracle):
    """Lane pacing with more lane work than the paced workgroups finish: 64
    chains of 1 MiB (the quad part) beside 60000 chains of ~64 KiB, ragged
    (an exclusive batch; ~59 paced workgroups hold ~15 K chains at a time,
    ~4 rounds of 512 compressions against the quad part's 8192), so the
    helper k_lane_rest queued behind the quad part typically claims the
    last tiles — every chain hashed exactly once either way."""
    import torch
    rng = random.Random(0x1EF7)
    lens = [1 << 20] * 64 + [65536 - rng.randrange(0, 3) * 128 - rng.randrange(0, 2) * 5
                             for _ in range(60000)]
    rng.shuffle(lens)
    offs, pos = [], 0
    for ln in lens:
        pos += (-pos) % 16
        offs.append(pos)
        pos += ln
    data = dev_random(gpu, pos, seed=53)
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * len(lens), dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                        out.data_ptr(), 0)
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    del data
    ao = np.array(offs, dtype=np.uint64)
    al = np.array(lens, dtype=np.uint32)
    want = np.zeros(32 * len(lens), dtype=np.uint8)
    oracle.oracle_hash_blocks(host.ctypes.data, ao.ctypes.data, al.ctypes.data, len(lens),
                              want.ctypes.data, 16)
    assert first_bad(out.cpu().numpy(), want) is None


def test_desc_quad_capacity_overflow(gpu, ctx, oracle):
    """More long chains than the quad part holds (n_long > 64 x 256 = 16384
    chains of >= 128 KiB in a batch of >= 49153): the longest 16384 chains of
    the sorted order run in quad mode, every other one (long ones included)
    in lane mode -- every chain hashed exactly once."""
    import torch
    rng = random.Random(0x0F10)
    q = 1024 * 128
    lens = [rng.choice([q, q + 1, q + 4096, 2 * q - 3]) for _ in range(17000)]
    lens += [rng.randrange(0, 4097) for _ in range(40000)]
    rng.shuffle(lens)
    offs, pos = [], 0
    for ln in lens:
        pos += (-pos) % 16
        offs.append(pos)
        pos += ln
    data = dev_random(gpu, pos, seed=43)
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * len(lens), dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                        out.data_ptr(), 0)
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    del data
    ao = np.array(offs, dtype=np.uint64)
    al = np.array(lens, dtype=np.uint32)
    want = np.zeros(32 * len(lens), dtype=np.uint8)
    oracle.oracle_hash_blocks(host.ctypes.data, ao.ctypes.data, al.ctypes.data, len(lens),
                              want.ctypes.data, 16)
    assert first_bad(out.cpu().numpy(), want) is None


@pytest.mark.parametrize("copy", ["direct", "nt"])
def test_host_blocks_many_batches(small_ctx, oracle, copy, monkeypatch):
    monkeypatch.setenv("CIR_STAGE_COPY", copy)  # the gather into the slots, both modes
    rng = random.Random(11)
    arena = os.urandom(6 << 20)
    n = 3000
    lens = [rng.choice([0, 1, 100, 4096, 32768, rng.randrange(0, 70000)]) for _ in range(n)]
    offs = [rng.randrange(0, len(arena) - ln + 1) for ln in lens]
    got = small_ctx.hash_blocks(arena, offs, lens)
    for i in range(n):
        assert got[32 * i:32 * i + 32] == oracle_digest(oracle, arena[offs[i]:offs[i] + lens[i]])


@pytest.mark.parametrize("size", [0, 1, 32767, 32768, 32769, 5 * 32768 + 3, (3 << 20) + 11])
def test_hash_file(small_ctx, oracle, tmp_path, size):
    data = os.urandom(size)
    p = tmp_path / "f.bin"
    p.write_bytes(data)
    with open(p, "rb") as f:
        got_size, hashes = small_ctx.hash_file(f.fileno(), 32768)
    assert got_size == size
    want = b"".join(oracle_digest(oracle, data[i:i + 32768]) for i in range(0, size, 32768))
    assert hashes == want
    assert small_ctx.hash_memory(data, 32768) == want


def test_hashes_api(gpu, oracle, tmp_path):
    data = os.urandom(100000)
    p = tmp_path / "x"
    p.write_bytes(data)
    with open(p, "rb") as f:
        size, hs = gpu.Hashes.hash_file(gpu.HashType.blake2b_256(), 4096, f)
    assert size == 100000 and len(hs) == 25 and hs.block_size() == 4096
    assert hs.get(24) == oracle_digest(oracle, data[24 * 4096:])


def make_tree(root):
    rng = random.Random(5)
    (root / "a" / "b" / "c").mkdir(parents=True)
    (root / "empty_dir").mkdir()
    (root / "z").mkdir()
    (root / "hello.txt").write_bytes(b"hello\n")
    (root / "test.txt").write_bytes(b"")
    (root / "a" / "big.bin").write_bytes(os.urandom(5 * 32768 + 1234))
    (root / "a" / "exact.bin").write_bytes(os.urandom(2 * 32768))
    (root / "a" / "b" / "run.sh").write_bytes(b"#!/bin/sh\necho hi\n")
    os.chmod(root / "a" / "b" / "run.sh", 0o755)
    (root / "a" / "b" / "c" / "deep").write_bytes(os.urandom(rng.randrange(1, 5000)))
    for i in range(60):
        (root / "z" / ("f%03d" % i)).write_bytes(os.urandom(rng.randrange(0, 70000)))
    (root / "z" / "with space").write_bytes(b"x")
    (root / "z" / "back\\slash").write_bytes(b"y")
    os.symlink("../hello.txt", root / "a" / "link")
    os.symlink("target with space", root / "dangling")


@pytest.mark.parametrize("copy", ["direct", "nt"])
def test_scan_vs_oracle(gpu, small_ctx, tmp_path, copy, monkeypatch):
    """v1::scan of a tree with every entry kind, at 1, 4 and auto reader
    threads, with the readers' two copy modes (pread straight into the
    pinned slot, or through a bounce buffer and streaming stores)."""
    monkeypatch.setenv("CIR_STAGE_COPY", copy)
    make_tree(tmp_path)
    want = dirsig_oracle.scan(str(tmp_path), 32768)
    for threads in (1, 4, 0):  # 0: auto_threads (the library's host_copy_threads)
        cfg = gpu.ScannerConfig.new().threads(threads).hash(gpu.HashType.blake2b_256())
        cfg.add_dir(str(tmp_path), "/")
        got = gpu.v1.scan(cfg, context=small_ctx)
        assert got == want, threads
    # block size other than the default
    cfg = gpu.ScannerConfig.new().block_size(4096).add_dir(str(tmp_path), "/")
    assert gpu.v1.scan(cfg, context=small_ctx) == dirsig_oracle.scan(str(tmp_path), 4096)


@pytest.mark.parametrize("block_size,hash_name", [
    (1, "blake2b/256"), (100, "blake2b/256"), (127, "blake2b/256"), (129, "blake2b/256"),
    (65537, "blake2b/256"), ((1 << 20) + 7, "blake2b/256"), (129, "sha512/256"),
    (65537, "sha512/256")])
def test_scan_odd_block_sizes(gpu, small_ctx, tmp_path, block_size, hash_name):
    """v1::scan with block sizes that are not multiples of the 128-B line
    (every block then ends in a partial line; size 1 makes one chain per byte)
    and above the staging granularity, against the scan oracle."""
    if block_size == 1:  # one digest (65 index bytes) per file byte: a small tree
        (tmp_path / "d").mkdir()
        for i, n in enumerate((0, 1, 2, 127, 128, 129, 300)):
            (tmp_path / "d" / ("f%d" % i)).write_bytes(os.urandom(n))
        (tmp_path / "top").write_bytes(b"xyz")
    else:
        make_tree(tmp_path)
    ht = gpu.HashType.blake2b_256() if hash_name == "blake2b/256" else gpu.HashType.sha512_256()
    cfg = gpu.ScannerConfig.new().block_size(block_size).threads(4).hash(ht)
    cfg.add_dir(str(tmp_path), "/")
    want = dirsig_oracle.scan(str(tmp_path), block_size, hash_name)
    assert gpu.v1.scan(cfg, context=small_ctx) == want


def test_sync_flow_register_and_serve(gpu, small_ctx, tmp_path):
    """scan -> register_index -> register_dir -> read_block of every block
    (src/client/sync/uploads.rs:70-78), and the daemon-side invariant
    BlockHash::hash_bytes(block) == index hash (fetch_blocks.rs:77)."""
    make_tree(tmp_path)
    cfg = gpu.ScannerConfig.new().add_dir(str(tmp_path), "/")
    buf = bytearray()
    gpu.v1.scan(cfg, buf, context=small_ctx)
    index = bytes(buf)
    idxs = gpu.InMemoryIndexes()
    image_id = idxs.register_index(index)
    hash_name, bs, dirs, footer = dirsig_oracle.parse(index)
    assert bytes(image_id) == footer
    assert footer == dirsig_oracle.h_blake2b256(index[index.index(b"\n") + 1:-65])
    reader = gpu.ThreadedBlockReader()
    reader.register_dir(str(tmp_path), index)
    n = 0
    for _, entries in dirs:
        for e in entries:
            if e[0] == "f":
                for d in e[4]:
                    block = reader.read_block(gpu.BlockHash(d), gpu.BlockHint.empty())
                    assert bytes(gpu.BlockHash.hash_bytes(block)) == d
                    n += 1
    assert n >= len(reader)  # equal blocks share one entry


def test_index_rewrite_roundtrip(gpu, small_ctx, tmp_path):
    """RawIndex::into_mut + to_raw_data == input (the reference's own
    `roundtrip` test, src/cluster/download.rs:368-382, on a blake2b index)."""
    make_tree(tmp_path)
    os.rmdir(tmp_path / "empty_dir")  # the re-emitter drops empty directories
    cfg = gpu.ScannerConfig.new().add_dir(str(tmp_path), "/")
    index = gpu.v1.scan(cfg, context=small_ctx)
    assert small_ctx.index_rewrite(index) == index
    # the footer on the GPU chain (one descriptor) gives the same bytes
    small_ctx.set_footer_mode(small_ctx.FOOTER_GPU)
    try:
        assert small_ctx.index_rewrite(index) == index
    finally:
        small_ctx.set_footer_mode(small_ctx.FOOTER_HOST)


def test_memory_blocks(gpu, oracle):
    data = os.urandom(int(2.5 * 4096))
    r = gpu.ThreadedBlockReader()
    r.register_memory_blocks(gpu.HashType.blake2b_256(), 4096, data)
    assert len(r) == 3
    for i in range(3):
        blk = data[i * 4096:(i + 1) * 4096]
        assert r.read_block(oracle_digest(oracle, blk)) == blk


@pytest.mark.parametrize("teardown", ["0", "1"])
def test_cli_sync(gpu, tmp_path, teardown):
    """One `ciruela-index sync` process; by default it leaves its context to
    process exit (`_exit` after flushing), CIR_CLI_TEARDOWN=1 destroys it
    first: both print the same line and write the same index."""
    import subprocess
    from conftest import ROOT
    make_tree(tmp_path / "src")
    env = dict(os.environ, CIR_CLI_TEARDOWN=teardown)
    p = subprocess.run([os.path.join(ROOT, "bin", "ciruela-index"), "sync",
                        "--append", str(tmp_path / "src") + ":/dest",
                        "--index-dir", str(tmp_path)], env=env, capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr
    image_id, kind, dest, src = p.stdout.decode().split()
    want = dirsig_oracle.scan(str(tmp_path / "src"), 32768)
    assert (tmp_path / (image_id + ".ds1")).read_bytes() == want
    assert kind == "append" and dest == "/dest"
    assert want.endswith(image_id.encode() + b"\n")
    assert b"Indexed" in p.stderr


def test_cli_sync_several_jobs(gpu, tmp_path):
    """Several `--append` / `--append-weak` / `--replace` jobs in one
    `ciruela-index sync` (src/client/sync/mod.rs:168-220 walks its uploads
    the same way): one line per job in order, each index the scan oracle's
    for its own directory, a block size given with --block-size, a one-shot
    context for the jobs' total input (CIR_TRACE)."""
    import subprocess
    from conftest import ROOT
    rng = random.Random(0xC11)
    srcs = []
    for k in range(3):
        d = tmp_path / ("src%d" % k)
        d.mkdir()
        for i in range(rng.randrange(1, 8)):
            (d / ("f%d" % i)).write_bytes(rng.randbytes(rng.randrange(0, 200000)))
        srcs.append(d)
    args = [os.path.join(ROOT, "bin", "ciruela-index"), "sync", "--block-size", "65536",
            "--append", "%s:/a" % srcs[0], "--append-weak", "%s:/b/c" % srcs[1],
            "--replace", "%s:/d" % srcs[2], "--index-dir", str(tmp_path)]
    p = subprocess.run(args, env=dict(os.environ, CIR_TRACE="1"), capture_output=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr
    lines = [ln.split() for ln in p.stdout.decode().splitlines()]
    assert [(ln[1], ln[2], ln[3]) for ln in lines] == [
        ("append", "/a", str(srcs[0])), ("append-weak", "/b/c", str(srcs[1])),
        ("replace", "/d", str(srcs[2]))]
    for ln, src in zip(lines, srcs):
        want = dirsig_oracle.scan(str(src), 65536)
        assert (tmp_path / (ln[0] + ".ds1")).read_bytes() == want
        assert want.endswith(ln[0].encode() + b"\n")
    assert p.stderr.count(b"Indexed") == 3
    assert b"1 device(s) for" in p.stderr


def test_cli_exits_normally_under_a_profiler(gpu, tmp_path):
    """With a profiler's environment (ROCPROF_* / ROCP_TOOL_LIBRARIES, as
    rocprofv3 sets for its tool library) `ciruela-index` skips cir_destroy
    but returns from main, so exit handlers -- where the tool writes its
    trace -- still run; the output is the same."""
    import subprocess
    from conftest import ROOT
    make_tree(tmp_path / "src")
    env = dict(os.environ, CIR_TRACE="1", ROCPROF_CIRUELA_TEST="1")
    p = subprocess.run([os.path.join(ROOT, "bin", "ciruela-index"), "sync",
                        "--append", str(tmp_path / "src") + ":/dest"], env=env,
                       capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert b"profiler present: normal exit" in p.stderr
    assert b"blit copies" in p.stderr  # a small input skips the SDMA engines' start-up
    want = dirsig_oracle.scan(str(tmp_path / "src"), 32768)
    assert want.endswith(p.stdout.split()[0] + b"\n")


def test_cli_hash(gpu, oracle, tmp_path):
    """`ciruela-index hash FILE...` (the per-file Hashes::hash_file list):
    every line -- path, size, one digest per block -- equal to the oracle,
    through a pipe (stdout fully buffered, flushed before the process exits
    without tearing its context down)."""
    import subprocess
    from conftest import ROOT
    sizes = [0, 1, 4096, 4097, 3 * 4096 + 100]
    paths = []
    for i, n in enumerate(sizes):
        f = tmp_path / ("f%d" % i)
        f.write_bytes(os.urandom(n))
        paths.append(str(f))
    p = subprocess.run([os.path.join(ROOT, "bin", "ciruela-index"), "hash", "--block-size", "4096"]
                       + paths, capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr
    lines = p.stdout.decode().splitlines()
    assert len(lines) == len(paths)
    for path, n, line in zip(paths, sizes, lines):
        data = open(path, "rb").read()
        want = [oracle_digest(oracle, data[k:k + 4096]).hex() for k in range(0, n, 4096)]
        assert line.split() == [path, str(n)] + want, path


@pytest.mark.parametrize("mib,states", [(300, 1), (520, 2), (0, 1)])
def test_cli_opens_devices_for_its_input(gpu, tmp_path, mib, states):
    """`ciruela-index sync` opens ceil(input / (2 x 256 MiB)) devices
    (cir_devices_for_bytes + cir_init_n), not every GPU of the node: on the
    one-GPU box CIR_DEBUG_SPLIT=4 offers four device states, and a 300 MiB
    tree takes one, a 520 MiB tree two, a tree of empty files one (0 bytes
    is a measured size, not cir_devices_for_bytes' "unknown").  The index is
    the scan oracle's either way (sparse files: the bytes are zeros, the
    sizes are real)."""
    import subprocess
    from conftest import ROOT
    src = tmp_path / "src"
    (src / "d").mkdir(parents=True)
    per = (mib << 20) // 4
    for k in range(4):
        with open(src / "d" / ("f%d" % k), "wb") as f:
            f.truncate(per + 1000 * k if mib else 0)
    env = dict(os.environ, CIR_DEBUG_SPLIT="4", CIR_TRACE="1")
    p = subprocess.run([os.path.join(ROOT, "bin", "ciruela-index"), "sync",
                        "--append", str(src) + ":/dest", "--index-dir", str(tmp_path)],
                       env=env, capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    if mib:
        assert "SDMA copies" in p.stderr.decode()  # a large input keeps the link's full rate
    total = 4 * per + 6000 if mib else 0
    line = [ln for ln in p.stderr.decode().splitlines() if "device(s) for" in ln]
    assert line and (" %d device(s) for %d input bytes" % (states, total)) in line[0], line
    image_id = p.stdout.decode().split()[0]
    want = dirsig_oracle.scan(str(src), 32768)
    assert (tmp_path / (image_id + ".ds1")).read_bytes() == want


def test_context_device_hint(gpu, monkeypatch):
    """cir_init_n: at most max_devices of the masked device states."""
    monkeypatch.setenv("CIR_DEBUG_SPLIT", "3")
    c = gpu.Context(device_mask=1, staging_bytes=1 << 20, max_devices=2)
    c0 = gpu.Context(device_mask=1, staging_bytes=1 << 20)
    monkeypatch.delenv("CIR_DEBUG_SPLIT")
    assert len(c.devices()) == 2 and len(c0.devices()) == 3
    data = os.urandom(3 << 20)
    assert c.hash_memory(data, 32768) == c0.hash_memory(data, 32768)
    c.close()
    c0.close()


def test_one_shot_context(gpu, oracle, tmp_path):
    """CIR_INIT_ONE_SHOT (the CLI's context for a small input): one stream
    and one staging slot.  Every path still runs and matches the oracle: a
    config-3-shaped descriptor batch and an exclusive-quad batch (the quad
    part behind the lane part on the one stream, no relay), a ragged file on
    the device, host batches over several slots (allocated on demand), a scan
    with the GPU footer (its chain stream created on demand) and verify."""
    with gpu.Context(device_mask=1, staging_bytes=1 << 20, one_shot=True) as c:
        one_shot_paths(gpu, c, oracle, tmp_path)
    with pytest.raises(gpu.CiruelaError):  # closed: the handle is gone
        c.hash_memory(b"x", 4096)


def one_shot_paths(gpu, c, oracle, tmp_path):
    test_desc_mixed_ragged_shuffled(gpu, c, oracle)
    test_desc_large_batch_exclusive_quad(gpu, c, oracle)
    test_chunks_dev_vs_oracle(gpu, c, oracle, 32768, 32768 * 4099 + 77)
    rng = random.Random(0x1D)
    arena = rng.randbytes(5 << 20)
    offs = list(range(0, len(arena) - 32768, 32768))
    lens = [32768 - (i % 3) for i in range(len(offs))]
    want = b"".join(oracle_digest(oracle, arena[o:o + ln]) for o, ln in zip(offs, lens))
    assert c.hash_blocks(arena, offs, lens) == want
    assert c.hash_memory(arena, 4096) == b"".join(
        oracle_digest(oracle, arena[i:i + 4096]) for i in range(0, len(arena), 4096))
    exp = bytearray(want)
    exp[32 * 7] ^= 1
    assert c.verify_blocks(arena, offs, lens, bytes(exp)) == [i != 7 for i in range(len(offs))]
    t = c.verify_submit(arena[:32768], want[:32])
    assert c.verify_wait(t) is True
    root = tmp_path / "tree"
    make_tree(root)
    for mode in (c.FOOTER_GPU, c.FOOTER_HOST):
        c.set_footer_mode(mode)
        cfg = gpu.ScannerConfig.new().block_size(32768)
        cfg.add_dir(str(root), "/")
        assert gpu.v1.scan(cfg, context=c) == dirsig_oracle.scan(str(root), 32768, "blake2b/256")


def test_sha512_256_single_and_batches(gpu, ctx, oracle):
    """dir-signature's second hash type on the GPU vs the oracle."""
    import torch
    sha = gpu.HashType.sha512_256()
    for n in [0, 1, 7, 111, 112, 113, 127, 128, 129, 239, 240, 255, 256, 1000, 32768]:
        d = os.urandom(n)
        assert gpu.sha512_256(d) == oracle_sha(oracle, d), n
    rng = random.Random(9)
    lens = [rng.choice([0, 1, 111, 112, 128, 4096, 32768, rng.randrange(0, 70000)])
            for _ in range(1500)]
    arena = os.urandom(sum(lens) + 64)
    offs, pos = [], 0
    for ln in lens:
        offs.append(pos)
        pos += ln
    got = ctx.hash_blocks(arena, offs, lens, hash_type=sha)
    for i in range(0, len(lens), 7):
        assert got[32 * i:32 * i + 32] == oracle_sha(oracle, arena[offs[i]:offs[i] + lens[i]]), i
    # device-resident descriptors
    t = torch.tensor(bytearray(arena), dtype=torch.uint8, device="cuda:0")
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * len(lens), dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev(t.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                        out.data_ptr(), 0, hash_type=sha)
    torch.cuda.synchronize()
    assert out.cpu().numpy().tobytes() == got
    data = os.urandom(5 * 32768 + 17)
    assert ctx.hash_memory(data, 32768, hash_type=sha) == b"".join(
        oracle_sha(oracle, data[i:i + 32768]) for i in range(0, len(data), 32768))


def test_reference_roundtrip_fixture_on_gpu(gpu, small_ctx, dirsig_example):
    """The reference's own test, src/cluster/download.rs:368-382 (`roundtrip`):
    RawIndex::into_mut + to_raw_data reproduces EXAMPLE byte for byte -- here
    parsed, re-emitted and re-footed (SHA-512/256 on the GPU)."""
    idx = dirsig_example["index"].encode()
    assert small_ctx.index_rewrite(idx) == idx


def test_scan_sha512(gpu, small_ctx, tmp_path):
    make_tree(tmp_path)
    cfg = gpu.ScannerConfig.new().hash(gpu.HashType.sha512_256()).add_dir(str(tmp_path), "/")
    assert gpu.v1.scan(cfg, context=small_ctx) == \
        dirsig_oracle.scan(str(tmp_path), 32768, hash_name="sha512/256")


def _corrupt(b, i):
    return b[:i] + bytes([b[i] ^ 0x01]) + b[i + 1:]


@pytest.mark.parametrize("ht", ["blake2b", "sha512"])
def test_verify_blocks_host_and_device(gpu, ctx, oracle, ht):
    """Row f2: fetch_blocks.rs:77 `hash_bytes(&data) == blk.hash`, batched."""
    import torch
    hasht = gpu.HashType.blake2b_256() if ht == "blake2b" else gpu.HashType.sha512_256()
    dig = (lambda d: oracle_digest(oracle, d)) if ht == "blake2b" else \
        (lambda d: oracle_sha(oracle, d))
    rng = random.Random(21)
    lens = [rng.choice([0, 1, 127, 128, 4096, 32768, rng.randrange(0, 40000)])
            for _ in range(700)]
    arena = os.urandom(sum(lens) + 16)
    offs, pos = [], 0
    for ln in lens:
        offs.append(pos)
        pos += ln
    expected = b"".join(dig(arena[o:o + ln]) for o, ln in zip(offs, lens))
    bad = set(rng.sample(range(len(lens)), 37))
    exp_bad = expected
    for b in bad:
        exp_bad = _corrupt(exp_bad, 32 * b + rng.randrange(32))
    assert ctx.verify_blocks(arena, offs, lens, expected, hash_type=hasht) == [True] * len(lens)
    ok = ctx.verify_blocks(arena, offs, lens, exp_bad, hash_type=hasht)
    assert [i for i, g in enumerate(ok) if not g] == sorted(bad)
    # device-resident: received blocks in HBM, expected digests in HBM
    t = torch.tensor(bytearray(arena), dtype=torch.uint8, device="cuda:0")
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    d_exp = torch.tensor(bytearray(exp_bad), dtype=torch.uint8, device="cuda:0")
    d_dig = torch.zeros(32 * len(lens), dtype=torch.uint8, device="cuda:0")
    d_ok = torch.full((len(lens),), 7, dtype=torch.uint8, device="cuda:0")
    d_nbad = torch.full((1,), 12345, dtype=torch.int32, device="cuda:0")
    ctx.verify_blocks_dev(t.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                          d_exp.data_ptr(), d_dig.data_ptr(), d_ok.data_ptr(),
                          d_nbad.data_ptr(), hash_type=hasht)
    torch.cuda.synchronize()
    assert d_dig.cpu().numpy().tobytes() == expected
    assert [i for i, g in enumerate(d_ok.cpu().tolist()) if g != 1] == sorted(bad)
    assert set(d_ok.cpu().tolist()) <= {0, 1}
    assert int(d_nbad.item()) == len(bad)


def test_check_file_commit(gpu, small_ctx, tmp_path):
    """Row f2: Hashes::check_file at commit (src/daemon/disk/commit.rs:104)."""
    data = os.urandom(3 * 32768 + 999)
    p = tmp_path / "f"
    p.write_bytes(data)
    for ht in (gpu.HashType.blake2b_256(), gpu.HashType.sha512_256()):
        with open(p, "rb") as f:
            size, hashes = gpu.Hashes.hash_file(ht, 32768, f, context=small_ctx)
        assert size == len(data) and len(hashes) == 4
        with open(p, "rb") as f:
            assert hashes.check_file(f, context=small_ctx)
        for bad in (_corrupt(data, 40000), data[:-1], data + b"x", data[:3 * 32768]):
            q = tmp_path / "g"
            q.write_bytes(bad)
            with open(q, "rb") as f:
                assert not hashes.check_file(f, context=small_ctx)
    empty = tmp_path / "e"
    empty.write_bytes(b"")
    with open(empty, "rb") as f:
        assert gpu.Hashes(b"", 32768).check_file(f, context=small_ctx)


@pytest.mark.parametrize("aligned", [True, False])
def test_desc_quad_fast_loop_edges(gpu, ctx, oracle, aligned):
    """The hand-scheduled quad loop (quad_fast) at its edges: a small batch
    (every chain of >= 8 lines in quad mode) whose waves mix chains of 8..40
    lines, exact multiples of 128 (the last full line is the final one) and
    ragged tails, so the wave-uniform count nu lands on 0, 6, 8 (the loop's
    minimum) and above, with the rest of each chain in the general loop;
    with misaligned starts every wave falls back to the general loop."""
    import torch
    rng = random.Random(0xFA57 + aligned)
    lens = []
    for _ in range(900):
        lines = rng.randrange(8, 41)
        lens.append(lines * 128 - rng.choice([0, 0, 1, 64, 127]))
    lens += [9 * 128, 9 * 128 + 1, 10 * 128, 8 * 128, 8 * 128 + 1, 17 * 128 - 1]
    rng.shuffle(lens)
    offs, pos = [], 0
    for i, ln in enumerate(lens):
        pos += (-pos) % 16 + (0 if aligned else (i % 7) + 1)
        offs.append(pos)
        pos += ln
    data = dev_random(gpu, pos, seed=61 + aligned)
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * len(lens), dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                        out.data_ptr(), 0)
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    want = np.zeros(32 * len(lens), dtype=np.uint8)
    ao = np.array(offs, dtype=np.uint64)
    al = np.array(lens, dtype=np.uint32)
    oracle.oracle_hash_blocks(host.ctypes.data, ao.ctypes.data, al.ctypes.data, len(lens),
                              want.ctypes.data, 8)
    assert first_bad(out.cpu().numpy(), want) is None


@pytest.mark.parametrize("bs", [8 * 128, 9 * 128, 10 * 128 + 5, 4096])
def test_chunks_quad_fast_loop_block_sizes(gpu, ctx, oracle, bs):
    """Chunk-form files in quad mode with blocks of 8 / 9 / 10+ lines: the
    fast loop's count nu is 6 (loop skipped), 8 (its minimum) and 10, plus
    a short last block."""
    import torch
    nbytes = 3000 * bs + 333
    data = dev_random(gpu, nbytes, seed=bs)
    nb = (nbytes + bs - 1) // bs
    out = torch.zeros(nb * 32, dtype=torch.uint8, device="cuda:0")
    ctx.hash_chunks_dev(data.data_ptr(), nbytes, bs, out.data_ptr(), 0)
    torch.cuda.synchronize()
    want = oracle_chunks(oracle, data.cpu().numpy(), nbytes, bs)
    assert first_bad(out.cpu().numpy(), want) is None


def test_desc_quad_mode_edges(gpu, ctx, oracle):
    """Chains around the quad-mode threshold (1024 lines = 128 KiB) and long
    ragged chains: 37 long chains (a partial 16-chain wave), misaligned and
    128-aligned starts, final lines of 1..127 bytes, next to short chains
    that share the launch (k_quad_long + k_lane_rest)."""
    import torch
    q = 1024 * 128  # kQuadMinLines (kernels.hpp)
    rng = random.Random(0x9A4D)
    lens = [q - 1, q, q + 1, q + 127, q + 128, q + 129, 2 * q - 1, 2 * q, 2 * q + 1,
            1 << 20, (1 << 20) + 5, (3 << 20) + 77]
    lens += [rng.randrange(q, 2 << 20) for _ in range(25)]
    lens += [rng.choice([0, 1, 128, 4096, 32768, rng.randrange(1, 70000)]) for _ in range(500)]
    rng.shuffle(lens)
    offs, pos = [], 0
    for i, ln in enumerate(lens):
        pos += (-pos) % 16 + (i % 5)
        offs.append(pos)
        pos += ln
    data = dev_random(gpu, pos, seed=17)
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * len(lens), dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                        out.data_ptr(), 0)
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    want = np.zeros(32 * len(lens), dtype=np.uint8)
    ao = np.array(offs, dtype=np.uint64)  # kept alive across the call
    al = np.array(lens, dtype=np.uint32)
    oracle.oracle_hash_blocks(host.ctypes.data, ao.ctypes.data, al.ctypes.data, len(lens),
                              want.ctypes.data, 8)
    assert first_bad(out.cpu().numpy(), want) is None


@pytest.mark.parametrize("mode,hash_name", [("host", "blake2b/256"), ("gpu", "blake2b/256"),
                                            ("host", "sha512/256"), ("gpu", "sha512/256")])
def test_scan_long_index_footer(gpu, small_ctx, tmp_path, mode, hash_name):
    """An index body of several MiB (128-byte blocks): the footer is fed in
    stretches while later batches hash -- to the host thread (scan.cpp
    HostFooter, the default, both hash types) or, for blake2b, to the device
    chain in >= 256 KiB pieces (FooterChain); a sha512/256 footer in GPU mode
    is one lane at the end -- and must still equal H(body)
    (src/index.rs:98-105)."""
    rng = random.Random(5)
    for k in range(6):
        (tmp_path / ("f%d.bin" % k)).write_bytes(rng.randbytes(rng.randrange(1 << 20, 3 << 20)))
    ht = gpu.HashType.sha512_256() if hash_name == "sha512/256" else gpu.HashType.blake2b_256()
    cfg = gpu.ScannerConfig.new().block_size(128).hash(ht).add_dir(str(tmp_path), "/")
    small_ctx.set_footer_mode(small_ctx.FOOTER_HOST if mode == "host" else small_ctx.FOOTER_GPU)
    small_ctx.scan_timing(True)
    try:
        got = gpu.v1.scan(cfg, context=small_ctx)
        ph = small_ctx.scan_phases()
    finally:
        small_ctx.scan_timing(False)
        small_ctx.set_footer_mode(small_ctx.FOOTER_HOST)
    assert len(got) > (4 << 20)
    assert got == dirsig_oracle.scan(str(tmp_path), 128, hash_name)
    assert ph["footer_mode"] == (0 if mode == "host" else 1)
    if mode == "host" or hash_name == "blake2b/256":
        assert ph["footer_feeds"] >= 3 and ph["footer_busy_ms"] > 0  # fed while the scan ran
    assert ph["index_bytes"] == len(got)


class CountingBuffer(bytearray):
    """A bytearray that counts the appends cir_scan_v1_write makes into it."""
    pieces = 0

    def extend(self, data):
        self.pieces += 1
        super().extend(data)


@pytest.mark.parametrize("hash_name", ["blake2b/256", "sha512/256"])
@pytest.mark.parametrize("mode", ["host", "gpu"])
def test_scan_written_as_it_goes(gpu, small_ctx, tmp_path, mode, hash_name):
    """cir_scan_v1_write (v1::scan into the caller's Vec, src/client/sync/
    uploads.rs:55-57): a several-MiB index arrives in many pieces while the
    batches run -- header first, the footer line last -- and equals the
    oracle's index byte for byte with either footer placement (the library
    keeps only the unwritten tail; a sha512/256 footer in GPU mode keeps the
    whole body for its one-lane hash at the end)."""
    rng = random.Random(6)
    for k in range(6):
        (tmp_path / ("f%d.bin" % k)).write_bytes(rng.randbytes(rng.randrange(1 << 20, 3 << 20)))
    ht = gpu.HashType.sha512_256() if hash_name == "sha512/256" else gpu.HashType.blake2b_256()
    cfg = gpu.ScannerConfig.new().block_size(128).hash(ht).add_dir(str(tmp_path), "/")
    small_ctx.set_footer_mode(small_ctx.FOOTER_HOST if mode == "host" else small_ctx.FOOTER_GPU)
    small_ctx.scan_timing(True)
    try:
        out = CountingBuffer(b"keep:")  # appended to, as the reference's Vec
        assert gpu.v1.scan(cfg, out=out, context=small_ctx) is None
        ph = small_ctx.scan_phases()
    finally:
        small_ctx.scan_timing(False)
        small_ctx.set_footer_mode(small_ctx.FOOTER_HOST)
    want = dirsig_oracle.scan(str(tmp_path), 128, hash_name)
    assert bytes(out) == b"keep:" + want
    assert out.pieces >= 4, out.pieces
    assert ph["index_bytes"] == len(want)


def test_scan_writer_failure_is_an_io_error(gpu, small_ctx, tmp_path):
    """A writer that fails (the reference's io::Error from the Vec/Write)
    stops the scan: the exception comes back to the caller, the C status is
    CIR_EIO, and the context scans normally afterwards."""
    n = gpu._n
    rng = random.Random(8)
    for k in range(4):
        (tmp_path / ("f%d.bin" % k)).write_bytes(rng.randbytes(1 << 20))
    cfg = gpu.ScannerConfig.new().block_size(1024).add_dir(str(tmp_path), "/")

    class Full(bytearray):
        def extend(self, data):
            if len(self) > 0:
                raise OSError(28, "No space left on device")
            super().extend(data)
    with pytest.raises(OSError):
        gpu.v1.scan(cfg, out=Full(), context=small_ctx)
    calls = []

    @n.WRITE_FN
    def refuse(_user, _data, _n):
        calls.append(1)
        return 7
    dirs = (ctypes.c_char_p * 1)(os.fsencode(str(tmp_path)))
    pres = (ctypes.c_char_p * 1)(b"/")
    rc = n.lib.cir_scan_v1_write(small_ctx.handle, dirs, pres, 1, 1024, 1, 0, refuse, None, None)
    assert rc == n.CIR_EIO and calls == [1]
    out = bytearray()
    gpu.v1.scan(cfg, out=out, context=small_ctx)
    assert bytes(out) == dirsig_oracle.scan(str(tmp_path), 1024)


def test_scan_timing_rows(gpu, tmp_path):
    """cir_debug_scan_timing: one row per staged batch (bytes add up to the
    tree's, block counts to its blocks), each batch's events in order (reads,
    then upload, then hash and digests back), and a phase record per scan."""
    ctx = gpu.Context(device_mask=1, staging_bytes=4 << 20)
    rng = random.Random(9)
    sizes = [rng.randrange(0, 3 << 20) for _ in range(20)]
    for k, n in enumerate(sizes):
        (tmp_path / ("f%02d" % k)).write_bytes(rng.randbytes(n))
    cfg = gpu.ScannerConfig.new().threads(4).add_dir(str(tmp_path), "/")
    ctx.scan_timing(True)
    got = gpu.v1.scan(cfg, context=ctx)
    rows, ph = ctx.scan_batches(), ctx.scan_phases()
    ctx.scan_timing(False)
    assert got == dirsig_oracle.scan(str(tmp_path), 32768)
    assert len(rows) == ph["batches"] >= 5
    assert sum(r["blocks"] for r in rows) == sum((n + 32767) // 32768 for n in sizes)
    assert sum(r["bytes"] for r in rows) >= sum(sizes)  # + 16-B alignment of file segments
    eps = 0.05  # ms: event vs host clock
    for r in rows:
        assert r["device"] == 0
        assert 0 <= r["read_start_ms"] <= r["read_end_ms"] <= r["h2d_start_ms"] + eps
        assert r["h2d_start_ms"] <= r["h2d_end_ms"] <= r["hash_start_ms"] + eps
        assert r["hash_start_ms"] <= r["done_ms"]
    assert ph["hash_loop_ms"] > 0 and ph["footer_mode"] == 0
    # off: a later scan records nothing
    gpu.v1.scan(cfg, context=ctx)
    assert len(ctx.scan_batches()) == len(rows)


def test_lazy_staging_context(gpu, oracle):
    """CIR_STAGING_LAZY: cir_init pins no staging slots (the device-resident
    line of every rank of a multi-GPU run), the *_dev entry points work at
    once, and the first host-path call allocates the slots itself."""
    import torch

    def rss():
        with open("/proc/self/status") as f:
            return next(int(ln.split()[1]) << 10 for ln in f if ln.startswith("VmRSS:"))
    gpu.Context(device_mask=1, staging_bytes=1 << 20).close()  # runtime warm-up
    r0 = rss()
    c = gpu.Context(device_mask=1, staging_bytes=gpu._n.CIR_STAGING_LAZY)
    assert rss() - r0 < (96 << 20), (rss() - r0) >> 20  # an eager context pins 768 MiB
    data = dev_random(gpu, 1 << 20, 0x1A2)
    out = torch.empty(32 * 32, dtype=torch.uint8, device="cuda:0")
    c.hash_chunks_dev(data.data_ptr(), 1 << 20, 32768, out.data_ptr(), 0)
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    assert first_bad(out.cpu().numpy(), oracle_chunks(oracle, host, 1 << 20, 32768)) is None
    blob = host.tobytes()
    assert c.hash_memory(blob, 4096) == b"".join(
        oracle_digest(oracle, blob[i:i + 4096]) for i in range(0, len(blob), 4096))
    c.close()


def test_concurrent_callers_one_context(gpu, small_ctx, oracle):
    """The ABI is callable from several host threads at once on one context
    (the scan's worker threads, the daemon's fetch and commit tasks): host
    batches, in-memory files and device batches on distinct streams."""
    import threading

    import torch
    rng = random.Random(77)
    arena = rng.randbytes(3 << 20)
    jobs, errors = [], []

    def host_blocks(seed):
        r = random.Random(seed)
        lens = [r.choice([0, 1, 4096, 32768, r.randrange(1, 300000)]) for _ in range(300)]
        offs = [r.randrange(0, len(arena) - ln + 1) for ln in lens]
        got = small_ctx.hash_blocks(arena, offs, lens)
        for i in range(len(lens)):
            if got[32 * i:32 * i + 32] != oracle_digest(oracle, arena[offs[i]:offs[i] + lens[i]]):
                errors.append(("blocks", seed, i))
                return

    def device_blocks(seed):
        r = random.Random(seed)
        lens = [r.choice([128, 32768, 200000, r.randrange(1, 70000)]) for _ in range(200)]
        offs = [r.randrange(0, len(arena) - ln + 1) for ln in lens]
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            data = torch.frombuffer(bytearray(arena), dtype=torch.uint8).to("cuda:0")
            d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
            d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
            out = torch.zeros(32 * len(lens), dtype=torch.uint8, device="cuda:0")
        small_ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                                  out.data_ptr(), s.cuda_stream)
        s.synchronize()
        got = out.cpu().numpy().tobytes()
        for i in range(len(lens)):
            if got[32 * i:32 * i + 32] != oracle_digest(oracle, arena[offs[i]:offs[i] + lens[i]]):
                errors.append(("device", seed, i))
                return

    for k in range(4):
        jobs.append(threading.Thread(target=host_blocks, args=(k,)))
        jobs.append(threading.Thread(target=device_blocks, args=(100 + k,)))
    for t in jobs:
        t.start()
    for t in jobs:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in jobs)
    assert errors == []


@pytest.mark.parametrize("copy", ["direct", "nt"])
def test_hash_file_parallel_reads_offset_and_pipe(ctx, oracle, tmp_path, copy, monkeypatch):
    """Regular files are read with pread by several threads per staging batch
    starting at the fd's current offset, which ends at EOF (the reference
    reads the Read object to its end); pipes go through plain read().  Both
    staging copy modes (CIR_STAGE_COPY)."""
    monkeypatch.setenv("CIR_STAGE_COPY", copy)
    import threading
    bs = 32768
    data = os.urandom((21 << 20) + 5)
    p = tmp_path / "big.bin"
    p.write_bytes(data)
    with open(p, "rb") as f:
        f.seek(1000)
        size, hashes = ctx.hash_file(f.fileno(), bs)
        assert os.lseek(f.fileno(), 0, os.SEEK_CUR) == len(data)
    tail = data[1000:]
    assert size == len(tail)
    assert hashes == b"".join(oracle_digest(oracle, tail[i:i + bs]) for i in range(0, len(tail), bs))
    rfd, wfd = os.pipe()
    payload = data[:(5 << 20) + 77]

    def writer():
        with os.fdopen(wfd, "wb") as w:
            w.write(payload)
    t = threading.Thread(target=writer)
    t.start()
    try:
        size, hashes = ctx.hash_file(rfd, bs)
    finally:
        t.join()
        os.close(rfd)
    assert size == len(payload)
    assert hashes == b"".join(oracle_digest(oracle, payload[i:i + bs])
                              for i in range(0, len(payload), bs))


def test_multi_device_split_paths(gpu, oracle, tmp_path):
    """The host paths' multi-device splits (one contiguous
    block range per device for hash_memory / hash_file / hash_blocks, stripes
    dealt round-robin for a scan; one thread per device), run on one GPU
    through CIR_DEBUG_SPLIT=3 (the GPU appears as three independent device
    states): hash_memory, hash_file from an offset, hash_blocks, and a
    directory scan whose footer is fed from the device threads, with the
    default stripes and with stripes of 3 blocks."""
    os.environ["CIR_DEBUG_SPLIT"] = "3"
    try:
        ctx = gpu.Context(device_mask=1, staging_bytes=1 << 20)
    finally:
        del os.environ["CIR_DEBUG_SPLIT"]
    assert len(ctx.devices()) == 3
    rng = random.Random(33)
    bs = 32768
    data = rng.randbytes((10 << 20) + 5)
    want = b"".join(oracle_digest(oracle, data[i:i + bs]) for i in range(0, len(data), bs))
    assert ctx.hash_memory(data, bs) == want
    p = tmp_path / "f.bin"
    p.write_bytes(data)
    with open(p, "rb") as f:
        f.seek(100)
        size, hashes = ctx.hash_file(f.fileno(), bs)
        assert os.lseek(f.fileno(), 0, os.SEEK_CUR) == len(data)
    assert size == len(data) - 100
    assert hashes == b"".join(oracle_digest(oracle, data[100 + i:100 + i + bs])
                              for i in range(0, len(data) - 100, bs))
    lens = [rng.choice([0, 1, 4096, bs, rng.randrange(1, 200000)]) for _ in range(500)]
    offs = [rng.randrange(0, len(data) - ln + 1) for ln in lens]
    got = ctx.hash_blocks(data, offs, lens)
    assert got == b"".join(oracle_digest(oracle, data[o:o + ln]) for o, ln in zip(offs, lens))
    tree = tmp_path / "tree"
    for k in range(12):
        d = tree / ("d%d" % (k % 3))
        d.mkdir(parents=True, exist_ok=True)
        (d / ("f%02d" % k)).write_bytes(rng.randbytes(rng.choice([0, 1, 5000, 70000, 1 << 20])))
    for block_size in (32768, 1024):
        cfg = gpu.ScannerConfig.new().block_size(block_size).threads(4).add_dir(str(tree), "/")
        want = dirsig_oracle.scan(str(tree), block_size)
        for mode in (ctx.FOOTER_HOST, ctx.FOOTER_GPU):
            ctx.set_footer_mode(mode)
            assert gpu.v1.scan(cfg, context=ctx) == want, (block_size, mode)
            os.environ["CIR_DEBUG_STRIPE_BLOCKS"] = "3"
            try:
                assert gpu.v1.scan(cfg, context=ctx) == want, (block_size, mode, 3)
            finally:
                del os.environ["CIR_DEBUG_STRIPE_BLOCKS"]


class _CountingSink(bytearray):
    """A bytearray that counts the writer calls cir_scan_v1_write made."""
    writes = 0

    def extend(self, b):
        self.writes += 1
        super().extend(b)


def test_split_scan_streams_within_stripes(gpu, monkeypatch, tmp_path):
    """A scan over two device states whose stripes take several batches
    each: every batch that extends the complete prefix reaches the emitter
    (stripes.hpp), so the index is written in many pieces while stripe 0 is
    still open -- before, a batch inside the first open stripe was never
    reported and the sink saw only the header, stripe completions and the
    tail.  128 one-block files in one directory, stripes of 64 blocks, 64 KiB
    staging slots (16 blocks; ramped 2, 4, 8, 16): stripe 0 alone takes >= 5
    batches on device state 0.  Index = the scan oracle's."""
    monkeypatch.setenv("CIR_DEBUG_SPLIT", "2")
    c = gpu.Context(device_mask=1, staging_bytes=64 << 10)
    monkeypatch.delenv("CIR_DEBUG_SPLIT")
    assert len(c.devices()) == 2
    rng = random.Random(64)
    tree = tmp_path / "tree" / "d"
    tree.mkdir(parents=True)
    for k in range(128):
        (tree / ("f%03d" % k)).write_bytes(rng.randbytes(4096))
    root = str(tmp_path / "tree")
    want = dirsig_oracle.scan(root, 4096)
    monkeypatch.setenv("CIR_DEBUG_STRIPE_BLOCKS", "64")
    cfg = gpu.ScannerConfig.new().block_size(4096).threads(2).add_dir(root, "/")
    for mode in (c.FOOTER_HOST, c.FOOTER_GPU):
        c.set_footer_mode(mode)
        sink = _CountingSink()
        n = c.scan_into(cfg, sink)
        assert bytes(sink) == want and n == len(want), mode
        # >= 5 batches of stripe 0 + the last emit / footer line
        assert sink.writes >= 6, (mode, sink.writes)
    c.close()


def test_scan_after_a_failed_scan(gpu, oracle, monkeypatch, tmp_path):
    """A scan that fails part-way (an unreadable file: CIR_EIO, the
    reference's io::Error) leaves no staging slot busy (SlotDrain), so the
    next scan on the same context is right.  Before, a slot left busy on
    device state 1 was retired by the next scan as one of its own batches
    with a wrapped-around progress count, which emitted files before their
    digests were back whenever stripe 0 finished before state 1's first
    real batch -- a race this test exercises but cannot force (the build
    without the drain passed it on one box).  Then the host paths on the
    same context.  Needs a non-root user (chmod 000 must deny the read)."""
    if os.geteuid() == 0:
        pytest.skip("root reads a chmod-000 file")
    n = gpu._n
    monkeypatch.setenv("CIR_DEBUG_SPLIT", "2")
    c = gpu.Context(device_mask=1, staging_bytes=64 << 10)
    monkeypatch.delenv("CIR_DEBUG_SPLIT")
    monkeypatch.setenv("CIR_DEBUG_STRIPE_BLOCKS", "8")
    rng = random.Random(65)
    bad_root, good_root = tmp_path / "bad", tmp_path / "good"
    for root in (bad_root, good_root):
        (root / "d").mkdir(parents=True)
        for k in range(96):
            (root / "d" / ("f%03d" % k)).write_bytes(rng.randbytes(4096))
    want = dirsig_oracle.scan(str(good_root), 4096)
    good = gpu.ScannerConfig.new().block_size(4096).threads(2).add_dir(str(good_root), "/")
    bad = gpu.ScannerConfig.new().block_size(4096).threads(2).add_dir(str(bad_root), "/")
    for k in (40, 41, 43, 45, 57, 60, 75, 90):
        f = bad_root / "d" / ("f%03d" % k)
        f.chmod(0)
        try:
            with pytest.raises(n.CiruelaError) as e:
                gpu.v1.scan(bad, context=c)
            assert e.value.status == n.CIR_EIO, e.value
        finally:
            f.chmod(0o644)
        assert gpu.v1.scan(good, context=c) == want, k
    data = rng.randbytes(3 << 20)
    assert c.hash_memory(data, 32768) == b"".join(
        oracle_digest(oracle, data[i:i + 32768]) for i in range(0, len(data), 32768))
    c.close()


def test_error_paths_are_codes_not_aborts(gpu, small_ctx, tmp_path):
    """SURVEY.md 8b errors: bad arguments give CIR_EINVAL, unreadable sources
    CIR_EIO (the reference's io::Error), never an abort; the context stays
    usable afterwards."""
    import torch
    n = gpu._n
    with pytest.raises(n.CiruelaError) as e:
        small_ctx.hash_chunks_dev(0, 4096, 0, 0, 0)  # block_size 0
    assert e.value.status == n.CIR_EINVAL
    buf = torch.empty(4096 + 64, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(n.CiruelaError) as e:  # digests not 16-byte aligned
        small_ctx.hash_chunks_dev(buf.data_ptr(), 4096, 1024, buf.data_ptr() + 8, 0)
    assert e.value.status == n.CIR_EINVAL
    with pytest.raises(n.CiruelaError) as e:
        small_ctx.hash_memory(b"abc", 32768, gpu.HashType(77, "bogus"))  # unknown hash type
    assert e.value.status == n.CIR_EINVAL
    dfd = os.open(str(tmp_path), os.O_RDONLY)  # read() on a directory: EISDIR
    try:
        with pytest.raises(n.CiruelaError) as e:
            small_ctx.hash_file(dfd, 32768)
        assert e.value.status == n.CIR_EIO
    finally:
        os.close(dfd)
    cfg = gpu.ScannerConfig.new().add_dir(str(tmp_path / "does-not-exist"), "/")
    with pytest.raises(n.CiruelaError) as e:
        gpu.v1.scan(cfg, context=small_ctx)
    assert e.value.status == n.CIR_EIO
    # still fine afterwards, on both the device and the host paths
    data = os.urandom(100000)
    want = b"".join(oracle_digest_any(data[i:i + 32768]) for i in range(0, len(data), 32768))
    assert small_ctx.hash_memory(data, 32768) == want
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda:0")
    out = torch.empty(32 * 4, dtype=torch.uint8, device="cuda:0")
    small_ctx.hash_chunks_dev(t.data_ptr(), len(data), 32768, out.data_ptr(), 0)
    torch.cuda.synchronize()
    assert out.cpu().numpy().tobytes() == want


@pytest.mark.skipif(os.geteuid() == 0, reason="root reads files whatever their mode")
def test_scan_reports_the_first_failure_in_walk_order(gpu, small_ctx, tmp_path):
    """The walk reads directories in parallel but reports a failure as the
    serial, depth-first walk meets it first: of 40 unreadable directories
    the first by name (d00, under a tree whose other branches are read
    first or at the same time), every time."""
    n = gpu._n
    for k in range(40):
        d = tmp_path / "t" / ("d%02d" % k)
        (d / "sub").mkdir(parents=True)
        (d / "sub" / "f").write_bytes(b"x" * k)
    for k in range(8):
        (tmp_path / "t" / ("a%d" % k)).mkdir()
        for i in range(50):
            (tmp_path / "t" / ("a%d" % k) / ("f%02d" % i)).write_bytes(b"y")
    locked = [tmp_path / "t" / ("d%02d" % k) / "sub" for k in range(40)]
    for d in locked:
        os.chmod(d, 0)
    try:
        cfg = gpu.ScannerConfig.new().threads(8).add_dir(str(tmp_path / "t"), "/")
        for _ in range(5):
            with pytest.raises(n.CiruelaError) as e:
                gpu.v1.scan(cfg, context=small_ctx)
            assert e.value.status == n.CIR_EIO
            assert str(locked[0]) in str(e.value), e.value
    finally:
        for d in locked:
            os.chmod(d, 0o755)


@pytest.mark.skipif(os.geteuid() == 0, reason="root reads files whatever their mode")
@pytest.mark.parametrize("what", ["file", "dir"])
def test_scan_unreadable_entry_is_an_io_error(gpu, small_ctx, tmp_path, what):
    """v1::scan returns io::Error for a file or directory it cannot read
    (src/client/sync/uploads.rs:57 wraps it as "error indexing dir"): the
    GPU scan gives CIR_EIO, after its reader threads and staging pipeline
    have started, and the context indexes the same tree once it is readable."""
    n = gpu._n
    (tmp_path / "a").mkdir()
    (tmp_path / "a" / "ok.bin").write_bytes(os.urandom(100000))
    (tmp_path / "b").mkdir()
    victim = tmp_path / "b" / "secret.bin"
    victim.write_bytes(os.urandom(70000))
    target = victim if what == "file" else tmp_path / "b"
    os.chmod(target, 0)
    try:
        cfg = gpu.ScannerConfig.new().add_dir(str(tmp_path), "/")
        with pytest.raises(n.CiruelaError) as e:
            gpu.v1.scan(cfg, context=small_ctx)
        assert e.value.status == n.CIR_EIO
    finally:
        os.chmod(target, 0o755 if what == "dir" else 0o644)
    assert gpu.v1.scan(cfg, context=small_ctx) == dirsig_oracle.scan(str(tmp_path), 32768)


def oracle_digest_any(b):
    import hashlib
    return hashlib.blake2b(b, digest_size=32).digest()


@pytest.mark.parametrize("seed", range(6))
def test_randomized_batches_and_files(gpu, ctx, oracle, seed):
    """Seeded random shapes across every routing decision: descriptor batches
    below and above the small-batch limit (49152), chain lengths around the
    quad thresholds (8 and 1024 lines), misaligned offsets; device-resident
    files with random block sizes (multiples of 128 or not) and block counts
    on both sides of the limit."""
    random_case(gpu, ctx, oracle, 1000 + seed)


def test_randomized_sweep(gpu, ctx, oracle):
    """The same random cases over CIR_SWEEP_SEEDS more seeds (0 = skipped;
    a long parity sweep run by hand, profiles/r02/parity_sweep/)."""
    n = int(os.environ.get("CIR_SWEEP_SEEDS", "0"))
    if n == 0:
        pytest.skip("set CIR_SWEEP_SEEDS to run the sweep")
    first = int(os.environ.get("CIR_SWEEP_FIRST", "5000"))
    for s in range(first, first + n):
        random_case(gpu, ctx, oracle, s)
        print("seed %d ok" % s, flush=True)


def random_case(gpu, ctx, oracle, seed):
    import torch
    rng = random.Random(seed)
    # descriptor batch
    n = rng.choice([1, 7, 300, 5000, 49152, 49153, 60000])
    lens = []
    for _ in range(n):
        kind = rng.random()
        if kind < 0.5:
            lens.append(rng.randrange(0, 4097))
        elif kind < 0.8:
            lens.append(rng.choice([1023, 1024, 1025, 8 * 128, 8 * 128 - 1, 32768]))
        elif kind < 0.98:
            lens.append(rng.randrange(4097, 200000))
        else:
            lens.append(rng.choice([1024 * 128 - 1, 1024 * 128, 1024 * 128 + 1, 1 << 20]))
    offs, pos = [], 0
    for ln in lens:
        pos += rng.randrange(0, 17)
        offs.append(pos)
        pos += ln
    data = dev_random(gpu, pos, seed=7 + seed)
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * n, dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, out.data_ptr(), 0)
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    ao = np.array(offs, dtype=np.uint64)
    al = np.array(lens, dtype=np.uint32)
    want = np.zeros(32 * n, dtype=np.uint8)
    oracle.oracle_hash_blocks(host.ctypes.data, ao.ctypes.data, al.ctypes.data, n,
                              want.ctypes.data, 8)
    assert first_bad(out.cpu().numpy(), want) is None
    # the same batch through the bounds-checked entry point (the arena is
    # exactly [0, pos)), with a few descriptors moved out of range (drawn
    # apart from rng, so the other draws of a seed stay as they were)
    brng = random.Random(seed ^ 0xB0B0)
    bad = sorted(brng.sample(range(n), brng.randrange(0, min(n, 12) + 1)))
    b_off, b_len = list(offs), list(lens)
    for b in bad:
        b_off[b], b_len[b] = brng.choice([
            (pos - b_len[b] + 1, b_len[b]) if b_len[b] else (pos + 1, 0),  # just past the end
            ((1 << 64) - brng.randrange(1, 1 << 20), brng.randrange(1 << 20, 1 << 21)),  # wraps
            (brng.randrange(pos + 1, 1 << 50), brng.randrange(0, 70000))])  # far outside
    d_off = torch.tensor(np.array(b_off, dtype=np.uint64).view(np.int64), device="cuda:0")
    d_len = torch.tensor(np.array(b_len, dtype=np.uint32).view(np.int32), device="cuda:0")
    out.fill_(0x5A)
    nrange = torch.full((1,), -1, dtype=torch.int32, device="cuda:0")
    gpu._n.check(gpu._n.lib.cir_hash_blocks_dev_bounded(
        ctx.handle if brng.random() < 0.7 else None, 1, data.data_ptr(), pos, d_off.data_ptr(),
        d_len.data_ptr(), n, out.data_ptr(), nrange.data_ptr(), None))
    torch.cuda.synchronize()
    want = want.reshape(-1, 32)
    want[bad] = 0
    assert first_bad(out.cpu().numpy(), want.reshape(-1)) is None
    assert int(nrange.item()) == len(bad)
    del data, d_off, d_len, out
    # device-resident file
    bs = rng.choice([128 * rng.randrange(1, 64), rng.randrange(100, 9000)])
    nblk = rng.choice([rng.randrange(1, 2000), rng.randrange(49000, 49300)])
    nbytes = max(1, nblk * bs - rng.randrange(0, bs))
    skew = rng.choice([0, 0, 16, 3])
    fdata = dev_random(gpu, nbytes + skew, seed=99 + seed)
    nb = (nbytes + bs - 1) // bs
    fout = torch.zeros(nb * 32, dtype=torch.uint8, device="cuda:0")
    ctx.hash_chunks_dev(fdata.data_ptr() + skew, nbytes, bs, fout.data_ptr(), 0)
    torch.cuda.synchronize()
    fh = fdata.cpu().numpy()[skew:].copy()
    assert first_bad(fout.cpu().numpy(), oracle_chunks(oracle, fh, nbytes, bs)) is None
    del fdata, fout
    # SHA-512/256 descriptors (k_sha_desc), a smaller batch
    n = rng.choice([1, 3, 200, 3000])
    lens = [rng.choice([0, 1, 111, 112, 127, 128, 129, 239, 240, 4096, 32768,
                        rng.randrange(0, 300000)]) for _ in range(n)]
    offs, pos = [], 0
    for ln in lens:
        pos += rng.randrange(0, 9)
        offs.append(pos)
        pos += ln
    data = dev_random(gpu, max(pos, 1), seed=31 + seed)
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * n, dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, out.data_ptr(), 0,
                        hash_type=gpu.HashType.sha512_256())
    torch.cuda.synchronize()
    host = data.cpu().numpy().tobytes()
    want = b"".join(oracle_sha(oracle, host[o:o + ln]) for o, ln in zip(offs, lens))
    assert first_bad(out.cpu().numpy(), np.frombuffer(want, dtype=np.uint8)) is None


def test_reference_hidden_line_on_gpu(gpu, small_ctx, tmp_path, dirsig_example):
    """The one block digest the reference holds (src/cluster/download.rs:363,
    `.hidden f 7 6d7f5f98...` = SHA-512/256(b"Hidden\\n")), reproduced by
    the GPU scan: subdir/.hidden scanned with HashType::sha512_256() emits
    that line byte for byte."""
    want = [ln for ln in dirsig_example["index"].encode().split(b"\n")
            if ln.startswith(b"  .hidden ")]
    assert len(want) == 1
    (tmp_path / "subdir").mkdir()
    (tmp_path / "subdir" / ".hidden").write_bytes(b"Hidden\n")
    cfg = gpu.ScannerConfig.new().hash(gpu.HashType.sha512_256()).add_dir(str(tmp_path), "/")
    index = gpu.v1.scan(cfg, context=small_ctx)
    got = [ln for ln in index.split(b"\n") if ln.startswith(b"  .hidden ")]
    assert got == want
    assert index.startswith(b"DIRSIGNATURE.v1 sha512/256 block_size=32768\n/\n/subdir\n")
    # and through the per-block entry points
    assert gpu.sha512_256(b"Hidden\n").hex() == want[0].split()[-1].decode()


def test_memory_blocks_sha512(gpu, oracle):
    """register_memory_blocks(HashType::sha512_256(), ..) keys blocks by their
    SHA-512/256 digests (put-file against a sha512/256 index,
    src/client/put_file/network.rs:56, src/blocks.rs:187-204)."""
    data = os.urandom(int(2.5 * 4096))
    r = gpu.ThreadedBlockReader()
    r.register_memory_blocks(gpu.HashType.sha512_256(), 4096, data)
    assert len(r) == 3
    for i in range(3):
        blk = data[i * 4096:(i + 1) * 4096]
        assert r.read_block(oracle_sha(oracle, blk)) == blk
    with pytest.raises(gpu.ReadError):
        r.read_block(oracle_digest(oracle, data[:4096]))  # not a blake2b registry


def test_current_device_is_preserved(gpu, ctx, small_ctx, tmp_path):
    """No entry point changes the caller's current HIP device (the header's
    contract; a NULL stream means the current device's null stream)."""
    import torch
    dev = torch.cuda.current_device()
    data = os.urandom(100000)
    gpu.BlockHash.hash_bytes(data)
    assert torch.cuda.current_device() == dev
    ctx.hash_memory(data, 4096)
    ctx.hash_blocks(data, [0, 10], [10, 5000])
    assert torch.cuda.current_device() == dev
    make_tree(tmp_path)
    gpu.v1.scan(gpu.ScannerConfig.new().add_dir(str(tmp_path), "/"), context=small_ctx)
    assert torch.cuda.current_device() == dev
    c2 = gpu.Context(device_mask=1)
    c2.close()
    assert torch.cuda.current_device() == dev
    # the ordering scratch lives on the stream's device
    t = torch.tensor(bytearray(data), dtype=torch.uint8, device="cuda:0")
    off = torch.tensor([0, 4096], dtype=torch.int64, device="cuda:0")
    ln = torch.tensor([4096, 90000], dtype=torch.int32, device="cuda:0")
    out = torch.zeros(64, dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev(t.data_ptr(), off.data_ptr(), ln.data_ptr(), 2, out.data_ptr(), 0)
    torch.cuda.synchronize()
    assert torch.cuda.current_device() == dev
    assert out.cpu().numpy().tobytes() == gpu.BlockHash.hash_bytes(data[:4096]).__bytes__() + \
        gpu.BlockHash.hash_bytes(data[4096:94096]).__bytes__()


def test_rewrite_rejects_invalid_paths(gpu, small_ctx):
    """RawIndex::into_mut's InvalidPath (src/cluster/download.rs:143-161) with
    a real context: `..` / `.` components and names are parse errors."""
    for bad in (b"/\n/a/../b\n  f f 0\n", b"/\n  .. f 0\n", b"/\n  . s x\n"):
        idx = b"DIRSIGNATURE.v1 blake2b/256 block_size=32768\n" + bad + b"ab" * 32 + b"\n"
        with pytest.raises(gpu.CiruelaError) as e:
            small_ctx.index_rewrite(idx)
        assert e.value.status == gpu._n.CIR_EPARSE


@pytest.mark.parametrize("bs,nbytes", [(4096, 70000 * 4096 + 1234), (32768, 65535 * 32768)])
def test_chunks_dev_without_context(gpu, oracle, bs, nbytes):
    """cir_hash_chunks_dev with a NULL context: the fused single launch
    (k_chunks with the ragged rest in lane mode) gives the same digests."""
    import torch
    data = dev_random(gpu, nbytes, seed=bs + nbytes)
    nb = (nbytes + bs - 1) // bs
    out = torch.zeros(nb * 32, dtype=torch.uint8, device="cuda:0")
    gpu._n.check(gpu._n.lib.cir_hash_chunks_dev(None, data.data_ptr(), nbytes, bs,
                                                out.data_ptr(), None))
    torch.cuda.synchronize()
    want = oracle_chunks(oracle, data.cpu().numpy(), nbytes, bs)
    assert first_bad(out.cpu().numpy(), want) is None


def lane_wave_slots():
    import torch
    return 64 * 4 * torch.cuda.get_device_properties(0).multi_processor_count


# (block size, whole waves per SIMD k -- lane waves of 64 chains, or quad
# waves of 16 ("q") below the small-batch limit -- extra whole blocks, tail)
RELAY_SHAPES = [
    (32768, 1, 1, 0),          # one extra chain: 16 segments of 16 lines
    (32768, 1, 1000, 777),     # 63 groups + the short last block beside
    (4096, 2, 4000, 1),        # k = 2, 32-line chains: 4 segments each
    (2048, 1, 2000, 0),        # 125 groups of 16-line chains: 2 segments each
    (131072, 1, 3, 0),         # 1024-line chains: 64 segments
    (4096, 4, 100, 5),         # k >= 3: the lane part with padded LDS (2 waves per SIMD)
    (32768, "2q", 1, 0),       # quad regime: 2 quad waves per SIMD + 1 chain
    (16384, "2q", 3000, 99),   # 2 quad waves per SIMD + 3000 chains + a tail
    (65536, "1q", 2, 0),       # 1 quad wave per SIMD + 2 chains
    (32768, "3q", 4, 0),       # past the small-batch limit: quad base of 3 waves
    (4096, "2q", 77, 3),       # 32-line chains beside 2 quad waves per SIMD
    (16384, "1q", "q/2", 5),   # half a quad wave per SIMD of 128-line chains
    (4096, 1, "l/2", 0),       # half a lane wave per SIMD of 32-line chains
    (2048, 17, 5, 0),          # past 16 lane waves per SIMD
]


def relay_extra(extra):
    return {"q/2": lane_wave_slots() // 8, "l/2": lane_wave_slots() // 2}.get(extra, extra)


def relay_nfull(k, extra):
    slots = lane_wave_slots()
    extra = relay_extra(extra)
    if isinstance(k, str):
        return int(k[:-1]) * slots // 4 + extra
    return k * slots + extra


@pytest.mark.parametrize("bs,k,extra,tail", RELAY_SHAPES)
@pytest.mark.parametrize("polls", [None, "0"])
def test_chunks_dev_relay(gpu, ctx, oracle, bs, k, extra, tail, polls, monkeypatch):
    """A file of k whole lane waves per SIMD plus `extra` blocks: the extra
    blocks run as relayed quad chains (k_quad_relay) beside the lane part.
    polls "0": every waiting segment gives up at once, so the finisher
    (k_quad_relay_finish) completes the chains from the handed-on state."""
    import torch
    if polls is not None:
        monkeypatch.setenv("CIR_RELAY_POLLS", polls)
    nfull = relay_nfull(k, extra)
    extra = relay_extra(extra)
    assert gpu._n.lib.cir_debug_relay_blocks(nfull, bs) == extra
    nbytes = nfull * bs + tail
    data = dev_random(gpu, nbytes, seed=nfull ^ bs)
    nb = (nbytes + bs - 1) // bs
    out = torch.zeros(nb * 32, dtype=torch.uint8, device="cuda:0")
    for _ in range(2):  # the second call reuses the flags and the state buffer
        ctx.hash_chunks_dev(data.data_ptr(), nbytes, bs, out.data_ptr(), 0)
    torch.cuda.synchronize()
    want = oracle_chunks(oracle, data.cpu().numpy(), nbytes, bs)
    del data
    assert first_bad(out.cpu().numpy(), want) is None, "block %s" % first_bad(out.cpu().numpy(), want)


def test_relay_rule_bounds(gpu):
    """No relay below one quad wave per SIMD, beyond k = 32 lane waves, past
    min(5/8, lines / 32) of a lane wave or 1/2 of a quad wave
    (1/64 past the small-batch limit) of extra blocks, below 16 lines, or in
    the quad regime below 64 lines at k = 1 / 32 above (128 past 1/4 of a
    quad wave)."""
    slots = lane_wave_slots()
    qslots = slots // 4
    f = gpu._n.lib.cir_debug_relay_blocks
    assert f(slots - 1, 32768) == 0
    assert f(slots, 32768) == 0
    assert f(slots + 1, 32768) == 1
    assert f(3 * slots + 1, 32768) == 1
    assert f(16 * slots + 5, 32768) == 5
    assert f(17 * slots + 1, 32768) == 1
    assert f(32 * slots + 7, 32768) == 7
    assert f(33 * slots + 1, 32768) == 0
    assert f(slots + slots * 5 // 8, 32768) == slots * 5 // 8
    assert f(slots + slots * 5 // 8 + 1, 32768) == 0
    assert f(slots + slots * 5 // 8, 4096) == slots * 5 // 8
    assert f(slots + slots * 5 // 8 + 1, 4096) == 0
    assert f(slots + slots // 2, 2048) == slots // 2
    assert f(slots + slots // 2 + 1, 2048) == 0
    assert f(slots + slots * 5 // 8, 8192) == slots * 5 // 8
    assert f(slots + slots // 4, 8192) == slots // 4
    assert f(slots + 1, 1024) == 0
    assert f(slots + 1, 2048) == 1
    assert f(qslots - 1, 32768) == 0
    assert f(qslots + 1, 32768) == 1
    assert f(qslots + 1, 8192) == 1
    assert f(qslots + 1, 4096) == 0
    assert f(2 * qslots + 1, 4096) == 1
    assert f(2 * qslots + 1, 2048) == 0
    assert f(2 * qslots + 1, 32768) == 1
    assert f(2 * qslots + qslots // 4, 32768) == qslots // 4
    assert f(2 * qslots + qslots // 4 + 1, 8192) == 0
    assert f(2 * qslots + qslots // 4 + 1, 16384) == qslots // 4 + 1
    assert f(qslots + qslots // 2, 16384) == qslots // 2
    assert f(2 * qslots + qslots // 2 + 1, 32768) == 0
    assert f(3 * qslots + qslots // 64, 32768) == qslots // 64
    assert f(3 * qslots + qslots // 64 + 1, 32768) == 0


def desc_batch_check(gpu, ctx, oracle, lens, offs_skew, seed):
    """Hash lens as a device descriptor batch (offsets 16-B aligned, plus
    offs_skew(i) bytes) and compare every digest with the oracle."""
    import torch
    offs, pos = [], 0
    for i, ln in enumerate(lens):
        pos += (-pos) % 16 + offs_skew(i)
        offs.append(pos)
        pos += ln
    data = dev_random(gpu, pos, seed=seed)
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens, dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * len(lens), dtype=torch.uint8, device="cuda:0")
    for _ in range(2):  # the second call reuses the relay's flags and state
        ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                            out.data_ptr(), 0)
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    del data
    ao = np.array(offs, dtype=np.uint64)
    al = np.array(lens, dtype=np.uint32)
    want = np.zeros(32 * len(lens), dtype=np.uint8)
    oracle.oracle_hash_blocks(host.ctypes.data, ao.ctypes.data, al.ctypes.data, len(lens),
                              want.ctypes.data, 8)
    got = out.cpu().numpy()
    assert first_bad(got, want) is None, "descriptor %s" % first_bad(got, want)


@pytest.mark.parametrize("case", ["uniform1", "uniform1000", "ragged", "k2", "k4", "wide", "longq",
                                  "q1", "q2", "q2ragged", "q2short", "qhalf", "qmixed",
                                  "shorthalf"])
@pytest.mark.parametrize("polls", [None, "0"])
def test_desc_relay(gpu, ctx, oracle, case, polls, monkeypatch):
    """Descriptor batches of k lane waves per SIMD plus a few chains: the
    last chains of the order are relayed (k_desc_relay, decided on the
    device) beside the lane part.  ragged: the relayed chains have mixed
    lengths (the shortest of the batch: ragged, empty, misaligned starts);
    longq: a few long chains make a quad part, so no relay runs.  q*: small
    batches (quad regime: k whole quad waves per SIMD plus a few chains,
    relayed beside the quad part); qmixed has chains below 8 lines, so no
    relay runs.  polls "0": the finisher completes every chain."""
    if polls is not None:
        monkeypatch.setenv("CIR_RELAY_POLLS", polls)
    slots = lane_wave_slots()
    qslots = slots // 4
    rng = random.Random(zlib.crc32(case.encode()))  # stable across processes
    skew = lambda i: 0  # noqa: E731
    if case == "uniform1":
        lens = [32768] * (slots + 1)
    elif case == "uniform1000":
        lens = [32768] * (slots + 1000)
    elif case == "ragged":
        lens = [32768] * (slots + 700) + [rng.randrange(0, 32768) for _ in range(77)] + [0, 0, 1]
        rng.shuffle(lens)
        skew = lambda i: 5 if i % 13 == 0 else 0  # noqa: E731
    elif case == "k2":
        lens = [4096] * (2 * slots + 4000)
    elif case == "k4":  # the lane part padded to two waves per SIMD beside the relay
        lens = [8192] * (4 * slots + 1500)
    elif case == "wide":  # 9/16 of a lane wave per SIMD relayed, behind the gate
        lens = [32768] * (slots + slots * 9 // 16)
    elif case == "longq":
        lens = [32768] * (slots + 300) + [1 << 18] * 20
        rng.shuffle(lens)
    elif case == "q1":
        lens = [65536] * (qslots + 2)
    elif case == "q2":
        lens = [32768] * (2 * qslots + 1)
    elif case == "q2ragged":
        lens = [32768] * (2 * qslots + 250) + [rng.randrange(1024, 32768) for _ in range(50)]
        rng.shuffle(lens)
        skew = lambda i: 3 if i % 17 == 0 else 0  # noqa: E731
    elif case == "q2short":
        lens = [4096] * (2 * qslots + 999)
    elif case == "shorthalf":  # half a lane wave per SIMD of 32-line chains
        lens = [4096] * (slots + slots // 2)
    elif case == "qhalf":  # half a quad wave per SIMD relayed, ragged at the end
        lens = [16384] * (qslots + qslots // 2 - 40) + [rng.randrange(1, 16384) for _ in range(40)]
        rng.shuffle(lens)
    else:
        lens = [32768] * (2 * qslots + 100) + [rng.randrange(0, 1000) for _ in range(10)]
        rng.shuffle(lens)
    desc_batch_check(gpu, ctx, oracle, lens, skew, seed=len(lens))


def test_relays_from_concurrent_callers(gpu, ctx, oracle):
    """A chunk-form relay and both descriptor relays (lane and quad regime)
    issued from three threads on three streams of one context at once: the
    relays share the device's scratch and are ordered by its quad-part
    stream; every digest against the oracle."""
    import threading
    import torch
    slots = lane_wave_slots()
    jobs = []
    # chunk form: one lane wave per SIMD + 3 blocks of 32 KiB
    nb1 = slots + 3
    d1 = dev_random(gpu, nb1 * 32768, seed=71)
    o1 = torch.zeros(nb1 * 32, dtype=torch.uint8, device="cuda:0")
    jobs.append(("chunks", d1, o1, nb1 * 32768))
    # descriptor batches: lane regime (slots + 5 x 16 KiB), quad regime
    # (slots / 4 + 7 x 64 KiB)
    for name, n, bs, seed in (("desc_lane", slots + 5, 16384, 72), ("desc_quad", slots // 4 + 7, 65536, 73)):
        d = dev_random(gpu, n * bs, seed=seed)
        off = torch.arange(n, dtype=torch.int64, device="cuda:0") * bs
        ln = torch.full((n,), bs, dtype=torch.int32, device="cuda:0")
        o = torch.zeros(n * 32, dtype=torch.uint8, device="cuda:0")
        jobs.append((name, d, o, (off, ln, n, bs)))
    streams = [torch.cuda.Stream() for _ in jobs]
    torch.cuda.synchronize()
    errors = []

    def run(job, st):
        try:
            name, d, o, arg = job
            for _ in range(3):
                if name == "chunks":
                    ctx.hash_chunks_dev(d.data_ptr(), arg, 32768, o.data_ptr(), st.cuda_stream)
                else:
                    off, ln, n, _ = arg
                    ctx.hash_blocks_dev(d.data_ptr(), off.data_ptr(), ln.data_ptr(), n,
                                        o.data_ptr(), st.cuda_stream)
            st.synchronize()
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    th = [threading.Thread(target=run, args=(j, st)) for j, st in zip(jobs, streams)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for name, d, o, arg in jobs:
        host = d.cpu().numpy()
        if name == "chunks":
            want = oracle_chunks(oracle, host, arg, 32768)
        else:
            _, _, n, bs = arg
            want = oracle_chunks(oracle, host, n * bs, bs)
        got = o.cpu().numpy()
        assert first_bad(got, want) is None, (name, first_bad(got, want))


@pytest.mark.parametrize("regime", ["lane", "lane_1m", "quad", "quad_1m"])
def test_desc_relay_unordered_lengths_in_one_bin(gpu, ctx, oracle, regime):
    """Relayed chains of different lengths that share one length bin of the
    ordering (order.hip: bins are exact only below 2048 lines, then 16 lines
    wide at 256 KiB and 64 at 1 MiB), so a group's first chain is not always
    its longest.  Most chains end on a segment boundary and ~10 % run a few
    lines past it: before the fix, a group whose first chain ended on the
    boundary raised the final flag while a longer chain was still unfinished,
    and that chain's digest was never written (kernels.hip
    relay_segment).  Descriptors overlap in one small arena (each (offset,
    length) pair is hashed once by the oracle); every digest is checked."""
    import torch
    slots = lane_wave_slots()
    qslots = slots // 4
    if regime.startswith("lane"):   # no quad part: > 16384 long chains, lane mode + relay
        n, extra = slots + slots // 8, slots // 8
    else:                           # small batch: every chain in the quad part + relay
        n, extra = 2 * qslots + 2000, 2000
    base_lines, over = (2048, 15) if not regime.endswith("1m") else (8192, 63)
    rng = np.random.default_rng(zlib.crc32(regime.encode()))
    long_ = rng.random(n) < 0.1
    lines = np.where(long_, base_lines + rng.integers(1, over + 1, size=n), base_lines)
    # ragged ends on some of the long chains (still in the same bin)
    tail = np.where(long_ & (rng.random(n) < 0.5), rng.integers(1, 128, size=n), 0)
    lens = (lines * 128 - np.where(tail > 0, 128 - tail, 0)).astype(np.int64)
    offs = 16 * rng.integers(0, 64, size=n)
    arena_bytes = int(offs.max() + lens.max()) + 64
    data = dev_random(gpu, arena_bytes, seed=n ^ 0xB1)
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda:0")
    d_len = torch.tensor(lens.astype(np.int32), dtype=torch.int32, device="cuda:0")
    out = torch.zeros(32 * n, dtype=torch.uint8, device="cuda:0")
    host = data.cpu().numpy()
    pairs = sorted(set(zip(offs.tolist(), lens.tolist())))
    po = np.array([p[0] for p in pairs], dtype=np.uint64)
    pl = np.array([p[1] for p in pairs], dtype=np.uint32)
    pd = np.zeros(32 * len(pairs), dtype=np.uint8)
    oracle.oracle_hash_blocks(host.ctypes.data, po.ctypes.data, pl.ctypes.data, len(pairs),
                              pd.ctypes.data, 8)
    index = {p: i for i, p in enumerate(pairs)}
    sel = np.array([index[(o, ln)] for o, ln in zip(offs.tolist(), lens.tolist())])
    want = pd.reshape(-1, 32)[sel].reshape(-1)
    for _ in range(3):  # the order within a bin varies between calls
        out.zero_()
        ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                            out.data_ptr(), 0)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert first_bad(got, want) is None, "descriptor %s" % first_bad(got, want)


def test_context_lifecycle_releases_device_memory(gpu, oracle):
    """cir_init allocates a device state's working set up front (three
    staging slots, ordering and relay scratch, the footer chain's state; the
    chain's text buffers and timing events on first use) and cir_destroy
    must give all of it back.  The first two cycles of a process
    leave ~0.2 GiB with the HIP runtime for good (its own lazily created
    state; tools/lifecycle_probe.py: 184 + 24 MiB, then 0 per cycle), so
    after two warm-up cycles ten more create / use / destroy cycles of a
    64 MiB-staging context must leave the device's free memory unchanged."""
    import torch
    data = np.frombuffer(os.urandom(1 << 20), dtype=np.uint8)
    want = np.empty(32 * 32, dtype=np.uint8)
    oracle.oracle_hash_chunks(data.ctypes.data, data.size, 32768, want.ctypes.data, 4)

    def cycle():
        c = gpu.Context(device_mask=1, staging_bytes=64 << 20)
        size, hashes = gpu.Hashes.hash_file(gpu.HashType.blake2b_256(), 32768,
                                            data.tobytes(), context=c)
        assert size == data.size and hashes.raw() == want.tobytes()
        c.close()
        torch.cuda.synchronize()
        return torch.cuda.mem_get_info()[0]
    def rss():
        with open("/proc/self/status") as f:
            return next(int(ln.split()[1]) << 10 for ln in f if ln.startswith("VmRSS:"))
    cycle()
    free0 = cycle()
    rss0 = rss()
    for _ in range(10):
        free1 = cycle()
    assert free0 - free1 < (16 << 20), (free0 - free1) >> 20
    # the pinned staging (3 x 64 MiB per context) goes back to the host too
    assert rss() - rss0 < (64 << 20), (rss() - rss0) >> 20


def test_blocks_larger_than_the_staging_slot(gpu, oracle, tmp_path):
    """A block size (and single blocks) larger than the context's staging
    slot: the slots grow to one block (scan, hash_file, hash_memory,
    hash_blocks, the asynchronous verify); every digest and the index equal
    the oracles'.  bs = 3 MiB + 5 on 1 MiB slots.  Until round 5 the scan
    sent a batch's 16-byte-aligned end instead of its packed bytes, past the
    end of a slot sized bs + 16 (not a multiple of 16): the upload failed
    with an invalid argument."""
    c = gpu.Context(device_mask=1, staging_bytes=1 << 20)
    rng = random.Random(91)
    bs = (3 << 20) + 5
    root = tmp_path / "tree"
    (root / "d").mkdir(parents=True)
    sizes = [0, 1, bs, bs + 1, 2 * bs + 100, (10 << 20) + 7]
    for k, n in enumerate(sizes):
        (root / "d" / ("f%d" % k)).write_bytes(rng.randbytes(n))
    cfg = gpu.ScannerConfig.new().block_size(bs).threads(3).add_dir(str(root), "/")
    assert gpu.v1.scan(cfg, context=c) == dirsig_oracle.scan(str(root), bs)
    data = (root / "d" / "f5").read_bytes()
    want = b"".join(oracle_digest(oracle, data[i:i + bs]) for i in range(0, len(data), bs))
    assert c.hash_memory(data, bs) == want
    with open(root / "d" / "f5", "rb") as f:
        size, hashes = c.hash_file(f.fileno(), bs)
    assert size == len(data) and hashes == want
    lens = [5 << 20, 1, 0, (2 << 20) + 3]
    offs = [0, 17, 40, 123]
    got = c.hash_blocks(data, offs, lens)
    assert got == b"".join(oracle_digest(oracle, data[o:o + n]) for o, n in zip(offs, lens))
    t = c.verify_submit(data[:5 << 20], oracle_digest(oracle, data[:5 << 20]))
    assert c.verify_wait(t) is True
    c.close()
    # a staging size that is not a multiple of 16 (the scan's segments are
    # 16-byte aligned inside a slot): random trees at two block sizes
    c = gpu.Context(device_mask=1, staging_bytes=1000003)
    for k, bs2 in enumerate((4096, 65536 + 3)):
        root2 = tmp_path / ("odd%d" % k)
        root2.mkdir()
        random_tree(root2, rng, bs2)
        cfg = gpu.ScannerConfig.new().block_size(bs2).threads(2).add_dir(str(root2), "/")
        assert gpu.v1.scan(cfg, context=c) == dirsig_oracle.scan(str(root2), bs2), bs2
    c.close()


def test_extreme_block_sizes(gpu, oracle, tmp_path):
    """Block sizes at both ends of 1 .. 2^32-1: 1 and 7 bytes (a digest per
    byte or seven), and 2^32-1 over small inputs -- one short block per file,
    in slots sized to the input, not the block size (the process's resident
    memory grows by far less than one such block).  Scan, hash_memory,
    hash_file (a regular file shorter than a block: a slot of its size plus
    one byte); every digest and the index equal the oracles'."""
    c = gpu.Context(device_mask=1, staging_bytes=1 << 20)
    rng = random.Random(93)

    def rss():
        with open("/proc/self/status") as f:
            return next(int(ln.split()[1]) << 10 for ln in f if ln.startswith("VmRSS:"))
    for bs in (1, 7, (1 << 32) - 1):
        root = tmp_path / ("bs%d" % bs)
        (root / "d").mkdir(parents=True)
        for k, n in enumerate((0, 1, 7, 8, 1000, 5000)):
            (root / "d" / ("f%d" % k)).write_bytes(rng.randbytes(n))
        rss0 = rss()
        cfg = gpu.ScannerConfig.new().block_size(bs).threads(2).add_dir(str(root), "/")
        assert gpu.v1.scan(cfg, context=c) == dirsig_oracle.scan(str(root), bs), bs
        data = rng.randbytes(3000)
        want = b"".join(oracle_digest(oracle, data[i:i + bs]) for i in range(0, len(data), bs))
        assert c.hash_memory(data, bs) == want, bs
        p = root / "d" / "f5"
        with open(p, "rb") as f:
            size, hashes = c.hash_file(f.fileno(), bs)
        blob = p.read_bytes()
        assert size == 5000 and hashes == b"".join(
            oracle_digest(oracle, blob[i:i + bs]) for i in range(0, len(blob), bs)), bs
        assert rss() - rss0 < (512 << 20), (bs, (rss() - rss0) >> 20)
    c.close()


@pytest.mark.parametrize("size,hint_short", [(1000, 600), (1000, 999), (3 << 20, (3 << 20) - 100),
                                             (5000, 4984), (17, 1)])
def test_hash_file_that_grows(gpu, oracle, tmp_path, monkeypatch, size, hint_short):
    """cir_hash_file on a regular file that grows between its fstat and its
    reads (CIR_DEBUG_GROW: the file taken to be hint_short bytes shorter):
    a size below one block gets a slot of that size plus one byte, finds it
    full, and regrows it to the block form around the bytes already read --
    the digests are the whole file's, as Hashes::hash_file's read-to-EOF
    loop gives."""
    bs = (1 << 20) + 5
    c = gpu.Context(device_mask=1, staging_bytes=1 << 20)
    blob = os.urandom(size)
    p = tmp_path / "grows.bin"
    p.write_bytes(blob)
    monkeypatch.setenv("CIR_DEBUG_GROW", str(hint_short))
    for skip in (0, 3):
        with open(p, "rb") as f:
            f.seek(skip)
            got, hashes = c.hash_file(f.fileno(), bs)
        tail = blob[skip:]
        assert got == len(tail)
        assert hashes == b"".join(oracle_digest(oracle, tail[i:i + bs])
                                  for i in range(0, len(tail), bs)), (size, hint_short, skip)
    c.close()


def random_tree(root, rng, bs):
    """A random tree for the scan sweep: nested directories, files whose
    sizes sit on and around block and 128-B line edges (empty files
    included), odd names that need escaping, executables and symlinks."""
    names = ["a", "b c", "d\\e", "x.bin", "Ünï", "tab\tname", "z" * 40, ".hidden", "9"]
    dirs = [root]
    for _ in range(rng.randrange(0, 5)):
        parent = rng.choice(dirs)
        d = parent / ("d%d_%s" % (len(dirs), rng.choice(names)))
        d.mkdir(exist_ok=True)
        dirs.append(d)
    if rng.random() < 0.3:
        (root / "empty_dir").mkdir(exist_ok=True)
    for k in range(rng.randrange(1, 24)):
        d = rng.choice(dirs)
        nb = rng.choice([0, 0, 1, 1, 2, 3, 7])
        size = max(0, nb * bs + rng.choice([0, 0, -1, 1, 127, 128, -128, rng.randrange(-bs + 1, bs)]))
        p = d / ("f%02d_%s" % (k, rng.choice(names)))
        p.write_bytes(rng.randbytes(size))
        if rng.random() < 0.2:
            os.chmod(p, 0o755)
    for k in range(rng.randrange(0, 3)):
        d = rng.choice(dirs)
        os.symlink(rng.choice(["../a", "target %d" % k, "x" * 70]), d / ("l%d" % k))


def deep_chain(root, rng, bs):
    """A chain of directories whose path passes PATH_MAX below root (made
    through dir fds), with files of a few blocks at some levels: the scan
    opens such directories relative to their parent's fd and such files
    piecewise (scan.cpp read_dir, open_long)."""
    depth = rng.randrange(14, 24)
    fd = os.open(str(root), os.O_RDONLY | os.O_DIRECTORY)
    try:
        for i in range(depth):
            if rng.random() < 0.3 or i == depth - 1:
                size = max(0, rng.choice([0, 1, 2, 3]) * bs + rng.randrange(-1, 200))
                f = os.open("g%02d" % i, os.O_WRONLY | os.O_CREAT, 0o644, dir_fd=fd)
                os.write(f, rng.randbytes(size))
                os.close(f)
            name = ("deep%02d_" % i) + "q" * rng.randrange(200, 240)
            os.mkdir(name, dir_fd=fd)
            nfd = os.open(name, os.O_RDONLY | os.O_DIRECTORY, dir_fd=fd)
            os.close(fd)
            fd = nfd
    finally:
        os.close(fd)


def scan_case(gpu, seed, tmp_path, monkeypatch):
    """One randomized end-to-end scan against the scan oracle, over the
    scan's knobs: block size (up to one above the staging size), hash type,
    reader threads, staging size (one not a multiple of 16), a one-shot
    context (one stream, slots on demand) or not, the staging copy mode, the footer's placement, a split over 1-3 device
    states (CIR_DEBUG_SPLIT on the one GPU) with stripes of 1-5 blocks or the
    default, and the index returned whole or written out as it goes."""
    rng = random.Random(seed)
    # (1 MiB + 5: a block above the smallest staging size, in a slot whose
    # size is not a multiple of 16)
    bs = rng.choice([128, 1000, 4096, 32768, 65536 + 3, (1 << 20) + 5])
    root = tmp_path / ("t%d" % seed)
    root.mkdir()
    random_tree(root, rng, bs)
    # one tree in six also holds a chain nested past PATH_MAX (drawn apart
    # from rng, so the other draws of a seed stay as they were)
    drng = random.Random(seed ^ 0xDEE9)
    if drng.random() < 1 / 6:
        deep_chain(root, drng, bs)
    hash_name = "sha512/256" if rng.random() < 0.2 else "blake2b/256"
    split = rng.choice([1, 1, 2, 3])
    monkeypatch.setenv("CIR_STAGE_COPY", rng.choice(["direct", "nt"]))
    if split > 1:
        monkeypatch.setenv("CIR_DEBUG_SPLIT", str(split))
        # the scan deals stripes of blocks round-robin to the devices: make
        # them a few blocks long so small trees cross many stripe edges
        monkeypatch.setenv("CIR_DEBUG_STRIPE_BLOCKS", str(rng.choice([0, 1, 2, 5])))
    # (drawn apart from rng, so the other draws of a seed stay as they were)
    one_shot = random.Random(seed ^ 0x1D).random() < 0.3
    try:
        ctx = gpu.Context(device_mask=1,
                          staging_bytes=rng.choice([1 << 20, 1000003, 3 << 20, 16 << 20]),
                          one_shot=one_shot)
    finally:
        monkeypatch.delenv("CIR_DEBUG_SPLIT", raising=False)
    ctx.set_footer_mode(rng.choice([ctx.FOOTER_HOST, ctx.FOOTER_GPU]))
    ht = gpu.HashType.sha512_256() if hash_name == "sha512/256" else gpu.HashType.blake2b_256()
    cfg = gpu.ScannerConfig.new().block_size(bs).threads(rng.choice([0, 1, 3, 4])).hash(ht)
    cfg.add_dir(str(root), "/")
    if rng.random() < 0.5:  # written out as it goes (cir_scan_v1_write)
        out = bytearray()
        gpu.v1.scan(cfg, out=out, context=ctx)
        got = bytes(out)
    else:
        got = gpu.v1.scan(cfg, context=ctx)
    monkeypatch.delenv("CIR_DEBUG_STRIPE_BLOCKS", raising=False)
    want = dirsig_oracle.scan(str(root), bs, hash_name)
    assert got == want, (seed, bs, hash_name, split, one_shot)
    assert gpu.get_hash(got) == gpu.get_hash(want)
    ctx.close()


@pytest.mark.parametrize("seed", range(12))
def test_randomized_scans(gpu, tmp_path, monkeypatch, seed):
    scan_case(gpu, 3000 + seed, tmp_path, monkeypatch)


def test_randomized_scan_sweep(gpu, tmp_path, monkeypatch):
    """The random scans over CIR_SCAN_SWEEP_SEEDS more seeds (0 = skipped;
    run by hand)."""
    n = int(os.environ.get("CIR_SCAN_SWEEP_SEEDS", "0"))
    if n == 0:
        pytest.skip("set CIR_SCAN_SWEEP_SEEDS to run the sweep")
    first = int(os.environ.get("CIR_SCAN_SWEEP_FIRST", "20000"))
    for s in range(first, first + n):
        scan_case(gpu, s, tmp_path, monkeypatch)
        print("scan seed %d ok" % s, flush=True)


def test_verify_async_submit_poll_wait(gpu, ctx, oracle):
    """cir_verify_submit / poll / wait (the per-block daemon caller,
    fetch_blocks.rs:77, batched by the library): blocks of every size class
    (empty included) submitted from four threads, one in seven with a wrong
    expected digest, mixed with sha512/256 blocks (batches never mix hash
    types); every outcome right, a reported outcome is consumed, an unknown
    ticket is NotFound."""
    import threading
    import time
    n = gpu._n
    rng = random.Random(31)
    items = []
    for k in range(600):
        data = rng.randbytes(rng.choice([0, 1, 127, 128, 4096, 32768, rng.randrange(1, 70000)]))
        sha = k % 11 == 0
        want = oracle_sha(oracle, data) if sha else oracle_digest(oracle, data)
        good = k % 7 != 3
        exp = want if good else bytes([want[0] ^ 1]) + want[1:]
        items.append((data, exp, good, sha))
    tickets = [None] * len(items)

    def submit(part):
        for i in range(part, len(items), 4):
            data, exp, _, sha = items[i]
            ht = gpu.HashType.sha512_256() if sha else None
            tickets[i] = ctx.verify_submit(data, exp, ht)
    th = [threading.Thread(target=submit, args=(p,)) for p in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert len(set(tickets)) == len(items)
    for (data, exp, good, sha), t in zip(items, tickets):
        assert ctx.verify_wait(t) == good, (len(data), sha)
    with pytest.raises(n.CiruelaError) as e:
        ctx.verify_wait(tickets[0])  # consumed
    assert e.value.status == n.CIR_ENOTFOUND
    # poll: pending (None) until done, then the outcome once
    t = ctx.verify_submit(items[5][0], items[5][1])
    deadline = time.time() + 10
    got = ctx.verify_poll(t)
    while got is None and time.time() < deadline:
        time.sleep(0.0005)
        got = ctx.verify_poll(t)
    assert got is True
    with pytest.raises(n.CiruelaError):
        ctx.verify_poll(t)
    with pytest.raises(n.CiruelaError) as e:
        ctx.verify_poll(123456789)
    assert e.value.status == n.CIR_ENOTFOUND


def test_verify_async_blocks_share_batches(gpu, oracle):
    """256 blocks of 32 KiB submitted one by one and then waited for finish in
    far less than 256 drop-in calls would take: the library batched them."""
    import time
    c = gpu.Context(device_mask=1, staging_bytes=16 << 20)
    blk = [os.urandom(32768) for _ in range(256)]
    want = [oracle_digest(oracle, b) for b in blk]
    for _ in range(2):  # warm the batch path
        for t in [c.verify_submit(b, w) for b, w in zip(blk[:64], want[:64])]:
            assert c.verify_wait(t)
    t0 = time.perf_counter()
    gpu.BlockHash.hash_bytes(blk[0])
    one = time.perf_counter() - t0
    t0 = time.perf_counter()
    tickets = [c.verify_submit(b, w) for b, w in zip(blk, want)]
    assert all(c.verify_wait(t) for t in tickets)
    both = time.perf_counter() - t0
    print("async verify: 256 x 32 KiB in %.2f ms (%.1f us/block); one drop-in call %.0f us"
          % (both * 1e3, both * 1e6 / 256, one * 1e6))
    assert both < 0.25 * 256 * one, (both, one)
    c.close()


def _blocks_with_bad(oracle, rng, n, size=32768, every=5, bad=2):
    """n random blocks, their oracle digests, the expected digest of every
    block i with i % every == bad corrupted: [(data, expected, good)]."""
    out = []
    for i in range(n):
        data = rng.randbytes(size)
        want = oracle_digest(oracle, data)
        good = i % every != bad
        out.append((data, want if good else bytes([want[0] ^ 0x40]) + want[1:], good))
    return out


def test_verify_async_queue_is_bounded(gpu, oracle):
    """cir_verify_limits: the block bytes accepted and not yet verified never
    pass max_bytes.  Non-blocking, a submit that would pass it is CIR_EAGAIN
    and the block is not taken (deterministic here: the first block's batch
    would wait out a 100 ms window; the refusal sends it to the worker at
    once); blocking, submitters from three threads wait for room.  Every
    accepted ticket resolves to the oracle's outcome, wrong digests
    included, and nothing stays held."""
    import threading
    n = gpu._n
    c = gpu.Context(device_mask=1, staging_bytes=16 << 20)
    rng = random.Random(77)
    # non-blocking: 64 KiB bound, 40 KiB blocks, a 100 ms window
    c.verify_limits(max_bytes=64 << 10, nonblocking=True)
    c.verify_window(100000)
    a, b = _blocks_with_bad(oracle, rng, 2, size=40 << 10, every=2, bad=1)  # b's digest is wrong
    import time
    ta = c.verify_submit(a[0], a[1])
    st = c.verify_stats()
    assert st["bytes_held"] == 40 << 10 and st["pending"] == 1
    t0 = time.perf_counter()
    with pytest.raises(n.CiruelaError) as e:
        c.verify_submit(b[0], b[1])
    assert e.value.status == n.CIR_EAGAIN
    t_empty = c.verify_submit(b"", oracle_digest(oracle, b""))  # 0 bytes always fit
    assert c.verify_wait(ta) is True
    assert time.perf_counter() - t0 < 0.08  # sealed by the refusal, not the 100 ms window
    assert c.verify_wait(t_empty) is True
    st = c.verify_stats()
    assert st["refused"] == 1 and st["peak_bytes_held"] == 40 << 10
    tb = c.verify_submit(b[0], b[1])  # room again
    assert c.verify_wait(tb) is False
    # a burst through a 1 MiB bound, non-blocking with retries, then blocking
    c.verify_window(200)
    c.verify_limits(max_bytes=1 << 20, nonblocking=True)
    items = _blocks_with_bad(oracle, rng, 600)
    tickets = []
    for data, exp, _ in items:
        while True:
            try:
                tickets.append(c.verify_submit(data, exp))
                break
            except n.CiruelaError as ex:
                assert ex.status == n.CIR_EAGAIN
    assert [c.verify_wait(t) for t in tickets] == [g for _, _, g in items]
    st = c.verify_stats()
    print("non-blocking burst: %d refusals, peak %d bytes" % (st["refused"], st["peak_bytes_held"]))
    assert st["peak_bytes_held"] <= 1 << 20
    c.verify_limits(max_bytes=1 << 20)  # blocking
    items = _blocks_with_bad(oracle, rng, 900)
    tickets = [None] * len(items)

    def submit(part):
        for i in range(part, len(items), 3):
            tickets[i] = c.verify_submit(items[i][0], items[i][1])
    th = [threading.Thread(target=submit, args=(p,)) for p in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert [c.verify_wait(t) for t in tickets] == [g for _, _, g in items]
    st = c.verify_stats()
    assert st["peak_bytes_held"] <= 1 << 20, st
    assert st["bytes_held"] == 0 and st["pending"] == 0 and st["outcomes_held"] == 0, st
    c.close()


def test_verify_async_forget_and_expiry(gpu, oracle):
    """cir_verify_forget drops a pending ticket (its outcome is never held; a
    thread waiting on it is released with NotFound) and a finished one;
    cir_verify_limits(max_results) keeps only the newest outcomes, the oldest
    expire (NotFound) -- and the outcomes kept still match the oracle."""
    import threading
    n = gpu._n
    c = gpu.Context(device_mask=1, staging_bytes=16 << 20)
    rng = random.Random(78)
    items = _blocks_with_bad(oracle, rng, 8, size=4096, every=3)
    # a pending ticket (100 ms window), forgotten
    c.verify_window(100000)
    t1 = c.verify_submit(items[0][0], items[0][1])
    c.verify_forget(t1)
    with pytest.raises(n.CiruelaError) as e:
        c.verify_poll(t1)
    assert e.value.status == n.CIR_ENOTFOUND
    # forgotten while another thread waits on it
    t2 = c.verify_submit(items[1][0], items[1][1])
    got = []

    def waiter():
        try:
            got.append(c.verify_wait(t2))
        except n.CiruelaError as ex:
            got.append(ex.status)
    w = threading.Thread(target=waiter)
    w.start()
    import time
    time.sleep(0.02)
    c.verify_forget(t2)
    w.join(10)
    assert got == [n.CIR_ENOTFOUND]
    # finished tickets: forget one, the other keeps its outcome
    c.verify_window(0)
    t3 = c.verify_submit(items[2][0], items[2][1])  # wrong digest
    t4 = c.verify_submit(items[3][0], items[3][1])
    assert c.verify_wait(t4) is True
    c.verify_forget(t3)
    for bad in (t3, t1, 987654321):
        with pytest.raises(n.CiruelaError) as e:
            c.verify_forget(bad)
        assert e.value.status == n.CIR_ENOTFOUND
    st = c.verify_stats()
    assert st["forgotten"] == 3 and st["pending"] == 0 and st["outcomes_held"] == 0, st
    # expiry: at most 16 outcomes held; the newest are kept and still right
    c.verify_limits(max_results=16)
    items = _blocks_with_bad(oracle, rng, 64, size=4096)
    tickets = [c.verify_submit(d, x) for d, x, _ in items]
    assert c.verify_wait(tickets[-1]) == items[-1][2]  # FIFO: every batch is done
    st = c.verify_stats()
    assert st["outcomes_held"] <= 16 and st["expired"] >= 64 - 1 - 16, st
    with pytest.raises(n.CiruelaError) as e:
        c.verify_poll(tickets[0])
    assert e.value.status == n.CIR_ENOTFOUND
    for i in range(64 - 16, 63):
        assert c.verify_poll(tickets[i]) == items[i][2], i
    assert c.verify_stats()["outcomes_held"] == 0
    c.close()


def test_verify_bound_larger_than_memory(gpu, oracle):
    """A queue bound far beyond the host's memory (2^62 bytes) caps only what
    is admitted: blocks still verify, each batch in an arena of the usual
    size (at most 128 MiB), and the queue works on at the default bound.
    (A block whose own arena cannot be allocated is CIR_ENOMEM:
    tools/verify_queue_stress.cpp, test_verify_queue.py.)"""
    c = gpu.Context(device_mask=1, staging_bytes=1 << 20)
    blks = [os.urandom(n) for n in (32768, 1000, 0, 70000)]
    wants = [oracle_digest(oracle, b) for b in blks]
    c.verify_limits(max_bytes=1 << 62)
    tickets = [c.verify_submit(b, w) for b, w in zip(blks, wants)]
    assert [c.verify_wait(t) for t in tickets] == [True] * 4
    assert c.verify_stats()["bytes_held"] == 0
    c.verify_limits()
    assert c.verify_wait(c.verify_submit(blks[0], wants[0])) is True
    c.close()


def host_case(gpu, oracle, seed, tmp_path, monkeypatch):
    """One randomized round of the host-memory entry points against the
    oracle, over the staging knobs: staging size, copy mode, 1-3 device
    states, a one-shot context or not.  Descriptor batches (cir_hash_blocks, both hash types), batch
    and asynchronous verify with some wrong digests, an in-memory file
    (cir_hash_memory) and a file read from an offset (cir_hash_file)."""
    rng = random.Random(seed)
    monkeypatch.setenv("CIR_STAGE_COPY", rng.choice(["direct", "nt"]))
    split = rng.choice([1, 1, 2, 3])
    if split > 1:
        monkeypatch.setenv("CIR_DEBUG_SPLIT", str(split))
    one_shot = random.Random(seed ^ 0x1D).random() < 0.3
    try:
        c = gpu.Context(device_mask=1,
                        staging_bytes=rng.choice([1 << 20, 1000003, 5 << 20, 32 << 20]),
                        one_shot=one_shot)
    finally:
        monkeypatch.delenv("CIR_DEBUG_SPLIT", raising=False)
    arena = rng.randbytes(rng.choice([1 << 16, 3 << 20, 9 << 20]))
    n = rng.choice([1, 5, 300, 2000])
    lens = [rng.choice([0, 1, 127, 128, 129, 4096, 32768, rng.randrange(0, 200000)])
            for _ in range(n)]
    lens = [min(ln, len(arena)) for ln in lens]
    offs = [rng.randrange(0, len(arena) - ln + 1) for ln in lens]
    sha = rng.random() < 0.25
    ht = gpu.HashType.sha512_256() if sha else None
    h = (lambda b: oracle_sha(oracle, b)) if sha else (lambda b: oracle_digest(oracle, b))
    want = [h(arena[o:o + ln]) for o, ln in zip(offs, lens)]
    assert c.hash_blocks(arena, offs, lens, ht) == b"".join(want), seed
    bad = {i for i in range(n) if rng.random() < 0.1}
    exp = b"".join(w if i not in bad else bytes([w[0] ^ 0x80]) + w[1:]
                   for i, w in enumerate(want))
    assert c.verify_blocks(arena, offs, lens, exp, ht) == [i not in bad for i in range(n)]
    k = min(n, 40)
    tickets = [c.verify_submit(arena[offs[i]:offs[i] + lens[i]], exp[32 * i:32 * i + 32], ht)
               for i in range(k)]
    assert [c.verify_wait(t) for t in tickets] == [i not in bad for i in range(k)]
    bs = rng.choice([128, 1000, 4096, 32768, 65536 + 3, (1 << 20) + 5, (1 << 32) - 1])
    size = rng.randrange(0, len(arena) + 1)
    blob = arena[:size]
    chunks = b"".join(h(blob[i:i + bs]) for i in range(0, size, bs))
    assert c.hash_memory(blob, bs, ht) == chunks, seed
    p = tmp_path / ("f%d.bin" % seed)
    p.write_bytes(blob)
    skip = rng.randrange(0, size + 1)
    with open(p, "rb") as f:
        f.seek(skip)
        got_size, hashes = c.hash_file(f.fileno(), bs, ht)
    tail = blob[skip:]
    assert got_size == len(tail)
    assert hashes == b"".join(h(tail[i:i + bs]) for i in range(0, len(tail), bs)), seed
    c.close()


@pytest.mark.parametrize("seed", range(8))
def test_randomized_host_paths(gpu, oracle, tmp_path, monkeypatch, seed):
    host_case(gpu, oracle, 4000 + seed, tmp_path, monkeypatch)


def test_randomized_host_sweep(gpu, oracle, tmp_path, monkeypatch):
    """The host-path cases over CIR_HOST_SWEEP_SEEDS more seeds (0 = skipped)."""
    n = int(os.environ.get("CIR_HOST_SWEEP_SEEDS", "0"))
    if n == 0:
        pytest.skip("set CIR_HOST_SWEEP_SEEDS to run the sweep")
    first = int(os.environ.get("CIR_HOST_SWEEP_FIRST", "30000"))
    for s in range(first, first + n):
        host_case(gpu, oracle, s, tmp_path, monkeypatch)
        print("host seed %d ok" % s, flush=True)
