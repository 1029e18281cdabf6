"""Untrusted descriptors on the device (cir_hash_blocks_dev_bounded,
cir_verify_blocks_dev_bounded): the daemon's received blocks arrive with
offsets and lengths from another party (src/daemon/tracking/fetch_blocks.rs:
77,91-103).  A descriptor that leaves the arena -- past its end, or with
off + len wrapping around 2^64 -- must not be read: it is flagged (zero
digest and a device count for hashing, a mismatch for verify) and every
other block's digest equals the oracle's.  Each case runs once; a kernel
reading such a descriptor would be a GPU memory fault (offsets of 2^40 and
2^64 - 16 lie far outside any allocation), so these tests also show that
nothing out of range is touched.
"""
import random

import numpy as np
import pytest

from conftest import oracle_digest, oracle_sha

pytestmark = pytest.mark.gpu

U64 = (1 << 64) - 1


@pytest.fixture(scope="module")
def ctx(gpu):
    return gpu.Context(device_mask=1, staging_bytes=8 << 20)


def _batch(rng, n, arena_bytes, long_every=0):
    """n descriptors inside [0, arena_bytes), some long, some empty."""
    offs, lens = [], []
    for i in range(n):
        if long_every and i % long_every == 0:
            ln = rng.choice([1 << 20, (1 << 20) + 77, 300 * 128])
        else:
            ln = rng.choice([0, 1, 127, 128, 4096, 32768, rng.randrange(0, 40000)])
        ln = min(ln, arena_bytes)
        offs.append(rng.randrange(0, arena_bytes - ln + 1))
        lens.append(ln)
    return offs, lens


def _poison(rng, offs, lens, arena_bytes, k):
    """Replace k descriptors by out-of-range ones of every kind; returns the
    flagged indices."""
    kinds = [
        lambda: (arena_bytes - 10, 11),          # one byte past the end
        lambda: (arena_bytes + 1, 0),            # empty, but starts past the end
        lambda: (1 << 40, 32768),                # far outside any allocation
        lambda: (U64 - 15, 100),                 # off + len wraps around 2^64
        lambda: (U64, 1),                        # wraps to 0
        lambda: (arena_bytes - 4096, 0xFFFFFFFF),  # longest length
    ]
    bad = sorted(rng.sample(range(8, len(offs)), k))  # 0..7: the in-range edge cases
    for j, b in enumerate(bad):
        offs[b], lens[b] = kinds[j % len(kinds)]()
    return bad


def _edges_in_range(arena_bytes):
    """Descriptors at the arena's very end: all in range."""
    return [(arena_bytes - 10, 10), (arena_bytes, 0), (0, arena_bytes), (0, 0)]


def _to_dev(torch, host, offs, lens):
    d_arena = torch.from_numpy(host).to("cuda:0")
    d_off = torch.tensor(np.array(offs, dtype=np.uint64).view(np.int64), device="cuda:0")
    d_len = torch.tensor(np.array(lens, dtype=np.uint32).view(np.int32), device="cuda:0")
    return d_arena, d_off, d_len


def _want_blake(oracle, host, offs, lens, bad):
    ao = np.array([0 if i in bad else o for i, o in enumerate(offs)], dtype=np.uint64)
    al = np.array([0 if i in bad else ln for i, ln in enumerate(lens)], dtype=np.uint32)
    want = np.zeros(32 * len(offs), dtype=np.uint8)
    oracle.oracle_hash_blocks(host.ctypes.data, ao.ctypes.data, al.ctypes.data, len(offs),
                              want.ctypes.data, 8)
    want = want.reshape(-1, 32)
    want[sorted(bad)] = 0
    return want


def _flagged(dig):
    return [i for i, row in enumerate(dig) if not row.any()]


@pytest.mark.parametrize("with_ctx", [True, False])
@pytest.mark.parametrize("n,long_every", [(700, 0), (900, 50), (60000, 997)])
def test_hash_bounded_flags_out_of_range(gpu, ctx, oracle, with_ctx, n, long_every):
    """Ordered (context: lane part, quad part, relays at 60000) and
    unordered (no context) batches."""
    import torch
    rng = random.Random(n * 7 + long_every + with_ctx)
    arena_bytes = (24 << 20) + 5
    # the arena sits inside a larger buffer: a read one byte past arena_bytes
    # would not fault, so only the flags show the exact bound
    host = np.frombuffer(rng.randbytes(arena_bytes + 4096), dtype=np.uint8).copy()
    offs, lens = _batch(rng, n, arena_bytes, long_every)
    for j, (o, ln) in enumerate(_edges_in_range(arena_bytes)):
        offs[j + 1], lens[j + 1] = o, ln
    bad = _poison(rng, offs, lens, arena_bytes, 11)
    d_arena, d_off, d_len = _to_dev(torch, host, offs, lens)
    out = torch.full((32 * n,), 0xAB, dtype=torch.uint8, device="cuda:0")
    nrange = torch.full((1,), 999, dtype=torch.int32, device="cuda:0")
    gpu._n.check(gpu._n.lib.cir_hash_blocks_dev_bounded(
        ctx.handle if with_ctx else None, 1, d_arena.data_ptr(), arena_bytes, d_off.data_ptr(),
        d_len.data_ptr(), n, out.data_ptr(), nrange.data_ptr(), None))
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(-1, 32)
    want = _want_blake(oracle, host, offs, lens, set(bad))
    diff = np.nonzero((got != want).any(1))[0]
    assert diff.size == 0, (diff[:10], [(offs[i], lens[i]) for i in diff[:10]])
    assert _flagged(got) == bad
    assert int(nrange.item()) == len(bad)


def test_hash_bounded_matches_unbounded_on_good_batch(gpu, ctx):
    """No descriptor out of range: the bounded call's digests are the plain
    call's, and the count is 0 (also with a NULL counter)."""
    import torch
    rng = random.Random(5)
    arena_bytes = 8 << 20
    host = np.frombuffer(rng.randbytes(arena_bytes), dtype=np.uint8).copy()
    offs, lens = _batch(rng, 3000, arena_bytes, 200)
    d_arena, d_off, d_len = _to_dev(torch, host, offs, lens)
    a = torch.zeros(32 * 3000, dtype=torch.uint8, device="cuda:0")
    b = torch.ones(32 * 3000, dtype=torch.uint8, device="cuda:0")
    nrange = torch.full((1,), 7, dtype=torch.int32, device="cuda:0")
    ctx.hash_blocks_dev(d_arena.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), 3000,
                        a.data_ptr())
    ctx.hash_blocks_dev_bounded(d_arena.data_ptr(), arena_bytes, d_off.data_ptr(),
                                d_len.data_ptr(), 3000, b.data_ptr(), nrange.data_ptr())
    c2 = torch.full((32 * 3000,), 3, dtype=torch.uint8, device="cuda:0")
    ctx.hash_blocks_dev_bounded(d_arena.data_ptr(), arena_bytes, d_off.data_ptr(),
                                d_len.data_ptr(), 3000, c2.data_ptr(), 0)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(a, c2)
    assert int(nrange.item()) == 0


def test_hash_bounded_sha512(gpu, ctx, oracle):
    import torch
    rng = random.Random(77)
    arena_bytes = 2 << 20
    host = np.frombuffer(rng.randbytes(arena_bytes), dtype=np.uint8).copy()
    offs, lens = _batch(rng, 300, arena_bytes)
    bad = _poison(rng, offs, lens, arena_bytes, 9)
    d_arena, d_off, d_len = _to_dev(torch, host, offs, lens)
    out = torch.full((32 * 300,), 0xAB, dtype=torch.uint8, device="cuda:0")
    nrange = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    ctx.hash_blocks_dev_bounded(d_arena.data_ptr(), arena_bytes, d_off.data_ptr(),
                                d_len.data_ptr(), 300, out.data_ptr(), nrange.data_ptr(),
                                hash_type=gpu.HashType.sha512_256())
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(-1, 32)
    raw = host.tobytes()
    for i, (o, ln) in enumerate(zip(offs, lens)):
        want = bytes(32) if i in bad else oracle_sha(oracle, raw[o:o + ln])
        assert got[i].tobytes() == want, i
    assert int(nrange.item()) == len(bad)


@pytest.mark.parametrize("ht", ["blake2b", "sha512"])
@pytest.mark.parametrize("with_ctx", [True, False])
def test_verify_bounded_out_of_range_is_a_mismatch(gpu, ctx, oracle, ht, with_ctx):
    """Row f2 with peer-supplied descriptors: an out-of-range block takes the
    mismatch branch (fetch_blocks.rs:91-103) like a corrupted one."""
    import torch
    rng = random.Random(31 + with_ctx)
    hasht = gpu.HashType.blake2b_256() if ht == "blake2b" else gpu.HashType.sha512_256()
    arena_bytes = 6 << 20
    host = np.frombuffer(rng.randbytes(arena_bytes + 64), dtype=np.uint8).copy()
    n = 800
    offs, lens = _batch(rng, n, arena_bytes, 100 if ht == "blake2b" else 0)
    raw = host.tobytes()
    if ht == "blake2b":
        expected = bytearray(_want_blake(oracle, host, offs, lens, set()).tobytes())
    else:
        expected = bytearray(b"".join(oracle_sha(oracle, raw[o:o + ln])
                                      for o, ln in zip(offs, lens)))
    # corrupt some expected digests, put others out of range (their expected
    # digest stays the true one of the original block: still a mismatch)
    corrupt = set(rng.sample(range(n), 13))
    for b in corrupt:
        expected[32 * b + rng.randrange(32)] ^= 0x40
    bad = _poison(rng, offs, lens, arena_bytes, 10)
    # an out-of-range block whose expected digest is all zeros (its digest
    # buffer is zeroed) must still fail
    expected[32 * bad[0]:32 * bad[0] + 32] = bytes(32)
    d_arena, d_off, d_len = _to_dev(torch, host, offs, lens)
    d_exp = torch.tensor(expected, dtype=torch.uint8, device="cuda:0")
    d_dig = torch.full((32 * n,), 0x55, dtype=torch.uint8, device="cuda:0")
    d_ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda:0")
    d_nbad = torch.full((1,), 12345, dtype=torch.int32, device="cuda:0")
    gpu._n.check(gpu._n.lib.cir_verify_blocks_dev_bounded(
        ctx.handle if with_ctx else None, hasht.code, d_arena.data_ptr(), arena_bytes,
        d_off.data_ptr(), d_len.data_ptr(), n, d_exp.data_ptr(), d_dig.data_ptr(),
        d_ok.data_ptr(), d_nbad.data_ptr(), None))
    torch.cuda.synchronize()
    ok = d_ok.cpu().tolist()
    assert set(ok) <= {0, 1}
    assert [i for i, g in enumerate(ok) if not g] == sorted(corrupt | set(bad))
    assert int(d_nbad.item()) == len(corrupt | set(bad))
    assert _flagged(d_dig.cpu().numpy().reshape(-1, 32)) == bad


def test_bounded_empty_and_argument_errors(gpu, ctx):
    import torch
    nrange = torch.full((1,), 5, dtype=torch.int32, device="cuda:0")
    nbad = torch.full((1,), 5, dtype=torch.int32, device="cuda:0")
    ctx.hash_blocks_dev_bounded(0, 0, 0, 0, 0, 0, nrange.data_ptr())
    ctx.verify_blocks_dev_bounded(0, 0, 0, 0, 0, 0, 0, 0, nbad.data_ptr())
    torch.cuda.synchronize()
    assert int(nrange.item()) == 0 and int(nbad.item()) == 0
    d = torch.zeros(64, dtype=torch.uint8, device="cuda:0")
    off = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    ln = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    with pytest.raises(gpu.CiruelaError) as e:  # misaligned digest buffer
        ctx.hash_blocks_dev_bounded(d.data_ptr(), 64, off.data_ptr(), ln.data_ptr(), 1,
                                    d.data_ptr() + 8)
    assert e.value.status == gpu._n.CIR_EINVAL
    with pytest.raises(gpu.CiruelaError) as e:  # unknown hash type
        gpu._n.check(gpu._n.lib.cir_hash_blocks_dev_bounded(
            ctx._h, 9, d.data_ptr(), 64, off.data_ptr(), ln.data_ptr(), 1, d.data_ptr(), None,
            None))
    assert e.value.status == gpu._n.CIR_EINVAL
    # a NULL arena of size 0: every non-empty block is out of range
    out = torch.full((32,), 1, dtype=torch.uint8, device="cuda:0")
    ln.fill_(5)
    ctx.hash_blocks_dev_bounded(0, 0, off.data_ptr(), ln.data_ptr(), 1, out.data_ptr(),
                                nrange.data_ptr())
    torch.cuda.synchronize()
    assert int(nrange.item()) == 1 and not out.any()


@pytest.mark.parametrize("ht", ["blake2b", "sha512"])
def test_host_bounded_batches(gpu, oracle, ht):
    """cir_hash_blocks_bounded / cir_verify_blocks_bounded: the host twins.
    Out-of-range descriptors (the same kinds) are never read -- one of 2^40
    past a 3 MiB arena would fault the process -- their digests are zeros
    and they fail verification; the rest equal the oracle's.  Through a
    context with two device states (the split host path) too."""
    import ctypes
    from ciruela_amd import _native as n
    hasht = gpu.HashType.blake2b_256() if ht == "blake2b" else gpu.HashType.sha512_256()
    dig = (lambda d: oracle_digest(oracle, d)) if ht == "blake2b" else \
        (lambda d: oracle_sha(oracle, d))
    rng = random.Random(91 + len(ht))
    arena_bytes = 3 << 20
    arena = rng.randbytes(arena_bytes)
    offs, lens = _batch(rng, 500, arena_bytes, 60 if ht == "blake2b" else 0)
    for j, (o, ln) in enumerate(_edges_in_range(arena_bytes)):
        offs[j + 1], lens[j + 1] = o, ln
    bad = _poison(rng, offs, lens, arena_bytes, 9)
    want = [bytes(32) if i in bad else dig(arena[o:o + ln])
            for i, (o, ln) in enumerate(zip(offs, lens))]
    for split in ("1", "2"):
        import os
        os.environ["CIR_DEBUG_SPLIT"] = split
        try:
            c = gpu.Context(device_mask=1, staging_bytes=1 << 20)
        finally:
            del os.environ["CIR_DEBUG_SPLIT"]
        k = len(offs)
        ao = (ctypes.c_uint64 * k)(*offs)
        al = (ctypes.c_uint32 * k)(*lens)
        buf = ctypes.create_string_buffer(arena, arena_bytes)
        out = ctypes.create_string_buffer(32 * k)
        nrange = ctypes.c_size_t(77)
        n.check(n.lib.cir_hash_blocks_bounded(c.handle, hasht.code, buf, arena_bytes, ao, al, k,
                                              out, ctypes.byref(nrange)))
        got = [out.raw[32 * i:32 * i + 32] for i in range(k)]
        assert [i for i in range(k) if got[i] != want[i]] == []
        assert nrange.value == len(bad)
        # verify: expected = the true digests of the original blocks (as a
        # peer would claim), one corrupted, one out-of-range block expecting
        # zeros
        exp = bytearray(b"".join(want))
        exp[32 * 5] ^= 1
        ok = c.verify_blocks_bounded(arena, offs, lens, bytes(exp), hash_type=hasht)
        assert [i for i, g in enumerate(ok) if not g] == sorted(set(bad) | {5})
        c.close()
