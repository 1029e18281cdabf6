"""Where the GPU batch verify beats one host core.

The daemon re-hashes every received block (`BlockHash::hash_bytes(&data)
== blk.hash`, reference src/daemon/tracking/fetch_blocks.rs:77).  Per call
through the drop-in `cir_blake2b256` one 32 KiB block costs one GPU chain's
latency; batched through `cir_verify_blocks` (host arena in, per-block ok
out) the chains run side by side.  This times, for n 32 KiB blocks:
  * gpu_batch_us: one cir_verify_blocks call over the n blocks (host memory
    in and out, the process-default context), median of --calls;
  * gpu_single_us: n calls of cir_blake2b256 (the drop-in) one after
    another, from the median single call;
  * gpu_concurrent_us: the same n calls made at once from n host threads
    (the drop-in coalesces callers that queue while a launch runs), median;
  * gpu_async_us: n blocks submitted one by one with cir_verify_submit
    and then waited for (the library batches what arrives within its
    window), median;
  * cpu_core_us: n blocks hashed by hashlib.blake2b(digest_size=32) on one
    host thread (CPython's C BLAKE2b: a stand-in for one core running the
    reference's `blake2` crate; not the oracle), median per block;
and prints the smallest n at which the batch call beats the host core.
Every GPU result is checked against hashlib first.

    python tools/verify_crossover.py [--calls 20]
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BS = 32768


def median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=20)
    args = ap.parse_args()
    import ciruela_amd as ca
    n_ = ca._n
    ctx = ca.default_context()
    sizes = [1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 4096]
    rng = np.random.default_rng(77)
    arena = rng.integers(0, 256, size=max(sizes) * BS, dtype=np.uint8)
    raw = arena.tobytes()
    want = b"".join(hashlib.blake2b(raw[i * BS:(i + 1) * BS], digest_size=32).digest()
                    for i in range(max(sizes)))
    exp = np.frombuffer(want, dtype=np.uint8).copy()
    # one host core, per block
    cpu = []
    for i in range(200):
        blk = raw[(i % 64) * BS:(i % 64 + 1) * BS]
        t0 = time.perf_counter()
        hashlib.blake2b(blk, digest_size=32).digest()
        cpu.append(time.perf_counter() - t0)
    cpu_blk = median(cpu)
    # the drop-in, one call per block
    one = raw[:BS]
    for _ in range(5):
        assert bytes(ca.BlockHash.hash_bytes(one)) == want[:32]
    single = []
    for _ in range(max(20, args.calls)):
        t0 = time.perf_counter()
        ca.BlockHash.hash_bytes(one)
        single.append(time.perf_counter() - t0)
    single_blk = median(single)
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(256)
    blocks = [raw[i * BS:(i + 1) * BS] for i in range(max(sizes))]

    def concurrent(n):
        futs = [pool.submit(lambda b: bytes(ca.BlockHash.hash_bytes(b)), blocks[i])
                for i in range(n)]
        return [f.result() for f in futs]
    rows = []
    for n in sizes:
        offs = np.arange(n, dtype=np.uint64) * BS
        lens = np.full(n, BS, dtype=np.uint32)
        ok = np.zeros(n, dtype=np.uint8)
        nbad = ctypes.c_size_t()

        def call():
            n_.check(n_.lib.cir_verify_blocks(ctx.handle, 1, arena.ctypes.data, offs.ctypes.data,
                                              lens.ctypes.data, n, exp.ctypes.data,
                                              ok.ctypes.data, ctypes.byref(nbad)))
        for _ in range(3):
            call()
        assert nbad.value == 0 and ok.all(), n
        ts = []
        for _ in range(args.calls):
            t0 = time.perf_counter()
            call()
            ts.append(time.perf_counter() - t0)
        g = median(ts)
        conc = None
        if n <= 256:
            got = concurrent(n)
            assert b"".join(got) == want[:32 * n], n
            tc = []
            for _ in range(max(5, args.calls // 2)):
                t0 = time.perf_counter()
                concurrent(n)
                tc.append(time.perf_counter() - t0)
            conc = median(tc)
        asy = []
        for _ in range(max(5, args.calls // 2)):
            t0 = time.perf_counter()
            tk = [ctx.verify_submit(blocks[i], want[32 * i:32 * i + 32]) for i in range(n)]
            assert all(ctx.verify_wait(t) for t in tk)
            asy.append(time.perf_counter() - t0)
        a_us = median(asy)
        rows.append({"n": n, "gpu_async_us": round(a_us * 1e6, 1),
                     "gpu_batch_us": round(g * 1e6, 1),
                     "gpu_batch_us_per_block": round(g * 1e6 / n, 2),
                     "gpu_single_us": round(single_blk * 1e6 * n, 1),
                     "gpu_concurrent_us": None if conc is None else round(conc * 1e6, 1),
                     "cpu_core_us": round(cpu_blk * 1e6 * n, 1)})
        print("n=%-5d batch %9.1f us (%7.2f us/block)  async %9.1f us  drop-in %9.1f us  "
              "drop-in x n threads %9s us  one core %9.1f us"
              % (n, g * 1e6, g * 1e6 / n, a_us * 1e6, single_blk * 1e6 * n,
                 "-" if conc is None else "%.1f" % (conc * 1e6), cpu_blk * 1e6 * n), flush=True)
    cross = next((r["n"] for r in rows if r["gpu_batch_us"] < r["cpu_core_us"]), None)
    print(json.dumps({"block_size": BS, "cpu_core_us_per_block": round(cpu_blk * 1e6, 2),
                      "hash_bytes_us_per_call": round(single_blk * 1e6, 1),
                      "crossover_blocks": cross, "rows": rows}))


if __name__ == "__main__":
    main()
