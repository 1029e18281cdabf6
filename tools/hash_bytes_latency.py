"""Latency of BlockHash::hash_bytes (cir_blake2b256, host buffer in, digest
out) per call through the one-launch path (k_single), checked against
hashlib.  (Round 2 also timed the staged batch path here: 77-88 / 119-128 /
401-421 us at 0 B / 4 KiB / 32 KiB, profiles/r02_final/latency.log.)

    python tools/hash_bytes_latency.py [--calls 100]
"""
import argparse
import hashlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=100)
    args = ap.parse_args()
    import ciruela_amd as ca
    for mode in ("single",):
        for n in (0, 100, 4096, 32768, 1 << 20):
            data = os.urandom(n)
            want = hashlib.blake2b(data, digest_size=32).digest()
            for _ in range(5):
                got = bytes(ca.BlockHash.hash_bytes(data))
            assert got == want, (mode, n)
            calls = args.calls if n <= 32768 else max(5, args.calls // 10)
            ts = []
            for _ in range(calls):
                t0 = time.perf_counter()
                ca.BlockHash.hash_bytes(data)
                ts.append(time.perf_counter() - t0)
            ts.sort()
            print("hash_bytes %-6s n=%-8d median %8.1f us  min %8.1f us  mean %8.1f us (%d calls)"
                  % (mode, n, ts[len(ts) // 2] * 1e6, ts[0] * 1e6, sum(ts) / len(ts) * 1e6,
                     calls), flush=True)


if __name__ == "__main__":
    main()
