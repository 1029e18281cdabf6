"""Latency of BlockHash::hash_bytes (cir_blake2b256, host buffer in, digest
out) per call, the one-launch path (k_single) against the staged batch path
(CIR_SINGLE_STAGED=1), each checked against hashlib.

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
    for mode in ("single", "staged"):
        if mode == "staged":
            os.environ["CIR_SINGLE_STAGED"] = "1"
        else:
            os.environ.pop("CIR_SINGLE_STAGED", None)
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
