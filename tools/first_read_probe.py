"""Where does config 5's first scan lose its time?  (round 3)

Generates a config-5-shaped tree (bench.make_tree) in /dev/shm, then:
  1. times N plain CPU read passes over every file (16 threads, pread into
     reused buffers, no GPU) -- does the FIRST read of a fresh tmpfs tree run
     slower than later ones, with no library involved at all?
  2. times cir_scan_v1 three times in a fresh context.
With --read-first 0 the scans run first (as in bench.py), then the reads.
"""
import argparse
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def read_pass(paths, threads=16, piece=4 << 20):
    bufs = [bytearray(piece) for _ in range(threads)]

    def work(k):
        mv = memoryview(bufs[k])
        n = 0
        for p in paths[k::threads]:
            fd = os.open(p, os.O_RDONLY)
            try:
                off = 0
                while True:
                    r = os.preadv(fd, [mv], off)
                    if r <= 0:
                        break
                    off += r
                    n += r
            finally:
                os.close(fd)
        return n
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        total = sum(ex.map(work, range(threads)))
    return total, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=16.0)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--read-first", type=int, default=1)
    ap.add_argument("--dir", default="/dev/shm/cir_first_read_probe")
    a = ap.parse_args()
    import bench
    t0 = time.perf_counter()
    bench.make_tree(a.dir, a.gib)
    print("tree %.1f GiB generated in %.1f s" % (a.gib, time.perf_counter() - t0), flush=True)
    paths = sorted(os.path.join(dp, f) for dp, _, fs in os.walk(a.dir) for f in fs
                   if f.endswith(".bin"))

    def reads():
        for i in range(a.passes):
            n, dt = read_pass(paths)
            print("cpu read pass %d: %.2f GiB in %.3f s = %.1f GiB/s"
                  % (i, n / 2**30, dt, n / 2**30 / dt), flush=True)

    def scans():
        import ciruela_amd as ca
        t0 = time.perf_counter()
        ctx = ca.Context(device_mask=1)
        print("cir_init %.3f s" % (time.perf_counter() - t0), flush=True)
        cfg = ca.ScannerConfig.new().threads(16).add_dir(a.dir, "/")
        for i in range(3):
            t0 = time.perf_counter()
            ca.v1.scan(cfg, context=ctx)
            dt = time.perf_counter() - t0
            print("scan %d: %.3f s = %.1f GiB/s" % (i, dt, a.gib / dt), flush=True)
    try:
        if a.read_first:
            reads()
            scans()
        else:
            scans()
            reads()
    finally:
        import shutil
        shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
