"""Does POSIX_FADV_NOREUSE take the cost out of the first read of a freshly
written tmpfs tree?  (round 5; the cold config-5 scan)

Writes a config-5-shaped tree (bench.make_tree) and reads it twice with
`threads` pread() threads, the files opened plainly or with
posix_fadvise(POSIX_FADV_NOREUSE) (Linux >= 6.3: reads of such a file do
not mark its pages accessed, i.e. do not move them between LRU lists);
the tree is rewritten before each mode so every first read meets fresh
pages.  CPU only.

    python tools/noreuse_probe.py [--gib 16] [--threads 16] [--rounds 2]
"""
import argparse
import os
import shutil
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def read_pass(paths, threads, noreuse, piece=4 << 20):
    bufs = [bytearray(piece) for _ in range(threads)]

    def work(k):
        mv, n = memoryview(bufs[k]), 0
        for p in paths[k::threads]:
            fd = os.open(p, os.O_RDONLY)
            try:
                if noreuse:
                    os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_NOREUSE)
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
    return total / 2**30 / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=16.0)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--dir", default="/dev/shm/cir_noreuse_probe")
    a = ap.parse_args()
    import bench
    print("kernel %s" % os.uname().release, flush=True)
    try:
        for rnd in range(a.rounds):
            for noreuse in (False, True):
                shutil.rmtree(a.dir, ignore_errors=True)
                bench.make_tree(a.dir, a.gib)
                paths = sorted(os.path.join(dp, f) for dp, _, fs in os.walk(a.dir) for f in fs
                               if f.endswith(".bin"))
                first = read_pass(paths, a.threads, noreuse)
                second = read_pass(paths, a.threads, noreuse)
                print("round %d %-8s %d threads: first read %.1f GiB/s, second %.1f GiB/s"
                      % (rnd, "noreuse" if noreuse else "plain", a.threads, first, second),
                      flush=True)
    finally:
        shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
