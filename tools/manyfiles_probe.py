"""A metadata-heavy tree (not a BASELINE config): 200,000 files of 0-4 KiB in
400 directories on tmpfs, scanned by v1.scan with 4 readers (the
reference's --disk-threads default) and with the library's own choice,
three times each, with the scan's phase record (walk, reads, hash, emit),
beside the CPU restatement of the reference indexer on 4 and 16 threads.
    python3 tools/manyfiles_probe.py   (on the GPU box)"""
import os
import shutil
import sys
import time

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
root = "/dev/shm/cir_many"
shutil.rmtree(root, ignore_errors=True)
n_dirs, per = 400, 500
t = time.time()
blob = os.urandom(4096)
total = 0
for d in range(n_dirs):
    p = os.path.join(root, "d%03d" % d)
    os.makedirs(p)
    for i in range(per):
        n = (i * 37) % 4097
        total += n
        with open(os.path.join(p, "f%04d" % i), "wb") as f:
            f.write(blob[:n])
print("made %d files, %d bytes, in %.1f s" % (n_dirs * per, total, time.time() - t), flush=True)
import ciruela_amd as ca  # noqa: E402
ctx = ca.Context(device_mask=1)
ctx.scan_timing(True)
idx = None
for threads in (4, 0):
    for rep in range(3):
        cfg = ca.ScannerConfig.new().block_size(32768).threads(threads).add_dir(root, "/")
        t = time.time()
        idx = ca.v1.scan(cfg, context=ctx)
        dt = time.time() - t
        ph = {k: round(v, 2) for k, v in ctx.scan_phases().items()}
        print("threads %d: scan %.3f s (%.0f files/s), index %d bytes; phases %s"
              % (threads, dt, n_dirs * per / dt, len(idx), ph), flush=True)
        for b in ctx.scan_batches():
            print("   batch %.1f MB %d blocks: wait %.1f, reads %.1f-%.1f, h2d %.1f-%.1f, "
                  "hash %.1f-%.1f ms" % (b["bytes"] / 1e6, b["blocks"], b["wait_ms"],
                                         b["read_start_ms"], b["read_end_ms"], b["h2d_start_ms"],
                                         b["h2d_end_ms"], b["hash_start_ms"], b["done_ms"]))
        ctx.scan_timing(True)  # (clears the rows)
import cpu_indexer  # noqa: E402  (the CPU baseline, oracle/)
for threads in (4, 16):
    t = time.time()
    ref = cpu_indexer.index(root, 32768, threads)
    dt = time.time() - t
    print("cpu indexer (Python walk, C hashing) %d threads: %.3f s, %s" % (
        threads, dt, "same index" if ref == idx else "DIFFERENT index"), flush=True)
shutil.rmtree(root, ignore_errors=True)
