"""Where config 5's time outside the hash loop goes: one tree (bench.py's
make_tree, --tree-gib), scanned through
  * the Python wrapper (ca.v1.scan: cir_scan_v1, then the index copied into
    a bytes object and the library buffer freed),
  * the raw cir_scan_v1 call alone (the index freed uncopied),
with the scan's own phase record beside each (walk, hash loop, footer tail).

    python tools/scan_output_probe.py [--tree-gib 16] [--runs 3]
"""
import argparse
import ctypes
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tree-gib", type=float, default=16)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--tree-dir", default="/dev/shm/ciruela_probe_tree")
    args = ap.parse_args()
    import bench
    import ciruela_amd as ca
    n_ = ca._n
    try:
        nfiles = bench.make_tree(args.tree_dir, args.tree_gib)
        nbytes = nfiles * (32 << 20)
        bench.tree_read_pass(args.tree_dir)
        ctx = ca.Context()
        cfg = ca.ScannerConfig.new().add_dir(args.tree_dir, "/")
        ctx.scan_timing(True)
        ref = ca.v1.scan(cfg, context=ctx)
        dirs = (ctypes.c_char_p * 1)(os.fsencode(args.tree_dir))
        pres = (ctypes.c_char_p * 1)(b"/")
        for r in range(args.runs):
            t0 = time.perf_counter()
            got = ca.v1.scan(cfg, context=ctx)
            t1 = time.perf_counter()
            ph = ctx.scan_phases()
            assert got == ref
            del got
            out = ctypes.c_void_p()
            ln = ctypes.c_size_t()
            t2 = time.perf_counter()
            n_.check(n_.lib.cir_scan_v1(ctx.handle, dirs, pres, 1, cfg._block_size,
                                        cfg._hash.code, cfg._threads, ctypes.byref(out),
                                        ctypes.byref(ln)))
            t3 = time.perf_counter()
            ph2 = ctx.scan_phases()
            t4 = time.perf_counter()
            n_.lib.cir_free(out.value)
            t5 = time.perf_counter()
            inside = ph["walk_ms"] + ph["hash_loop_ms"] + ph["footer_tail_ms"] + ph["output_ms"]
            inside2 = ph2["walk_ms"] + ph2["hash_loop_ms"] + ph2["footer_tail_ms"] + ph2["output_ms"]
            print("wrapper %.1f ms (%.2f GiB/s; phases %.1f: walk %.1f loop %.1f tail %.2f) | "
                  "raw call %.1f ms (%.2f GiB/s; phases %.1f) + cir_free %.1f ms | index %.1f MB"
                  % ((t1 - t0) * 1e3, nbytes / (t1 - t0) / 2**30, inside, ph["walk_ms"],
                     ph["hash_loop_ms"], ph["footer_tail_ms"], (t3 - t2) * 1e3,
                     nbytes / (t3 - t2) / 2**30, inside2, (t5 - t4) * 1e3, ln.value / 1e6),
                  flush=True)
        t0 = time.perf_counter()
        for _ in range(3):
            b = ctypes.string_at(ctypes.addressof(ctypes.create_string_buffer(1)), 1)
        buf = ctypes.create_string_buffer(len(ref))
        t0 = time.perf_counter()
        b = ctypes.string_at(buf, len(ref))
        t1 = time.perf_counter()
        print("string_at of %.1f MB: %.1f ms" % (len(ref) / 1e6, (t1 - t0) * 1e3))
    finally:
        shutil.rmtree(args.tree_dir, ignore_errors=True)


if __name__ == "__main__":
    main()
