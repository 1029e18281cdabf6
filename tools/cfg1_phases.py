"""Where config 1's in-process scan (100 files / 10 MiB, threads 4) spends its
time: cir_debug_scan_timing's phases and batch rows over repeated scans.

    python tools/cfg1_phases.py [--scans 20] [--threads 4]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=20)
    ap.add_argument("--threads", type=int, default=4)
    a = ap.parse_args()
    import bench
    import ciruela_amd as ca
    root = "/tmp/ciruela_cfg1_phases"
    bench.make_config1_tree(root)
    ctx = ca.Context(device_mask=1)
    cfg = ca.ScannerConfig.new().threads(a.threads).add_dir(root, "/")
    for _ in range(3):
        ca.v1.scan(cfg, context=ctx)
    walls = []
    for i in range(a.scans):
        ctx.scan_timing(True)
        t0 = time.perf_counter()
        ca.v1.scan(cfg, context=ctx)
        walls.append((time.perf_counter() - t0) * 1e3)
        ph = ctx.scan_phases()
        rows = ctx.scan_batches()
        ctx.scan_timing(False)
        if i < 3 or i == a.scans - 1:
            print("scan %d: %.3f ms | walk %.3f loop %.3f last_emit %.3f footer_tail %.3f output %.3f"
                  % (i, walls[-1], ph["walk_ms"], ph["hash_loop_ms"], ph["last_emit_ms"],
                     ph["footer_tail_ms"], ph["output_ms"]))
            for r in rows:
                print("   batch %.2f MiB %d blk: wait %.3f read %.3f-%.3f h2d %.3f-%.3f hash %.3f done %.3f"
                      % (r["bytes"] / 2**20, r["blocks"], r["wait_ms"], r["read_start_ms"],
                         r["read_end_ms"], r["h2d_start_ms"], r["h2d_end_ms"], r["hash_start_ms"],
                         r["done_ms"]))
    walls.sort()
    print("median %.3f ms, best %.3f ms" % (walls[len(walls) // 2], walls[0]))


if __name__ == "__main__":
    main()
