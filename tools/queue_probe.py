"""Config 3 with one context vs several contexts in one process.

Each context's device state creates its own streams (compute, copy, and on
its first ordered batch the quad-part / lane-part streams).  With
GPU_MAX_HW_QUEUES = 4 (HIP's default) ordinary streams of a process share
hardware queues, and when the quad and lane parts of a mixed batch landed on
one queue they ran one after the other (r01: 570-610 GiB/s instead of ~850).
CIR_PART_STREAMS = hiq (default: quad part on a high-priority stream, a
queue pool of its own) / own2 (both parts on CU-masked streams) / plain
(round 1).

    python tools/queue_probe.py --contexts 4 [--steps 10]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--contexts", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import torch
    import bench
    import ciruela_amd as ca
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.cuda.current_stream().cuda_stream
    # every context runs one small ordered batch first, so all their streams exist
    ctxs = [ca.Context(device_mask=1) for _ in range(args.contexts)]
    one = torch.zeros(4096, dtype=torch.uint8, device=dev)
    off = torch.zeros(1, dtype=torch.int64, device=dev)
    ln = torch.full((1,), 4096, dtype=torch.int32, device=dev)
    o1 = torch.empty(32, dtype=torch.uint8, device=dev)
    for c in ctxs:
        c.hash_blocks_dev(one.data_ptr(), off.data_ptr(), ln.data_ptr(), 1, o1.data_ptr(), s)
    torch.cuda.synchronize()
    offs, lens, nbytes = bench.config3_layout()
    data = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    ca._n.check(ca._n.lib.cir_fill_splitmix64_dev(data.data_ptr(), nbytes, 0x5EED0003, 0, 0, s))
    d_off = torch.from_numpy(offs).to(dev)
    d_len = torch.from_numpy(lens).to(dev)
    n = lens.size
    out = torch.empty(32 * n, dtype=torch.uint8, device=dev)
    ctx = ctxs[-1]

    def step():
        ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                            out.data_ptr(), s)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    hashed = int(lens.astype("int64").sum())
    print("config3 contexts=%d part_streams=%s: %.3f ms  %.1f GiB/s" % (
        args.contexts, os.environ.get("CIR_PART_STREAMS", "hiq"), dt * 1e3,
        hashed / dt / (1 << 30)), flush=True)


if __name__ == "__main__":
    main()
