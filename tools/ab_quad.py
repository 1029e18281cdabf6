"""In-process A/B of whole libciruela_amd builds on the quad-mode workloads.

Usage: python tools/ab_quad.py LIB.so [LIB.so ...]
Workloads (all device-resident, HIP events on one stream, interleaved rounds):
  cfg3   config 3 (10 GiB mixed 4K/32K/1M, ragged, shuffled) through
         cir_hash_blocks_dev with a context (order + quad + lane parts);
  1m     32768 x 1 MiB through cir_hash_chunks_dev (k_quad_chunks);
  4m     8192 x 4 MiB through cir_hash_chunks_dev (k_quad_chunks);
  d32k   8192 x 32 KiB descriptors (one 256 MiB staging batch) through
         cir_hash_blocks_dev (k_quad_long, small-batch policy);
  d1m    16384 x 1 MiB descriptors, same path;
  one    a single 16 MiB chain (one descriptor: the index-footer shape).
AB_LANE=1: cfg3 plus lane-part batches -- dl32k 1 M x 32 KiB and dl4k 8 M x
4 KiB descriptors, c3short config 3's 4 KiB / 32 KiB classes alone.
Checks that every library produces the same digests.
"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402  (config3_layout)

GIB = 1 << 30


def load(path):
    lib = ctypes.CDLL(path)
    vp, u64 = ctypes.c_void_p, ctypes.c_uint64
    lib.cir_init.argtypes = [ctypes.POINTER(vp), ctypes.c_uint32, u64]
    lib.cir_hash_chunks_dev.argtypes = [vp, vp, u64, u64, vp, vp]
    lib.cir_hash_blocks_dev.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, vp, vp]
    lib.cir_fill_splitmix64_dev.argtypes = [vp, u64, u64, u64, u64, vp]
    ctx = vp()
    assert lib.cir_init(ctypes.byref(ctx), 1, 1 << 20) == 0
    return lib, ctx


def main():
    paths = sys.argv[1:]
    libs = [load(p) for p in paths]
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    offs, lens, nbytes = bench.config3_layout()
    data = torch.empty(max(nbytes, 32 * GIB), dtype=torch.uint8, device="cuda:0")
    assert libs[0][0].cir_fill_splitmix64_dev(data.data_ptr(), data.numel(), 0x5EED0003, 0, 0,
                                              0) == 0
    d_off = torch.from_numpy(offs).cuda()
    d_len = torch.from_numpy(lens).cuda()
    n3 = lens.size
    hashed3 = int(lens.astype("int64").sum())
    work = {
        "cfg3": (n3, hashed3, lambda lib, ctx, out: lib.cir_hash_blocks_dev(
            ctx, data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n3, out.data_ptr(),
            s.cuda_stream)),
        "1m": (32768, 32 * GIB, lambda lib, ctx, out: lib.cir_hash_chunks_dev(
            ctx, data.data_ptr(), 32 * GIB, 1 << 20, out.data_ptr(), s.cuda_stream)),
        "4m": (8192, 32 * GIB, lambda lib, ctx, out: lib.cir_hash_chunks_dev(
            ctx, data.data_ptr(), 32 * GIB, 4 << 20, out.data_ptr(), s.cuda_stream)),
    }
    def desc(nblk, bs):
        o = torch.arange(nblk, dtype=torch.int64, device="cuda:0") * bs
        ln = torch.full((nblk,), bs, dtype=torch.int32, device="cuda:0")
        keep.append((o, ln))
        return (nblk, nblk * bs, lambda lib, ctx, out: lib.cir_hash_blocks_dev(
            ctx, data.data_ptr(), o.data_ptr(), ln.data_ptr(), nblk, out.data_ptr(),
            s.cuda_stream))
    keep = []
    if os.environ.get("AB_LANE"):  # lane-part workloads (descriptor batches without quad chains)
        for name in ("1m", "4m"):
            del work[name]
        work["dl32k"] = desc(1 << 20, 32768)
        work["dl4k"] = desc(8 << 20, 4096)
        # the config-3 short classes alone, shuffled and ragged (lane part only)
        short = lens < (1 << 20)
        o3, l3 = torch.from_numpy(offs[short]).cuda(), torch.from_numpy(lens[short]).cuda()
        keep.append((o3, l3))
        ns = int(short.sum())
        work["c3short"] = (ns, int(lens[short].astype("int64").sum()),
                           lambda lib, ctx, out: lib.cir_hash_blocks_dev(
                               ctx, data.data_ptr(), o3.data_ptr(), l3.data_ptr(), ns,
                               out.data_ptr(), s.cuda_stream))
    elif os.environ.get("AB_FIT"):  # fixed cost vs per-line cost of the small-batch quad path
        work.clear()
        for lines in (8, 32, 128, 512, 2048):
            work["d%dL" % lines] = desc(8192, 128 * lines)
    else:
        work["d32k"] = desc(8192, 32768)
        work["d1m"] = desc(16384, 1 << 20)
        work["one"] = desc(1, 16 << 20)
    if os.environ.get("AB_ONLY"):  # comma-separated workload names
        keep_names = os.environ["AB_ONLY"].split(",")
        work = {k: v for k, v in work.items() if k in keep_names}
    torch.cuda.synchronize()
    for name, (nblk, nb, call) in work.items():
        outs = [torch.empty(32 * nblk, dtype=torch.uint8, device="cuda:0") for _ in libs]
        times = [[] for _ in libs]
        for rnd in range(int(os.environ.get("AB_ROUNDS", "5"))):
            for k, (lib, ctx) in enumerate(libs):
                for rep in range(3):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    assert call(lib, ctx, outs[k]) == 0
                    e1.record(s)
                    e1.synchronize()
                    if rnd > 0:
                        times[k].append(e0.elapsed_time(e1))
        for k, p in enumerate(paths):
            t = statistics.median(times[k])
            print("%-5s %-36s median %8.3f ms  min %8.3f  GiB/s %7.1f  same=%s" % (
                name, p, t, min(times[k]), nb / GIB / (t / 1e3), torch.equal(outs[k], outs[0])),
                flush=True)


if __name__ == "__main__":
    main()
