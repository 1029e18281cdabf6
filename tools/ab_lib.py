"""In-process A/B of whole libciruela_amd builds on the config-2 workload.

Usage: python tools/ab_lib.py LIB.so [LIB.so ...]
Fills 1 M x 32 KiB once, then times cir_hash_chunks_dev of each library in
interleaved rounds (same box, same thermal state), HIP events on one stream.
Checks that every library produces the same digest array.
"""
import ctypes
import statistics
import sys

import torch

BS, NBLK = 32768, 1 << 20


def load(path):
    lib = ctypes.CDLL(path)
    vp, u64 = ctypes.c_void_p, ctypes.c_uint64
    lib.cir_init.argtypes = [ctypes.POINTER(vp), ctypes.c_uint32, u64]
    lib.cir_hash_chunks_dev.argtypes = [vp, vp, u64, u64, vp, vp]
    lib.cir_fill_splitmix64_dev.argtypes = [vp, u64, u64, u64, u64, vp]
    ctx = vp()
    assert lib.cir_init(ctypes.byref(ctx), 1, 1 << 20) == 0
    return lib, ctx


def main():
    paths = sys.argv[1:]
    libs = [load(p) for p in paths]
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    data = torch.empty(NBLK * BS, dtype=torch.uint8, device="cuda:0")
    assert libs[0][0].cir_fill_splitmix64_dev(data.data_ptr(), NBLK * BS, 0x5EED0002, 0, 0, 0) == 0
    outs = [torch.empty(NBLK * 32, dtype=torch.uint8, device="cuda:0") for _ in libs]
    torch.cuda.synchronize()
    times = [[] for _ in libs]
    for rnd in range(8):
        for k, (lib, ctx) in enumerate(libs):
            for rep in range(4):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                rc = lib.cir_hash_chunks_dev(ctx, data.data_ptr(), NBLK * BS, BS,
                                             outs[k].data_ptr(), s.cuda_stream)
                e1.record(s)
                assert rc == 0
                e1.synchronize()
                if rnd > 0:
                    times[k].append(e0.elapsed_time(e1))
        print("round", rnd, flush=True)
    for k, p in enumerate(paths):
        t = times[k]
        print("%-40s median %.3f ms  min %.3f  max %.3f  GiB/s %.1f  same=%s" % (
            p, statistics.median(t), min(t), max(t), 32 / (statistics.median(t) / 1e3),
            torch.equal(outs[k], outs[0])))


if __name__ == "__main__":
    main()
