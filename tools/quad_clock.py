"""Quad-part clock probe (diagnostics): runs config 3 and its 1 MiB chains
alone through a CIR_QUAD_CLOCK build (tools/build_variant.sh qclk
-DCIR_QUAD_CLOCK=1) and prints each workload's step time, the quad waves'
mean duration and their in-kernel shader clock (s_memtime / s_memrealtime).

Usage: python tools/quad_clock.py abtest/qclk.so
"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

GIB = 1 << 30


def main():
    lib = ctypes.CDLL(sys.argv[1])
    vp, u64 = ctypes.c_void_p, ctypes.c_uint64
    lib.cir_init.argtypes = [ctypes.POINTER(vp), ctypes.c_uint32, u64]
    lib.cir_hash_blocks_dev.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, vp, vp]
    lib.cir_fill_splitmix64_dev.argtypes = [vp, u64, u64, u64, u64, vp]
    ctx = vp()
    assert lib.cir_init(ctypes.byref(ctx), 1, 1 << 20) == 0
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    offs, lens, nbytes = bench.config3_layout()
    data = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    assert lib.cir_fill_splitmix64_dev(data.data_ptr(), data.numel(), 0x5EED0003, 0, 0, 0) == 0
    d_off = torch.from_numpy(offs).cuda()
    d_len = torch.from_numpy(lens).cuda()
    big = torch.nonzero(d_len >= (1 << 20)).flatten()
    work = {"cfg3": (d_off, d_len), "cfg3_1m_only": (d_off[big].contiguous(), d_len[big].contiguous())}
    clk = (ctypes.c_ulonglong * 4)()
    for name, (o, ln) in work.items():
        n = ln.numel()
        out = torch.empty(32 * n, dtype=torch.uint8, device="cuda:0")
        ts, ghz, wave_ms, max_ms = [], [], [], []
        for rep in range(12):
            torch.cuda.synchronize()
            lib.cir_debug_quad_clock(clk)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
            assert lib.cir_hash_blocks_dev(ctx, data.data_ptr(), o.data_ptr(), ln.data_ptr(), n,
                                           out.data_ptr(), s.cuda_stream) == 0
            e1.record(s)
            e1.synchronize()
            assert lib.cir_debug_quad_clock(clk) == 0
            if rep < 2 or clk[2] == 0:
                continue
            ts.append(e0.elapsed_time(e1))
            ghz.append(clk[0] / clk[1] * 0.1)
            wave_ms.append(clk[1] / clk[2] * 1e-5)
            max_ms.append(clk[3] * 1e-5)
        nw = (n + 15) // 16
        ticks = (ctypes.c_uint * nw)()
        if hasattr(lib, "cir_debug_quad_wave_ticks") and name.endswith("only"):
            lib.cir_debug_quad_wave_ticks(ticks, nw)
            by = {}
            for w in range(nw - 1):  # the last wave may be partial
                by.setdefault(("xcd", (w // 4) % 8), []).append(ticks[w] * 1e-5)
                by.setdefault(("simd", w % 4), []).append(ticks[w] * 1e-5)
            for k in sorted(by):
                v = by[k]
                print("   %s %d: waves %3d mean %.3f max %.3f min %.3f ms" % (
                    k[0], k[1], len(v), sum(v) / len(v), max(v), min(v)))
        print("%-13s n=%7d step %.3f ms  quad wave mean %.3f ms max %.3f ms  quad clock %.3f GHz" % (
            name, n, statistics.median(ts), statistics.median(wave_ms), statistics.median(max_ms),
            statistics.median(ghz)), flush=True)


if __name__ == "__main__":
    main()
