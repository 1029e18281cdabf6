"""Quad-mode probe: time cir_hash_blocks_dev on batches of long chains only
(1 MiB blocks: quad mode), on config 3's short blocks only (lane mode), and
on both together, to separate a chain's latency from the interference of the
lane-mode waves that share its SIMDs.  Diagnostics, not part of the product."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ciruela_amd as ca  # noqa: E402

ctx = ca.Context(device_mask=1)
s = torch.cuda.current_stream().cuda_stream


def timed(lens):
    n = len(lens)
    ln = torch.tensor(lens, dtype=torch.int64)
    off = torch.zeros(n, dtype=torch.int64)
    off[1:] = torch.cumsum((ln + 15) // 16 * 16, 0)[:-1]
    total = int(off[-1] + ln[-1])
    data = torch.empty(total + 16, dtype=torch.uint8, device="cuda:0")
    ca._n.check(ca._n.lib.cir_fill_splitmix64_dev(data.data_ptr(), data.numel() // 8 * 8, 9, 0, 0, s))
    doff = off.to("cuda:0")
    dlen = ln.to(torch.int32).to("cuda:0")
    out = torch.empty(n * 32, dtype=torch.uint8, device="cuda:0")
    ts = []
    for i in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ctx.hash_blocks_dev(data.data_ptr(), doff.data_ptr(), dlen.data_ptr(), n, out.data_ptr(), s)
        b.record()
        b.synchronize()
        if i:
            ts.append(a.elapsed_time(b))
    t = sorted(ts)[len(ts) // 2]
    return t, int(ln.sum())


MIB = 1 << 20
for n in (1, 16, 64, 1024, 3413):
    t, nb = timed([MIB] * n)
    print("quad only: %5d x 1 MiB  %.3f ms  %.3f us per compression  %.1f GiB/s" % (
        n, t, t * 1e3 / 8192, nb / t / 1e6 / 1.073741824), flush=True)
short = [4096] * 873813 + [32768] * 109227
t, nb = timed(short)
print("lane only: config-3 4 KiB + 32 KiB blocks  %.3f ms  %.1f GiB/s" % (t, nb / t / 1e6 / 1.073741824),
      flush=True)
t, nb = timed(short + [MIB] * 3413)
print("both:      config-3 shapes (no ragged, unshuffled)  %.3f ms  %.1f GiB/s" % (
    t, nb / t / 1e6 / 1.073741824), flush=True)
