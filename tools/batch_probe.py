"""Time cir_hash_blocks_dev (ordered, k_mixed) on batches of n x 32 KiB
descriptors: how long a scan batch's hash takes when it underfills the GPU."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ciruela_amd as ca

BS = 32768
ctx = ca.Context(device_mask=1)
s = torch.cuda.current_stream().cuda_stream
for n in (2048, 8192, 32768, 131072, 1 << 20):
    data = torch.empty(n * BS, dtype=torch.uint8, device="cuda:0")
    ca._n.check(ca._n.lib.cir_fill_splitmix64_dev(data.data_ptr(), n * BS, 5, 0, 0, s))
    off = torch.arange(n, dtype=torch.int64, device="cuda:0") * BS
    ln = torch.full((n,), BS, dtype=torch.int32, device="cuda:0")
    out = torch.empty(n * 32, dtype=torch.uint8, device="cuda:0")
    ts = []
    for i in range(6):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ctx.hash_blocks_dev(data.data_ptr(), off.data_ptr(), ln.data_ptr(), n, out.data_ptr(), s)
        b.record()
        b.synchronize()
        if i:
            ts.append(a.elapsed_time(b))
    t = sorted(ts)[len(ts) // 2]
    print("n=%7d (%6.0f MiB): %.3f ms  %.1f GB/s" % (n, n * BS / 2**20, t, n * BS / t / 1e6),
          flush=True)
    del data, off, ln, out
