import os, sys
sys.path.insert(0, os.getcwd())
import torch
import ciruela_amd as ca
import bench
ctx = ca.Context(device_mask=1)
s = torch.cuda.current_stream().cuda_stream
offs, lens, nbytes = bench.config3_layout()
import numpy as np
keep = lens < (1 << 17)   # lane-mode chains only
o = torch.from_numpy(offs[keep]).cuda(); l = torch.from_numpy(lens[keep]).cuda()
n = int(keep.sum())
data = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda:0")
ca._n.check(ca._n.lib.cir_fill_splitmix64_dev(data.data_ptr(), data.numel() // 8 * 8, 9, 0, 0, s))
out = torch.empty(n * 32, dtype=torch.uint8, device="cuda:0")
for i in range(6):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    ctx.hash_blocks_dev(data.data_ptr(), o.data_ptr(), l.data_ptr(), n, out.data_ptr(), s)
    b.record(); b.synchronize()
    print("lane-only n=%d %.3f ms" % (n, a.elapsed_time(b)), flush=True)
