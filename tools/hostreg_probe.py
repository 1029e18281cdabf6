"""Probe: DMA straight from page-cache pages of a tmpfs file.

mmap a 1 GiB /dev/shm file read-only, hipHostRegister(ReadOnly) 256 MiB
pieces, H2D them, unregister -- vs read() into a pinned buffer + H2D."""
import ctypes
import mmap
import os
import time

import torch

torch.cuda.set_device(0)
hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                               ctypes.c_void_p]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
H2D = 1
RO = 0x08  # hipHostRegisterReadOnly

PIECE = 256 << 20
TOTAL = 1 << 30
path = "/dev/shm/hostreg_probe.bin"
with open(path, "wb") as f:
    for _ in range(TOTAL // (64 << 20)):
        f.write(os.urandom(64 << 20))
fd = os.open(path, os.O_RDONLY)
mm = mmap.mmap(fd, TOTAL, prot=mmap.PROT_READ, flags=mmap.MAP_SHARED)
import numpy as np
arr = np.frombuffer(mm, dtype=np.uint8)
base = arr.ctypes.data
d = torch.empty(PIECE, dtype=torch.uint8, device="cuda:0")
s = torch.cuda.Stream()
sp = ctypes.c_void_p(s.cuda_stream)

for rep in range(3):
    t_reg = t_cp = t_unreg = 0.0
    for k in range(TOTAL // PIECE):
        p = base + k * PIECE
        t0 = time.perf_counter()
        rc = hip.hipHostRegister(p, PIECE, RO)
        t1 = time.perf_counter()
        assert rc == 0, "hipHostRegister rc=%d" % rc
        rc = hip.hipMemcpyAsync(d.data_ptr(), p, PIECE, H2D, sp)
        assert rc == 0
        hip.hipStreamSynchronize(sp)
        t2 = time.perf_counter()
        hip.hipHostUnregister(p)
        t3 = time.perf_counter()
        t_reg += t1 - t0
        t_cp += t2 - t1
        t_unreg += t3 - t2
    gb = TOTAL / 1e9
    print("register %.1f GB/s, h2d %.1f GB/s, unregister %.1f GB/s, serial total %.1f GB/s" % (
        gb / t_reg, gb / t_cp, gb / t_unreg, gb / (t_reg + t_cp + t_unreg)), flush=True)
    # check the bytes arrived
    assert torch.equal(d.cpu(), torch.from_numpy(arr[TOTAL - PIECE:].copy()))

# baseline: read() into pinned + H2D
h = torch.empty(PIECE, dtype=torch.uint8).pin_memory()
hv = memoryview(h.numpy())
t_rd = t_cp = 0.0
for k in range(TOTAL // PIECE):
    t0 = time.perf_counter()
    os.preadv(fd, [hv], k * PIECE)
    t1 = time.perf_counter()
    with torch.cuda.stream(s):
        d.copy_(h, non_blocking=True)
    s.synchronize()
    t2 = time.perf_counter()
    t_rd += t1 - t0
    t_cp += t2 - t1
print("pread 1 thread %.1f GB/s, pinned h2d %.1f GB/s" % (TOTAL / 1e9 / t_rd, TOTAL / 1e9 / t_cp))
os.close(fd)
os.unlink(path)
