"""Probe 2: first-time hipHostRegister of fresh tmpfs files, 1/4/8/16 threads
in parallel, and H2D from registered files while other files register."""
import ctypes
import mmap
import os
import threading
import time

import numpy as np
import torch

torch.cuda.set_device(0)
hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                               ctypes.c_void_p]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
RO = 0x08
FSZ = 32 << 20
NF = 128  # 4 GiB of files
root = "/dev/shm/hostreg2"
os.makedirs(root, exist_ok=True)
blob = os.urandom(FSZ)
for i in range(NF):
    with open("%s/f%03d" % (root, i), "wb") as f:
        f.write(blob)


def mapf(i):
    fd = os.open("%s/f%03d" % (root, i), os.O_RDONLY)
    mm = mmap.mmap(fd, FSZ, prot=mmap.PROT_READ, flags=mmap.MAP_SHARED)
    os.close(fd)
    return mm, np.frombuffer(mm, dtype=np.uint8).ctypes.data


maps = [mapf(i) for i in range(NF)]
d = torch.empty(FSZ, dtype=torch.uint8, device="cuda:0")
s = torch.cuda.Stream()
sp = ctypes.c_void_p(s.cuda_stream)


def register_range(idx, out):
    for i in idx:
        rc = hip.hipHostRegister(maps[i][1], FSZ, RO)
        out.append(rc)


start = 0
for nth in (1, 4, 8, 16):
    idx = list(range(start, start + 16 * nth // nth * 2))  # 32 files per setting
    idx = list(range(start, start + 32))
    start += 32
    rcs = []
    chunks = [idx[k::nth] for k in range(nth)]
    ths = [threading.Thread(target=register_range, args=(c, rcs)) for c in chunks]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    assert all(r == 0 for r in rcs), rcs
    print("register %2d threads: %.1f GB/s (32 x 32 MiB fresh files)" % (nth, 32 * FSZ / 1e9 / dt),
          flush=True)

# H2D from registered files (the last 64 registered) alone
t0 = time.perf_counter()
for i in range(64, 128):
    hip.hipMemcpyAsync(d.data_ptr(), maps[i][1], FSZ, 1, sp)
hip.hipStreamSynchronize(sp)
print("h2d from registered files: %.1f GB/s" % (64 * FSZ / 1e9 / (time.perf_counter() - t0)))
for i in range(NF):
    hip.hipHostUnregister(maps[i][1])
print("unregistered", flush=True)
for mm, _ in maps:
    pass
import shutil
shutil.rmtree(root)
