"""H2D bandwidth probe: pinned host -> HBM copies of 256 MiB, alone, split
over two streams, and while 16 host threads memcpy (the scan readers' load)."""
import os
import threading
import time

import numpy as np
import torch

N = 256 << 20
torch.cuda.set_device(0)
h = torch.empty(N, dtype=torch.uint8).pin_memory()
d = torch.empty(N, dtype=torch.uint8, device="cuda:0")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return N * reps / (time.perf_counter() - t0) / 1e9


def one():
    with torch.cuda.stream(s1):
        d.copy_(h, non_blocking=True)


def two():
    with torch.cuda.stream(s1):
        d[:N // 2].copy_(h[:N // 2], non_blocking=True)
    with torch.cuda.stream(s2):
        d[N // 2:].copy_(h[N // 2:], non_blocking=True)


stop = False


def hog():
    a = np.ones(64 << 20, dtype=np.uint8)
    b = np.empty_like(a)
    while not stop:
        np.copyto(b, a)


print("SDMA env:", os.environ.get("HSA_ENABLE_SDMA"))
timed(one, 2)
print("1 stream  : %.1f GB/s" % timed(one))
print("2 streams : %.1f GB/s" % timed(two))
ths = [threading.Thread(target=hog) for _ in range(16)]
for t in ths:
    t.start()
time.sleep(0.2)
print("1 stream  + 16 memcpy threads: %.1f GB/s" % timed(one))
print("2 streams + 16 memcpy threads: %.1f GB/s" % timed(two))
stop = True
for t in ths:
    t.join()
