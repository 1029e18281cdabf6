"""Device memory left after repeated cir_init / use / cir_destroy cycles in one
process (the lifecycle test in tests/test_gpu_parity.py): prints the free
device memory after every cycle and the per-cycle deltas."""
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import ciruela_amd as gpu
torch.cuda.synchronize()
data = np.frombuffer(os.urandom(1 << 20), dtype=np.uint8).tobytes()
def free():
    torch.cuda.synchronize(); return torch.cuda.mem_get_info()[0] >> 20
f = [free()]
for i in range(12):
    c = gpu.Context(device_mask=1, staging_bytes=64 << 20)
    if i % 2 == 0:
        gpu.Hashes.hash_file(gpu.HashType.blake2b_256(), 32768, data, context=c)
    c.close()
    f.append(free())
print("free MiB per cycle:", f)
print("deltas:", [f[i] - f[i+1] for i in range(len(f)-1)])
