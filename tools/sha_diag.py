"""Diagnostic: GPU SHA-512/256 vs hashlib over lengths 0..400 (deterministic data)."""
import hashlib, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ciruela_amd as ca

data = bytes((i * 7 + 3) & 0xff for i in range(2048))
res = {}
bad = []
for n in range(0, 401):
    g = ca.sha512_256(data[:n])
    res[n] = g.hex()
    if g != hashlib.new("sha512_256", data[:n]).digest():
        bad.append(n)
print("bad", len(bad), bad[:40])
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/sha_diag.json", "w"))
