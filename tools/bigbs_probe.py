import os, random, sys
sys.path.insert(0, "/root/repo")
import ciruela_amd as gpu
c = gpu.Context(device_mask=1, staging_bytes=1 << 20)
rng = random.Random(91)
bs = (3 << 20) + 5
root = "/tmp/bigbs_tree"
os.makedirs(root + "/d", exist_ok=True)
sizes = [0, 1, bs, bs + 1, 2 * bs + 100, (10 << 20) + 7]
for k, n in enumerate(sizes):
    open(root + "/d/f%d" % k, "wb").write(rng.randbytes(n))
for variant in (["f5"], ["f2"], ["f1", "f2"], None):
    sub = "/tmp/bigbs_sub"
    import shutil
    shutil.rmtree(sub, ignore_errors=True)
    os.makedirs(sub)
    for f in (variant or ["f%d" % k for k in range(6)]):
        os.link(root + "/d/" + f, sub + "/" + f)
    cfg = gpu.ScannerConfig.new().block_size(bs).threads(3).add_dir(sub, "/")
    try:
        gpu.v1.scan(cfg, context=c)
        print(variant, "ok", flush=True)
    except Exception as e:
        print(variant, "FAIL", e, flush=True)
