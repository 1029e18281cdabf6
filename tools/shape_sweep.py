"""Shape sweep of cir_hash_chunks_dev (one device-resident file, context
path): GiB/s per (block size, block count), one process, HIP events on the
launch stream; a checksum column per shape compares the digests between
runs of two builds (the relay's A/B in round 2 used an environment switch
that no longer exists: build the variant instead, tools/build_variant.sh).  SWEEP_DESC=1: the same blocks as a descriptor batch
(cir_hash_blocks_dev).  Diagnostics only (DESIGN.md §5 shapes)."""
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ciruela_amd as ca  # noqa: E402

SHAPES = [(32768, n) for n in (16384, 16385, 20480, 24576, 32768, 32769, 33792, 36864, 40960,
                               49152, 49153, 50176, 53248, 53249, 57344, 65535, 65536, 65537, 66560,
                               73728, 81920, 90112, 98304, 106496, 106497, 114688, 122880, 131072, 131073,
                               147456, 163840, 180224, 196608, 196609, 212992, 229376,
                               262144, 262145, 278528, 524288, 524289, 557056, 1048576,
                               1048577, 1064960)] + \
         [(262144, n) for n in (65536, 65537, 73728, 81920, 98304)] + \
         [(4096, n) for n in (65536, 65537, 66560, 69632, 73728, 81920, 98304, 131072,
                              131073, 139264)] + \
         [(16384, n) for n in (65536, 65537, 73728, 98304)] + \
         [(262144, n) for n in (32768, 32769, 49152, 49153)] + \
         [(4096, n) for n in (16384, 16385, 32768, 32769)] + \
         [(1048576, n) for n in (32768, 32769, 49152, 49153)] + \
         [(131072, 262144), (4096, 8388608), (4194304, 8192)]


def main():
    global SHAPES
    if os.environ.get("SWEEP_ONLY"):  # "bs:n,bs:n,..."
        SHAPES = [tuple(int(x) for x in t.split(":")) for t in os.environ["SWEEP_ONLY"].split(",")]
    steps = int(os.environ.get("SWEEP_STEPS", "10"))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    ctx = ca.Context(device_mask=1)
    stream = torch.cuda.current_stream().cuda_stream
    maxb = max(bs * n for bs, n in SHAPES)
    data = torch.empty(maxb, dtype=torch.uint8, device=dev)
    ca._n.check(ca._n.lib.cir_fill_splitmix64_dev(data.data_ptr(), maxb, 0x5EED, 0, 0, stream))
    out = torch.empty(max(n for _, n in SHAPES) * 32, dtype=torch.uint8, device=dev)
    relay = "1"
    desc = os.environ.get("SWEEP_DESC") == "1"  # the same blocks as descriptors
    for bs, n in SHAPES:
        nbytes = bs * n
        if desc:
            d_off = torch.arange(n, dtype=torch.int64, device=dev) * bs
            d_len = torch.full((n,), bs, dtype=torch.int32, device=dev)

            def call():
                ctx.hash_blocks_dev(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                                    out.data_ptr(), stream)
        else:
            def call():
                ctx.hash_chunks_dev(data.data_ptr(), nbytes, bs, out.data_ptr(), stream)
        for _ in range(2):
            call()
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(steps)]
        for a, b in evs:
            a.record()
            call()
            b.record()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in evs)
        med = ms[len(ms) // 2]
        csum = hashlib.sha256(out[:n * 32].cpu().numpy().tobytes()).hexdigest()[:12]
        rel = ca._n.lib.cir_debug_relay_blocks(n, bs)
        print("relay=%s bs=%d nblk=%d relayed=%d ms=%.4f min=%.4f GiB/s=%.1f digests=%s"
              % (relay, bs, n, rel, med, ms[0], nbytes / 2**30 / (med / 1e3), csum), flush=True)


if __name__ == "__main__":
    main()
