#!/usr/bin/env python3
"""Device-resident BLAKE2b-256 block hashing on MI355X (BASELINE.json metric).

One step = one pass of the hot path (cir_hash_chunks_dev: Hashes::hash_file
over a device-resident arena, one launch) over one GPU's batch:
  N = 1 : config 2 — 1,048,576 x 32 KiB blocks (32 GiB) of splitmix64 bytes
          (seed 0x5EED0002), blocks 0-15 all-zero, 16-31 bytes(range(256))*128.
  N > 1 : config 4 — rank g holds global blocks [g*2^20, (g+1)*2^20), block i
          = splitmix64 stream seeded 0x5EED0004 ^ i; no collective on the data
          path (range split), weak scaling.
Inputs are generated in HBM before timing.  W warmup steps, then K timed
steps bracketed by barrier + synchronize; value = all ranks' bytes / max
rank time.  The dominant kernel is also timed per launch with HIP events on
the launch stream for the roofline object; `traffic` comes from the
committed rocprofv3 PMC summary (profiles/) when one matches this config.

cpu_baseline: the oracle (C restatement of RFC 7693 BLAKE2b-256 +
dir-signature's block split, "port") on the host cores of this box, over a
bounded sample of the same config-2 blocks, at 4 threads (the reference's
default --disk-threads) and at all host cores (<= 16).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--loader glds|direct]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
METRIC = "GiB/s block-hashed (device-resident, blocks in HBM) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SEED_C2 = 0x5EED0002
SEED_C4 = 0x5EED0004


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--blocks", type=int, default=1 << 20, help="blocks per GPU")
    p.add_argument("--block-size", type=int, default=32768)
    p.add_argument("--loader", choices=["glds", "direct", "api"], default="api",
                   help="api = cir_hash_chunks_dev (production path, LDS-DMA loader)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=4.0,
                   help="target wall seconds per CPU-baseline measurement")
    return p.parse_args()


def fill_config2(ca, data, bs, stream):
    import torch
    ca._n.check(ca._n.lib.cir_fill_splitmix64_dev(data.data_ptr(), data.numel(), SEED_C2, 0, 0,
                                                  stream))
    nspecial = min(32, data.numel() // bs)
    data[:min(16, nspecial) * bs].zero_()
    if nspecial > 16:
        pat = torch.arange(256, dtype=torch.int32, device=data.device).to(torch.uint8)
        data[16 * bs:nspecial * bs].copy_(pat.repeat((nspecial - 16) * bs // 256))


def load_traffic(cfg_key):
    """HBM bytes per launch from a committed PMC summary matching cfg_key."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(cfg_key)
        return None if e is None else e.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(bs, target_s):
    """Oracle BLAKE2b-256 over config-2 blocks on the host (bounded sample)."""
    import numpy as np
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "liboracle_blake2b.so"))
    lib.oracle_hash_chunks.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_void_p, ctypes.c_int]
    lib.oracle_splitmix64_fill.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
    all_cores = max(1, min(16, len(os.sched_getaffinity(0))))

    def measure(threads):
        # calibrate on 64 blocks, then size the sample for ~target_s
        nblk = 64 * threads
        for _ in range(3):
            buf = np.empty(nblk * bs // 8, dtype=np.uint64)
            # config-2 bytes of blocks 32.. (random part of the arena)
            lib.oracle_splitmix64_fill(buf.ctypes.data, 32 * bs // 8, buf.size, SEED_C2, 0, 0)
            out = np.empty(nblk * 32, dtype=np.uint8)
            t0 = time.perf_counter()
            lib.oracle_hash_chunks(buf.ctypes.data, nblk * bs, bs, out.ctypes.data, threads)
            dt = time.perf_counter() - t0
            if dt >= 0.5 * target_s:
                return nblk, dt
            nblk = int(min(nblk * max(2.0, target_s / max(dt, 1e-4)), 1 << 17))
        return nblk, dt

    res = {}
    for threads in sorted({4, all_cores}):
        nblk, dt = measure(threads)
        res[threads] = (nblk * bs / dt / GIB, nblk)
    t4 = res[4]
    return {
        "value": round(t4[0], 4), "unit": "GiB/s", "cores": 4, "kind": "port",
        "sample": "%d x %d B config-2 blocks (splitmix64 seed 0x5EED0002, blocks 32..), "
                  "oracle/blake2b_oracle.c, 4 threads = reference default --disk-threads"
                  % (t4[1], bs),
        "all_cores": {"value": round(res[all_cores][0], 4), "cores": all_cores,
                      "sample_blocks": res[all_cores][1]},
    }


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        log("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    import torch
    import torch.distributed as dist

    import ciruela_amd as ca

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    bs = args.block_size
    nblk = args.blocks
    nbytes = nblk * bs
    stream = torch.cuda.current_stream().cuda_stream
    ctx = ca.Context(device_mask=1 << local)

    data = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    out = torch.empty(nblk * 32, dtype=torch.uint8, device=dev)
    if world == 1:
        workload = "config2"
        fill_config2(ca, data, bs, stream)
    else:
        workload = "config4"
        ca._n.check(ca._n.lib.cir_fill_splitmix64_dev(data.data_ptr(), nbytes, SEED_C4, bs,
                                                      rank * nblk, stream))
    torch.cuda.synchronize()

    lib = ca._n.lib
    if args.loader == "api":
        def step():
            ca._n.check(lib.cir_hash_chunks_dev(ctx.handle, data.data_ptr(), nbytes, bs,
                                                out.data_ptr(), stream))
    else:
        loader = 0 if args.loader == "glds" else 1

        def step():
            ca._n.check(lib.cir_debug_hash_uniform_dev(loader, data.data_ptr(), bs, nblk,
                                                       out.data_ptr(), stream))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ref_out = out.clone()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record()
        step()
        ev[i][1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max = float(t.item())

    # parity spot checks (no oracle here: golden digests + step-to-step identity)
    parity = "ok"
    if not torch.equal(out, ref_out):
        parity = "FAIL: digests differ between steps"
    if workload == "config2" and nblk >= 32:
        with open(os.path.join(ROOT, "tests", "golden", "blake2b256_vectors.json")) as f:
            gold = json.load(f)["config2"]
        if bs == gold["block_size"]:
            d = out[:32 * 32].cpu().numpy().reshape(32, 32)
            if any(d[i].tobytes().hex() != gold["zero_block"] for i in range(16)) or \
               any(d[i].tobytes().hex() != gold["range_block"] for i in range(16, 32)):
                parity = "FAIL: golden config-2 blocks differ"
    if parity != "ok":
        log("PARITY " + parity)

    if rank == 0:
        avg_kern_s = sum(kern_ms) / len(kern_ms) / 1e3
        algo_bytes = nbytes + 32 * nblk
        achieved = algo_bytes / avg_kern_s / 1e9
        loader_name = "glds" if args.loader in ("api", "glds") else "direct"
        cfg_key = "%s/bs%d/n%d/%s" % (workload, bs, nblk, loader_name)
        traffic = load_traffic(cfg_key)
        total_bytes = nbytes * world * args.steps
        rec = {
            "metric": METRIC,
            "value": round(total_bytes / elapsed_max / GIB, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {
                "workload": "%s: %d x %d B blocks per GPU (%.0f GiB), splitmix64, device-resident"
                            % (workload, nblk, bs, nbytes / GIB),
                "blocks_per_gpu": nblk, "block_size": bs, "loader": loader_name,
                "parallelism": "range-split x%d, no collective" % world,
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel_ms_avg": round(avg_kern_s * 1e3, 4),
                "kernel_ms_min": round(min(kern_ms), 4),
                "note": "binding roof is integer VALU (~2.0k VALU ops per 128-B "
                        "compression), see DESIGN.md",
            },
            "parity": parity,
        }
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(bs, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if parity == "ok" else 1


if __name__ == "__main__":
    sys.exit(main())
