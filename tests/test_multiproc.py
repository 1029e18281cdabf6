"""The N > 1 bench path on CPU: world_size-2 `gloo` processes.

The block hash shards with no data-path collective: rank g
owns global blocks [g*n, (g+1)*n) of config 4, each block its own splitmix64
stream (seed 0x5EED0004 ^ global index).  Checked here without a GPU:
  * the shards are disjoint and cover [0, world*n);
  * every rank regenerates its blocks from the global index alone, so a
    block's digest does not depend on which rank hashed it (oracle digests of
    boundary blocks computed on both sides agree);
  * the timing and the whole-job rate come from bench.py's own functions
    (timed_steps -> max_over_ranks -> job_rate), run here under gloo with
    ranks of different speed: the reported time is the slowest rank's;
  * bench.config4_check, the N>1 bench line's parity check, finds no
    mismatch on a shard's true digests and every corrupted one.
"""
import time
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

SEED_C4 = 0x5EED0004
BS = 4096  # small blocks: the property does not depend on the size


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle():
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "liboracle_blake2b.so"))
    vp, u64 = ctypes.c_void_p, ctypes.c_uint64
    lib.oracle_hash_chunks.argtypes = [vp, u64, u64, vp, ctypes.c_int]
    lib.oracle_splitmix64_fill.argtypes = [vp, u64, u64, u64, u64, u64]
    return lib


def _worker(rank, world, port, nblk, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = bench.shard(rank, world, nblk)
    lib = _oracle()
    # this rank's shard, generated exactly as bench.py fills HBM (per-block seeds)
    buf = np.empty(count * BS // 8, dtype=np.uint64)
    lib.oracle_splitmix64_fill(buf.ctypes.data, 0, buf.size, SEED_C4, BS // 8, first)
    dig = np.empty(count * 32, dtype=np.uint8)
    steps = 3

    def step(i):  # the rank's work; rank r is (r + 1) x slower
        lib.oracle_hash_chunks(buf.ctypes.data, count * BS, BS, dig.ctypes.data, 1)
        time.sleep(0.05 * (rank + 1))
    elapsed = bench.timed_steps(step, steps, lambda: None, dist.barrier)
    elapsed_max = bench.max_over_ranks(elapsed)
    value = bench.job_rate(count * BS, world, steps, elapsed_max)
    # bench's N>1 parity check on this shard: clean, then one corrupted digest
    nbad, checked = bench.config4_check(lib, dig, count * BS, BS, first, sample=8)
    bad = dig.copy()
    bad[32 * (count - 1)] ^= 1
    nbad2, _ = bench.config4_check(lib, bad, count * BS, BS, first, sample=8)
    # gather shard bounds, timings and the digest of every rank's first block
    t = torch.tensor([first, count, int(elapsed * 1e9), int(elapsed_max * 1e9), nbad, nbad2,
                      checked] + list(dig[:32].astype(np.int64)), dtype=torch.int64)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    if rank == 0:
        q.put(([p.tolist() for p in parts], value, elapsed_max))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_range_split_gloo(world):
    nblk = 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nblk, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts, value, elapsed_max = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    bounds = sorted((p[0], p[1]) for p in parts)
    assert bounds[0][0] == 0
    for (a, n), (b, _) in zip(bounds, bounds[1:]):
        assert a + n == b  # contiguous, disjoint
    assert bounds[-1][0] + bounds[-1][1] == world * nblk
    # max over ranks: every rank got the same maximum, the slowest rank's
    # time, at least its 3 x 0.05 * world seconds of sleep
    assert {p[3] for p in parts} == {max(p[2] for p in parts)}
    assert elapsed_max >= 3 * 0.05 * world
    assert value == pytest.approx(nblk * BS * world * 3 / elapsed_max / (1 << 30))
    for p in parts:
        assert p[4] == 0 and p[5] == 1 and p[6] >= 8
    # the first block of rank 1 == global block nblk, regenerated from scratch here
    lib = _oracle()
    buf = np.empty(BS // 8, dtype=np.uint64)
    lib.oracle_splitmix64_fill(buf.ctypes.data, 0, buf.size, SEED_C4, BS // 8, nblk)
    dig = np.empty(32, dtype=np.uint8)
    lib.oracle_hash_chunks(buf.ctypes.data, BS, BS, dig.ctypes.data, 1)
    assert [int(x) for x in dig] == parts[1][7:]


def test_bench_launches_ranks_itself():
    """`bench.py --gpus 2` with no launcher around it starts two rank
    processes itself (torch.distributed.run, rendezvous on 127.0.0.1) before
    touching a GPU; the line reports the process group's own world size and
    the config-4 workload, and the shards tile [0, 2n)."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dist-backend", "gloo", "--dry-run", "--steps", "2", "--blocks", "64"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["ranks_seen"] == 2
    assert rec["config"]["workload"] == "config4"
    assert sorted(map(tuple, rec["shards"])) == [(0, 64), (64, 64)]


def _run_bench(args, timeout=240):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                          capture_output=True, text=True, timeout=timeout, env=env)


def _line(r):
    import json
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (r.stdout, r.stderr[-2000:])
    return json.loads(lines[0])


def test_bad_digest_on_rank1_fails_the_job_line():
    """Rank 1 corrupts one digest of its shard: the line rank 0 prints says
    FAIL and names rank 1 (parity is reduced over the job, not rank 0's
    view), and the job exits non-zero."""
    r = _run_bench(["--gpus", "2", "--dist-backend", "gloo", "--dry-run", "--steps", "2",
                    "--blocks", "64", "--dry-run-bad-rank", "1"])
    rec = _line(r)
    assert r.returncode != 0
    assert rec["parity"].startswith("FAIL") and "rank(s) 1" in rec["parity"]
    assert [p["mismatches"] for p in rec["per_rank"]] == [0, 1]
    assert rec["parity_checked_blocks"] == sum(p["checked"] for p in rec["per_rank"]) > 0
    # and clean shards on both ranks pass
    r = _run_bench(["--gpus", "2", "--dist-backend", "gloo", "--dry-run", "--steps", "2",
                    "--blocks", "64"])
    rec = _line(r)
    assert r.returncode == 0 and rec["parity"] == "ok"
    assert [p["kernel_ms_avg"] for p in rec["per_rank"]] == [10.0, 11.0]


def test_force_dist_launches_one_rank():
    """`bench.py --gpus 1 --force-dist` with no launcher starts one rank
    through torch.distributed.run (the N>1 code path at world size 1)."""
    r = _run_bench(["--gpus", "1", "--force-dist", "--dist-backend", "gloo", "--dry-run",
                    "--steps", "2", "--blocks", "16"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "launching 1 ranks" in r.stderr
    rec = _line(r)
    assert rec["ranks_seen"] == 1 and rec["config"]["workload"] == "config4"
    assert rec["parity"] == "ok"


def test_devices_seen_in_the_line():
    """The N>1 line carries every rank's device identity (devices_seen,
    gathered over the process group) and whether they are distinct.  Under
    --dist-backend nccl (one GPU per rank) two ranks on one device fail the
    line and the job; a gloo rehearsal with shared GPUs only notes it."""
    r = _run_bench(["--gpus", "2", "--dist-backend", "gloo", "--dry-run", "--steps", "1",
                    "--blocks", "16"])
    rec = _line(r)
    assert r.returncode == 0 and rec["devices_distinct"] is True
    assert [d["rank"] for d in rec["devices_seen"]] == [0, 1]
    assert len({d["pci_bus_id"] for d in rec["devices_seen"]}) == 2
    r = _run_bench(["--gpus", "2", "--dist-backend", "nccl", "--dry-run", "--steps", "1",
                    "--blocks", "16", "--dry-run-shared-device"])
    rec = _line(r)
    assert r.returncode != 0 and rec["devices_distinct"] is False
    assert rec["parity"].startswith("FAIL") and "share a device" in rec["parity"]
    r = _run_bench(["--gpus", "2", "--dist-backend", "gloo", "--dry-run", "--steps", "1",
                    "--blocks", "16", "--dry-run-shared-device"])
    rec = _line(r)
    assert r.returncode == 0 and rec["parity"] == "ok" and rec["devices_distinct"] is False
    assert "share a device" in rec["devices_note"]


def test_devices_check_rule():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    a = {"pci_bus_id": "0000:05:00.0", "uuid": "aa"}
    b = {"pci_bus_id": "0000:15:00.0", "uuid": "bb"}
    assert bench.devices_check([a, b], True) == (True, None)
    ok, msg = bench.devices_check([a, b, dict(a)], True)
    assert not ok and msg.startswith("FAIL") and "0/2" in msg
    ok, msg = bench.devices_check([a, {"pci_bus_id": "0000:99:00.0", "uuid": "aa"}], False)
    assert not ok and not msg.startswith("FAIL")  # same UUID, another bus id: still one device
    assert bench.devices_check([a], True) == (True, None)
