"""bench.py's line assembly on CPU (no GPU): the secondary legs' bookkeeping.

* a config-5 leg whose tree cannot fit the tmpfs is skipped with a reason,
  before anything touches a device, and does not count as a parity failure;
* the host record names the CPU share the box grants (cgroup quota);
* the roofline's PMC-derived fields come from the committed summary.
"""
import argparse
import os
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_config5_leg_skips_when_the_tree_does_not_fit(tmp_path):
    args = argparse.Namespace(tree_dir=str(tmp_path / "tree"), tree_gib=1e9, steps=3)
    rec = bench.run_config5_leg(args, None, None, None, None)
    assert "skipped" in rec and rec["matches_oracle"] is None
    assert not os.path.exists(args.tree_dir)


def test_skipped_leg_is_not_a_parity_failure():
    sec = {"config5": {"skipped": "no room", "matches_oracle": None},
           "config3": {"matches_oracle": True}}
    assert not any(r.get("matches_oracle", False) is False for r in sec.values())
    sec["config2host"] = {"error": "RuntimeError: x", "matches_oracle": False}
    assert any(r.get("matches_oracle", False) is False for r in sec.values())


def test_host_record_fields():
    h = bench.host_info()
    assert {"nproc", "affinity_cpus", "cgroup_cpu_quota", "cpu_model",
            "cpu_share_per_gpu"} <= set(h)


def test_committed_pmc_summary_feeds_the_roofline():
    key = bench.traffic_key(32768, 1 << 20, "api")
    assert key == "bs32768/n1048576/cir_hash_chunks_dev"
    traffic = bench.load_traffic(key)
    cycles = bench.load_traffic(key, "cycles")
    assert traffic and abs(traffic / 34393292800 - 1) < 0.01
    assert 0.9 < cycles["cycle_frac"] <= 1.0
    assert cycles["clock_ghz_k_chunks"] < cycles["clock_ghz_k_compress_only"]


def test_entry_point_names_the_timed_call():
    """config.entry_point says which C-ABI call the timed steps made: the
    production cir_hash_chunks_dev for --loader api (the default), the A/B
    kernel for glds / direct; the PMC summary key follows it."""
    api = bench.entry_point("api")
    assert api == {"entry_point": "cir_hash_chunks_dev", "loader": "lds-dma"}
    for loader, name in (("glds", "lds-dma"), ("direct", "direct")):
        ep = bench.entry_point(loader)
        assert ep == {"entry_point": "cir_debug_hash_uniform_dev", "loader": name}
        assert bench.traffic_key(32768, 1 << 20, loader) != bench.traffic_key(32768, 1 << 20,
                                                                                "api")
    import sys as _s
    argv, _s.argv = _s.argv, ["bench.py"]
    try:
        assert bench.parse().loader == "api"
    finally:
        _s.argv = argv


def test_job_parity_names_failing_ranks():
    rows = [[0, 192, 0, 14.5, 14.3], [1, 192, 0, 14.9, 14.6]]
    parity, checked = bench.job_parity(rows)
    assert parity.startswith("FAIL") and "rank(s) 1" in parity and checked == 384
    assert bench.job_parity([[0, 192, 0, 1, 1], [0, 192, 0, 1, 1]]) == ("ok", 384)
    # a failed check with no mismatch count (steps differ) fails too
    assert bench.job_parity([[0, 32, 1, 1, 1]])[0].startswith("FAIL")


def test_scan_batch_summary_splits_h2d_by_reads():
    """Config 5's batch summary: an upload that runs while the readers fill
    the next slot is counted under h2d_ms_while_reading, one that runs alone
    under h2d_ms_without_reads; busy fractions are over the hash loop."""
    mib = 1 << 20
    rows = [  # batch 0: H2D alone; batch 1: H2D entirely under batch 2's reads
        dict(bytes=256 * mib, blocks=8192, wait_ms=0.0, read_start_ms=0.0, read_end_ms=4.0,
             h2d_start_ms=4.0, h2d_end_ms=9.0, hash_start_ms=9.0, done_ms=9.5),
        dict(bytes=256 * mib, blocks=8192, wait_ms=0.5, read_start_ms=10.0, read_end_ms=14.0,
             h2d_start_ms=14.0, h2d_end_ms=21.0, hash_start_ms=21.0, done_ms=21.5),
        dict(bytes=256 * mib, blocks=8192, wait_ms=0.0, read_start_ms=14.0, read_end_ms=22.0,
             h2d_start_ms=22.0, h2d_end_ms=27.0, hash_start_ms=27.0, done_ms=27.5)]
    s = bench.scan_batch_summary(rows, {"hash_loop_ms": 30.0})
    assert s["batches"] == 3
    assert s["h2d_ms_without_reads"] == {"median": 5.0, "batches": 2}
    assert s["h2d_ms_while_reading"] == {"median": 7.0, "batches": 1}
    assert s["h2d_ms"]["sum"] == 17.0 and s["read_ms"]["sum"] == 16.0
    assert s["copy_busy_frac"] == round(17 / 30, 3)
    assert s["read_busy_frac"] == round(16 / 30, 3)  # 0-4 and 10-22 merged
    assert bench.scan_batch_summary([], {}) is None


def test_config5_leg_checks_ram_and_reuses_a_complete_tree(tmp_path, monkeypatch):
    args = argparse.Namespace(tree_dir=str(tmp_path / "tree"), tree_gib=1.0, steps=1)
    monkeypatch.setattr(bench, "mem_available_gib", lambda: 2.0)
    rec = bench.run_config5_leg(args, None, None, None, None)
    assert "MemAvailable" in rec["skipped"] and rec["matches_oracle"] is None
    # a complete tree left behind is not re-checked against free space / RAM
    os.makedirs(args.tree_dir)
    open(os.path.join(args.tree_dir, ".complete-32-32"), "w").close()
    assert bench.tree_complete(args.tree_dir, 1.0)
    called = []
    monkeypatch.setattr(bench, "run_config5", lambda a, ca, ctx: called.append(1) or {"x": 1})
    assert bench.run_config5_leg(args, None, None, None, None) == {"x": 1} and called
    assert not os.path.exists(args.tree_dir)  # removed afterwards


def test_config5_leg_tree_write_failure_is_a_skip(tmp_path, monkeypatch):
    """A tree the box cannot write (tmpfs full, permissions) skips the leg
    with the reason instead of reporting a parity failure."""
    args = argparse.Namespace(tree_dir=str(tmp_path / "tree"), tree_gib=0.01, steps=1)
    monkeypatch.setattr(bench, "mem_available_gib", lambda: 1e6)

    def boom(root, gib):
        raise OSError(28, "No space left on device")
    monkeypatch.setattr(bench, "make_tree", boom)
    rec = bench.run_config5_leg(args, None, None, None, None)
    assert "No space left" in rec["skipped"] and rec["matches_oracle"] is None


def test_make_tree_replaces_a_tree_of_another_size(tmp_path):
    """A tree of another size left at --tree-dir (an earlier run with another
    --tree-gib) is removed before the new one is written, so the scan indexes
    exactly the files its byte count assumes."""
    root = str(tmp_path / "tree")

    def files():
        return sorted(f for _, _, fs in os.walk(root) for f in fs if not f.startswith("."))
    assert bench.make_tree(root, 4 / 1024, file_mib=1, ndirs=2) == 4
    assert len(files()) == 4
    assert bench.make_tree(root, 2 / 1024, file_mib=1, ndirs=2) == 2
    assert files() == ["f00000.bin", "f00001.bin"]
    assert bench.make_tree(root, 2 / 1024, file_mib=1, ndirs=2) == 2  # complete: reused
    assert os.listdir(root).count(".complete-2-1") == 1
