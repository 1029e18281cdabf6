"""Compact view of a config-5 record (bench.py --workload config5): per scan
the footer mode, seconds, GiB/s, footer busy / tail and the batch split."""
import json
import sys

rec = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
nbytes = rec["bytes"]
print("config5 value %.2f GiB/s (first %.2f), matches_oracle %s, index %.1f MB" % (
    rec["value"], rec["value_first"], rec["matches_oracle"], rec["index_bytes"] / 1e6))
print("by footer mode: %s" % json.dumps(rec.get("by_footer_mode")))
scans = rec.get("scans", [])
if scans and "phases_ms" not in scans[0]:  # compact form: the best scan in full
    print("(compact record: per-scan %s)" % json.dumps(scans))
    scans = [rec["phases_best"]]
for sc in scans:
    ph, b = sc["phases_ms"], sc["batches"] or {}
    print("%-4s %.3f s %6.2f GiB/s | loop %.0f tail %.1f footer busy %.0f ms feeds %d | "
          "h2d med %.2f p90 %.2f (reading %.2f n=%d, alone %s n=%d) read med %.2f wait sum %.0f "
          "copy busy %.2f read busy %.2f" % (
              sc["footer"], sc["seconds"], nbytes / sc["seconds"] / 2**30, ph["hash_loop_ms"],
              ph["footer_tail_ms"], ph["footer_busy_ms"], sc["footer_feeds"],
              b["h2d_ms"]["median"], b["h2d_ms"]["p90"], b["h2d_ms_while_reading"]["median"] or 0,
              b["h2d_ms_while_reading"]["batches"], b["h2d_ms_without_reads"]["median"],
              b["h2d_ms_without_reads"]["batches"], b["read_ms"]["median"], b["wait_ms"]["sum"],
              b["copy_busy_frac"], b["read_busy_frac"]))
