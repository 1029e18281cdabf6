"""Kernel statistics from a rocprofv3 database (rocpd SQLite, the default
output of `rocprofv3 --kernel-trace --stats` on ROCm 7) as the CSV files the
earlier rounds committed under profiles/:

  <out>/prof_kernel_stats.csv   Name, Calls, TotalDurationNs, AverageNs, Percentage
  <out>/prof_trace_<kernel>.csv every launch of one kernel, in order
                                (start, end, duration in ns)

    python tools/rocpd_stats.py gpurun_out/r6val/prof/run_results.db profiles/r06/final k_chunks
"""
import csv
import os
import sqlite3
import sys


def main(db, out, kernel=None):
    os.makedirs(out, exist_ok=True)
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage "
                     "from top_kernels order by total_duration desc").fetchall()
    with open(os.path.join(out, "prof_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for name, calls, total, avg, pct in rows:
            # (top_kernels reports microseconds)
            w.writerow([name, calls, round(total * 1e3), round(avg * 1e3), round(pct, 4)])
    if kernel:
        launches = c.execute("select start, end, duration from kernels where name like ? "
                             "order by start", ("%%dev::%s(%%" % kernel,)).fetchall()
        with open(os.path.join(out, "prof_trace_%s.csv" % kernel), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["StartNs", "EndNs", "DurationNs"])
            w.writerows(launches)
        durs = [d for _, _, d in launches]
        if durs:
            last = durs[-20:]
            print("%s: %d launches, average %.3f ms, last 20 average %.3f ms"
                  % (kernel, len(durs), sum(durs) / len(durs) / 1e6, sum(last) / len(last) / 1e6))


if __name__ == "__main__":
    main(*sys.argv[1:])
