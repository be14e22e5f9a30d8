#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run into the CSV committed under profiles/.

    python tools/prof_summary.py gpurun_out/prof/run_results.db profiles/rNN_<name>_kernel_stats.csv

Reads the rocpd SQLite output (rocprofv3's default format on ROCm 7.2) and
writes per-kernel Name, Calls, TotalDurationNs, AverageNs, Percentage, Min/Max,
the same columns as rocprofv3's kernel_stats.csv.
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
        "from kernels group by name order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, tot, avg, mn, mx in rows:
            w.writerow([name, n, tot, round(avg, 1), round(100.0 * tot / total, 3), mn, mx])
    for name, n, tot, avg, *_ in rows[:12]:
        print(f"{avg / 1e3:10.1f} us x{n:4d}  {name[:100]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
