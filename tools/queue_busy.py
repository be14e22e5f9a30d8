#!/usr/bin/env python3
"""Per-queue busy time and per-kernel time per step of a pipelined bench run (rocpd database):
    python tools/queue_busy.py gpurun_out/<tag>_prof/run_results.db [steps=5]"""
import collections
import sqlite3
import sys


def main(db, steps=5):
    c = sqlite3.connect(db)
    rows = c.execute("select name, queue_id, start, end from kernels order by start").fetchall()
    rows = [r for r in rows if "copyBuffer" not in r[0] and "at::" not in r[0]]
    starts = [r[2] for r in rows if "grab" in r[0]]
    t0, t1 = starts[-steps - 1], starts[-1]
    seg = [r for r in rows if t0 <= r[2] < t1]
    busy, per = collections.defaultdict(float), collections.defaultdict(float)
    for n, q, s, e in seg:
        busy[q] += (e - s) / 1e6
        per[n.split("(")[0].split("::")[-1]] += (e - s) / 1e6
    print(f"step {(t1 - t0) / 1e6 / steps:.3f} ms")
    for q, v in sorted(busy.items()):
        print(f"queue {q}: {v / steps:.3f} ms busy per step")
    for k, v in sorted(per.items(), key=lambda x: -x[1]):
        print(f"{k:40s} {v / steps:7.3f} ms/step")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
