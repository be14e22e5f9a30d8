#!/usr/bin/env python3
"""One pipelined step's kernel timeline per queue from a rocprofv3 run of bench.py (rocpd database), plus each
queue's chain length per step (first start to last end between two grab launches):
    python tools/timeline.py gpurun_out/<tag>_prof_c2/run_results.db [step_from_end=2] [min_grab_us=0]
(min_grab_us: count only grab launches at least that long -- e.g. 50 to skip bench.py's trailing B = 1 steps)"""
import collections
import sqlite3
import sys


def short(n):
    if "grab" in n:
        return "grab"
    b = n.split("(")[0]
    parts = [p for p in b.split("::") if p]
    return parts[-1] if parts else b


def main(db, back=2, min_grab_us=0.0):
    c = sqlite3.connect(db)
    rows = [(short(n), q, s, e) for n, q, s, e in c.execute("select name, queue_id, start, end from kernels order by start")
            if "copyBuffer" not in n and "at::" not in n]
    starts = [r[2] for r in rows if r[0] == "grab" and (r[3] - r[2]) / 1e3 >= min_grab_us]
    s0, s1 = starts[-back - 1], starts[-back]
    span = collections.defaultdict(lambda: [None, None])
    print(f"step {(s1 - s0) / 1e3:.0f} us (grab to grab)")
    for n, q, s, e in rows:
        if s0 <= s < s1:
            print(f"q{q} {(s - s0) / 1e3:7.0f} {(e - s0) / 1e3:7.0f} {(e - s) / 1e3:7.0f}  {n}")
            sp = span[q]
            sp[0] = s if sp[0] is None else min(sp[0], s)
            sp[1] = e if sp[1] is None else max(sp[1], e)
    for q, (a, b) in sorted(span.items()):
        print(f"queue {q}: chain {(b - a) / 1e3:.0f} us, ends {(b - s0) / 1e3:.0f} us after the step's grab")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2, float(sys.argv[3]) if len(sys.argv) > 3 else 0.0)
