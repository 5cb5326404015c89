#!/usr/bin/env python3
"""Per-scan kernel timeline from a rocprofv3 SQLite results database: for a few scans containing a marker kernel, every
lo:: kernel from that scan's first k_correspond (relative start / end in us, duration, queue)."""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_rank_runs"
    which = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [300, 301]
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, queue_id from kernels where name like '%lo::k_%' order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    for w in which:
        if w >= len(idx):
            continue
        j = idx[w]
        while j > 0 and not rows[j][0].startswith("lo::k_correspond("):
            j -= 1
        t0 = rows[j][1]
        print("--- scan with marker #%d" % w)
        k = j
        while k < len(rows) and (k == j or not rows[k][0].startswith("lo::k_correspond(")):
            r = rows[k]
            print(f"{r[0].split('(')[0][-34:]:34s} q{r[3]} {(r[1] - t0) / 1e3:8.2f} {(r[2] - t0) / 1e3:8.2f} dur {(r[2] - r[1]) / 1e3:7.2f}")
            k += 1


if __name__ == "__main__":
    main()
