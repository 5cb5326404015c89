#!/usr/bin/env python3
"""Per-kernel duration statistics from a rocprofv3 SQLite results database (rocprofv3 --kernel-trace without
--output-format csv): name, calls, total / average / min / max ns, sorted by total.  Optional name filter."""
import sqlite3
import sys


def main():
    db, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "lo::")
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     f"from kernels group by {name} order by sum(end-start) desc").fetchall()
    print('"Name","Calls","TotalDurationNs","AverageNs","MinNs","MaxNs"')
    for r in rows:
        if pat in r[0]:
            print(f'"{r[0]}",{r[1]},{r[2]},{r[3]:.1f},{r[4]},{r[5]}')


if __name__ == "__main__":
    main()
