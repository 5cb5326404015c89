#!/usr/bin/env python3
"""Duration histogram of one kernel from a rocprofv3 SQLite results database: name filter, min ns; prints count,
mean, median, p10 / p90 of the launches at or above the minimum (e.g. the 1M-point k_correspond launches of a run
that also times small scans)."""
import sqlite3
import sys

import numpy as np


def main():
    db, pat, lo = sys.argv[1], sys.argv[2], float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    d = np.array([r[0] for r in c.execute(f"select end-start from kernels where {name} like ?", (f"%{pat}%",))], float)
    d = d[d >= lo]
    if not len(d):
        print(f"{pat}: no launches >= {lo} ns")
        return
    print(f"{pat} (>= {lo:.0f} ns): {len(d)} launches, mean {d.mean():.0f} ns, median {np.median(d):.0f}, "
          f"p10 {np.percentile(d, 10):.0f}, p90 {np.percentile(d, 90):.0f}, min {d.min():.0f}")


if __name__ == "__main__":
    main()
