#!/usr/bin/env python3
"""Device busy vs idle time per solve from a rocprofv3 kernel-trace database: the kernels are grouped into solves at
every k_inlier launch (the loop-closure ICP's last kernel), and per solve the span (first start to last end), the
summed kernel time and the idle gaps (with the largest gap's position) are reported.  Diagnostic for
bench.py --config kitti_loop."""
import sqlite3
import statistics
import sys


def main():
    db, marker = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "k_inlier")
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, start, end from kernels order by start").fetchall()
    solves, cur = [], []
    for n, s, e in rows:
        cur.append((n.split("(")[0].replace("lo::", "").replace("void ", ""), s, e))
        if marker in n:
            solves.append(cur)
            cur = []
    spans, busy, gaps, between = [], [], [], []
    for k, sv in enumerate(solves[5:], 5):
        spans.append(sv[-1][2] - sv[0][1])
        busy.append(sum(e - s for _, s, e in sv))
        g = [sv[j + 1][1] - sv[j][2] for j in range(len(sv) - 1)]
        gaps.append(max(g) if g else 0)
        between.append(sv[0][1] - solves[k - 1][-1][2])
    med = statistics.median
    print(f"solves {len(spans)}  kernels/solve {med([len(s) for s in solves[5:]])}")
    print(f"span   median {med(spans) / 1e3:.1f} us   busy median {med(busy) / 1e3:.1f} us   "
          f"largest in-solve gap median {med(gaps) / 1e3:.1f} us   gap to previous solve median {med(between) / 1e3:.1f} us")
    sv = solves[len(solves) // 2]
    t0 = sv[0][1]
    for n, s, e in sv:
        print(f"  {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {n}")


if __name__ == "__main__":
    main()
