"""Device timeline of the timed ICP steps from a rocprofv3 kernel trace (which launch waits for what).

    python scripts/timeline.py gpurun_out/tl/run_kernel_trace.csv [--scans 6] [--out file.txt]

Finds the longest run of consecutive scans (each starts with a k_correspond launch; the fused small-scan path has
one per scan), reports the mean scan period over that run, the per-kernel mean duration split by queue and by
working / early-exit launches (< 3 us), and prints a few scans launch by launch: start offset, duration, the gap
since the previous launch on the same queue ended, queue id.
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"lo::(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--scans", type=int, default=6)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), q))
    rows.sort()
    icp = {"k_correspond", "k_pko_t", "k_pick_correspond", "k_pick", "k_wait_final", "k_wait_seq", "k_solve_correspond",
           "k_solve_pick"}
    # longest stretch of ICP-only launches
    best, cur = (0, 0), 0
    for i, r in enumerate(rows):
        if r[2] in icp:
            if i == 0 or rows[i - 1][2] not in icp:
                cur = i
            if i + 1 - cur > best[1] - best[0]:
                best = (cur, i + 1)
    seg = rows[best[0]:best[1]]
    starts = [r[0] for r in seg if r[2] == "k_correspond"]
    out = []
    if len(starts) > 2:
        per = (starts[-1] - starts[0]) / (len(starts) - 1) / 1e3
        out.append(f"scans in run: {len(starts)}; mean scan period {per:.2f} us ({1e6 / per:.0f} scans/s device-side)")
    agg = defaultdict(list)
    for s, e, n, q in seg:
        d = (e - s) / 1e3
        agg[(n, q, "exit" if d < 3.0 and n in ("k_pko_t", "k_pick_correspond", "k_pick") else "work")].append(d)
    nsc = max(1, len(starts))
    out.append(f"{'kernel':22s} {'queue':>6s} {'kind':>5s} {'count/scan':>10s} {'mean us':>8s} {'us/scan':>8s}")
    for (n, q, k), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        out.append(f"{n:22s} {q:>6s} {k:>5s} {len(v) / nsc:10.2f} {sum(v) / len(v):8.2f} {sum(v) / nsc:8.2f}")
    # a few scans in the middle, launch by launch
    mid = len(starts) // 2
    if starts:
        t0 = starts[mid]
        t1 = starts[min(mid + a.scans, len(starts) - 1)]
        last_end = {}
        out.append(f"\n{'t us':>9s} {'dur':>7s} {'gap':>7s} {'queue':>6s} kernel")
        for s, e, n, q in seg:
            if s < t0 or s > t1:
                last_end[q] = e
                continue
            gap = (s - last_end[q]) / 1e3 if q in last_end else float("nan")
            last_end[q] = e
            out.append(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:7.2f} {gap:7.2f} {q:>6s} {n}")
    txt = "\n".join(out)
    print(txt)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
