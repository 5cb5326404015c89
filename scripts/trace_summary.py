"""Per-kernel durations from a rocprofv3 kernel trace, split by phase.

    python scripts/trace_summary.py gpurun_out/stats_kitti/run_kernel_trace.csv [--out profiles/r01_kitti_trace_summary.json]

bench.py measures each kernel's `kernel_us` live with HIP events over back-to-back launches of that kernel
alone (lo_bench_kernel).  In the kernel trace those launches form long runs of one kernel name; the ICP steps
interleave k_init / k_correspond / k_pko / k_accumulate / k_solve.  This script reports both:
  * "isolated": mean duration over runs of >= 20 consecutive launches of the same kernel (= bench's kernel_us)
  * "in_step":  mean duration inside the interleaved ICP steps, split into working launches and the
                early-exit launches that follow convergence (DevState::done set; a few hundred ns each)
"""
from __future__ import annotations

import argparse
import csv
import json
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"lo::(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out", default="")
    ap.add_argument("--min-run", type=int, default=20)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    # runs of identical consecutive kernel names
    runs, i = [], 0
    while i < len(rows):
        j = i
        while j < len(rows) and rows[j][2] == rows[i][2]:
            j += 1
        runs.append((rows[i][2], rows[i:j]))
        i = j
    iso = defaultdict(list)
    step = defaultdict(list)
    for name, rr in runs:
        durs = [(e - s) / 1e3 for s, e, _ in rr]
        (iso if len(rr) >= a.min_run else step)[name].extend(durs)
    out = {"isolated_us": {}, "in_step_us": {}}
    for k, v in sorted(iso.items()):
        out["isolated_us"][k] = {"launches": len(v), "mean": sum(v) / len(v)}
    for k, v in sorted(step.items()):
        if not k.startswith("k_"):
            continue
        thr = 0.25 * max(v)
        work = [x for x in v if x >= thr]
        idle = [x for x in v if x < thr]
        out["in_step_us"][k] = {"launches": len(v), "mean_all": sum(v) / len(v),
                                "working_launches": len(work), "mean_working": sum(work) / max(len(work), 1),
                                "early_exit_launches": len(idle), "mean_early_exit": sum(idle) / max(len(idle), 1)}
    s = json.dumps(out, indent=2)
    print(s)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
