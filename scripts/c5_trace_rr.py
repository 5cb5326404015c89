#!/usr/bin/env python3
"""C5 roofline from a rocprofv3 kernel trace (r06): the bench's c5_hbm leg times its primary figure over back-to-back
round-robin correspondence launches (lo_bench_correspond_rr: 8 passes x 12 distinct 1M-point scans, HIP events around
the sequence).  This finds those sequences in the trace DB -- runs of >= 96 consecutive 1M-point k_correspond launches
with no other kernel between them -- and reports, per launch, the trace's own duration (end - start) and the period
(first start to last end over the run, / launches: duration + dispatch gap, what the events measure), with the
roofline fraction each gives for the bench's algorithmic bytes.  Every other 1M-point launch (single isolated launches
and the GN loop's) is summarised beside it.

    python scripts/c5_trace_rr.py <db> <bench_json_line_file> [--out profiles/r06_1m_trace_summary.json]"""
import json
import sqlite3
import sys

import numpy as np

HBM_PEAK = 8000.0   # GB/s


def main():
    db, bench_file = sys.argv[1], sys.argv[2]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else ""
    line = [ln for ln in open(bench_file).read().splitlines() if ln.strip().startswith("{")][-1]
    b = json.loads(line)["c5_hbm"]
    alg = float(b["roofline"]["alg_bytes_per_launch"])
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = list(c.execute(f"select start, end, {name} from kernels order by start"))
    big = lambda r: "k_correspond(" in r[2] and (r[1] - r[0]) >= 8000   # noqa: E731
    runs, cur = [], []
    for r in rows:
        if big(r):
            cur.append(r)
        else:
            if len(cur) >= 96:
                runs.append(cur)
            cur = []
    if len(cur) >= 96:
        runs.append(cur)
    in_runs = {id(r) for run in runs for r in run}
    dur = np.array([r[1] - r[0] for run in runs for r in run], float)
    per = np.array([(run[-1][1] - run[0][0]) / len(run) for run in runs], float)
    other = np.array([r[1] - r[0] for r in rows if big(r) and id(r) not in in_runs], float)
    frac = lambda ns: alg / (ns * 1e-9) / 1e9 / HBM_PEAK   # noqa: E731
    res = {
        "what": "rocprofv3 --kernel-trace of the bench's C5 leg (scripts/gpu_r06_t2.sh); the round-robin sequences of the "
                "primary c5_hbm timing found in the trace DB (scripts/c5_trace_rr.py)",
        "alg_bytes_per_launch": alg,
        "rr_sequences": len(runs),
        "rr_launches": int(len(dur)),
        "rr_duration_ns": {"mean": float(dur.mean()), "median": float(np.median(dur)), "p10": float(np.percentile(dur, 10)),
                           "p90": float(np.percentile(dur, 90))} if len(dur) else None,
        "rr_period_ns_per_launch": [float(p) for p in per],
        "frac_from_trace_duration_median": frac(float(np.median(dur))) if len(dur) else None,
        "frac_from_trace_period_mean": frac(float(per.mean())) if len(per) else None,
        "bench_primary": {"kernel_us": b["roofline"]["kernel_us"], "frac": b["roofline"]["frac"],
                          "kernel_us_span": b["roofline"].get("kernel_us_span"),
                          "kernel_us_events_single": b["roofline"].get("kernel_us_events_single")},
        "other_1M_launches": {"count": int(len(other)), "median_ns": float(np.median(other)) if len(other) else None,
                              "note": "single isolated launches (span / events legs) and the GN loop's launches"},
    }
    if len(per):
        res["bench_vs_trace_period"] = b["roofline"]["kernel_us"] * 1e3 / float(per.mean())
    s = json.dumps(res, indent=1)
    print(s)
    if out:
        open(out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
