"""Summarise rocprofv3 PMC passes into per-launch HBM traffic for one kernel.

    python scripts/pmc_summary.py --workload kitti --kernel k_correspond \
        --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --out profiles/pmc_traffic.json

Each pass directory holds rocprofv3 `--pmc <counter> --kernel-trace --output-format csv` output.
Per MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half
of the bytes of a wide (16 B/lane) coalesced stream and other widths are uncalibrated, so both the raw value
and the x2-corrected read side are recorded; `hbm_bytes_per_launch` uses the corrected read side.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os


def per_launch(pass_dir: str, counter: str, kernel: str, min_run: int = 20):
    """Mean counter value per launch of `kernel` over its isolated runs (>= min_run consecutive dispatches of
    the same kernel = bench.py's lo_bench_kernel phase, the launches `kernel_us` times), and over all launches."""
    files = glob.glob(os.path.join(pass_dir, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {pass_dir}")
    rows = []
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if (row.get("Counter_Name") or "") != counter:
                    continue
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                rows.append((int(row["Dispatch_Id"]), name, float(row["Counter_Value"])))
    rows.sort()
    match = lambda n: (kernel + "(") in n or (kernel + "<") in n   # noqa: E731  (k_correspond vs k_correspond_b)
    allv = [v for _, n, v in rows if match(n)]
    if not allv:
        raise SystemExit(f"no {counter} rows for {kernel} in {pass_dir}")
    iso, i = [], 0
    while i < len(rows):
        j = i
        while j < len(rows) and rows[j][1] == rows[i][1]:
            j += 1
        if match(rows[i][1]) and j - i >= min_run:
            iso.extend(v for _, _, v in rows[i:j])
        i = j
    mean = lambda v: sum(v) / len(v) if v else float("nan")   # noqa: E731
    return mean(iso), len(iso), mean(allv), len(allv)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", required=True)
    ap.add_argument("--kernel", default="k_correspond")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    f_kib, nf, f_all, nfa = per_launch(a.fetch, "FETCH_SIZE", a.kernel)
    w_kib, nw, w_all, nwa = per_launch(a.write, "WRITE_SIZE", a.kernel)
    entry = {
        "kernel": a.kernel,
        "launches": "isolated back-to-back launches (bench.py lo_bench_kernel / lo_batch_bench_correspond phase, "
                    "the ones kernel_us times)",
        "isolated_launches_fetch_pass": nf, "isolated_launches_write_pass": nw,
        "fetch_size_kib_raw": f_kib, "write_size_kib_raw": w_kib,
        "fetch_bytes_corrected": 2.0 * f_kib * 1024.0,
        "write_bytes": w_kib * 1024.0,
        "hbm_bytes_per_launch": 2.0 * f_kib * 1024.0 + w_kib * 1024.0,
        "all_launches": {"fetch_launches": nfa, "fetch_size_kib_raw": f_all, "write_size_kib_raw": w_all,
                         "note": "includes early-exit launches after convergence"},
        "correction": "FETCH_SIZE x2 (gfx950 wide-stream calibration, MI355X_MICROARCH.md §HBM); Infinity-Cache hits are "
                      "counted by these memory-side counters",
        "note": a.note,
    }
    d = {}
    if os.path.exists(a.out):
        with open(a.out) as fh:
            d = json.load(fh)
    d[a.workload] = entry
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(d, fh, indent=2)
    print(json.dumps({a.workload: entry}, indent=2))


if __name__ == "__main__":
    main()
