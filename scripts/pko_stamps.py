"""Diagnostic: phase timing of k_pko from the -DLO_PKO_STAMPS library (liblo_icp_diag.so).
Runs lo_pko_scale_factor on golden + ICP-like residual vectors and prints s_memtime deltas per phase."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LO_ICP_LIB"] = os.environ.get("LO_DIAG_LIB", os.path.join(ROOT, "lidar_odometry_amd", "liblo_icp_diag.so"))
sys.path.insert(0, ROOT)
from lidar_odometry_amd import IterativeClosestPointOptimizer, lib  # noqa: E402

icp = IterativeClosestPointOptimizer(max_points=1 << 17)
z = np.load(os.path.join(ROOT, "tests", "golden", "pko_inputs.npz"))
names = ["prefix", "sample", "kmeans", "initvar", "EM", "JS"]
for line in open(os.path.join(ROOT, "tests", "golden", "pko_golden.jsonl")):
    d = json.loads(line)
    r = z[f"case_{d['case']}"]
    for rep in range(2):
        a, _ = icp.pko_scale_factor(r)
    out = (C.c_ulonglong * 16)()
    lib().lo_debug_counters(icp.ctx, out)
    t = [out[i] for i in range(7)]
    dt = [t[i + 1] - t[i] for i in range(6)]
    print(f"case {d['case']:2d} n={d['n']:6d} alpha_ok={a == d['alpha']} em_iters={out[8]:3d} km_iters={out[9]:3d} "
          + " ".join(f"{n}={v}" for n, v in zip(names, dt)) + f" total={t[6] - t[0]}"
          + (f" | em50: E={out[11] - out[10]} reduce={out[12] - out[11]} M={out[13] - out[12]}" if out[13] else ""))
