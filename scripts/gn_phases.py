"""Diagnostic: phase timing of the persistent GN launch (k_gn, lo_persist.hip) on KITTI-like scans, from the
-DLO_PKO_STAMPS library (make -C lidar_odometry_amd/csrc diag).  Workgroup 0 stamps s_memrealtime (100 MHz) at each
phase boundary of GN iterations 0-2; prints the phase durations (us) per scan, and the whole optimize's device time
(HIP events) with the persistent launch on and off."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LO_ICP_LIB"] = os.environ.get("LO_DIAG_LIB", os.path.join(ROOT, "lidar_odometry_amd", "liblo_icp_diag.so"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

torch.zeros(1, device="cuda")
from lidar_odometry_amd import IterativeClosestPointOptimizer, lib  # noqa: E402
from tests import _data  # noqa: E402

frames = [int(a) for a in sys.argv[1:]] or [11, 13, 17, 21, 25, 31]
icp = IterativeClosestPointOptimizer(max_points=1 << 17)
names = ["A", "waitA", "B", "waitB", "C"]
acc = {k: [] for k in names}
for f in frames:
    m, pts, Ti, _ = _data.kitti_case(f)
    icp.set_surfels(*_data.surfels(m))
    dev = {}
    for pers in (False, True):
        icp.set_persistent(pers)
        ms = []
        for _ in range(5):
            icp.optimize(None, pts, Ti)
            ms.append(icp.get_last_stats().optimization_time_ms)
        dev[pers] = float(np.median(ms)) * 1e3
    out = (C.c_ulonglong * 16)()
    lib().lo_debug_counters(icp.ctx, out)
    it = icp.get_last_stats().num_iterations
    t = [int(out[i]) for i in range(16)]
    parts = []
    prev = t[0]
    for k in range(min(it, 3)):
        row = []
        for j, nm in enumerate(names):
            cur = t[1 + 5 * k + j]
            if cur == 0 or cur < prev:
                break
            d = (cur - prev) / 100.0
            row.append(f"{nm}={d:.1f}")
            acc[nm].append(d)
            prev = cur
        parts.append(f"it{k}[" + " ".join(row) + "]")
    print(f"frame {f}: n={len(pts)} iters={it} device us: launches {dev[False]:.1f} persistent {dev[True]:.1f} | "
          + " ".join(parts), flush=True)
print("mean us per phase: " + " ".join(f"{k}={np.mean(v):.2f}" for k, v in acc.items() if v))
