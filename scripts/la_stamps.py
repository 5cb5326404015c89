"""Diagnostic: stage timing of the lookahead launch (k_la) from the -DLO_PKO_STAMPS library (make -C
lidar_odometry_amd/csrc diag).  For KITTI-like scans: optimize() with the lookahead on, then the s_memtime deltas of
the last k_la launch's main workgroup 0 (PKO phases) and chain 0 (prefix, iteration-k solve, correspondences,
iteration-(k+1) PKO, solve, next correspondences)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LO_ICP_LIB"] = os.environ.get("LO_DIAG_LIB", os.path.join(ROOT, "lidar_odometry_amd", "liblo_icp_diag.so"))
sys.path.insert(0, ROOT)
from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer, lib  # noqa: E402
from tests import _data  # noqa: E402

icp = IterativeClosestPointOptimizer(ICPConfig(max_iterations=3, translation_tolerance=1e-9, rotation_tolerance=1e-9), max_points=1 << 17)
main_names = ["prefix", "sample", "kmeans", "initvar", "EM", "JS"]
chain_names = ["acc", "solve", "corr", "pko", "acc", "solve", "corr"]
for f in (11, 13, 17, 21, 25, 31):
    m, pts, Ti, _ = _data.kitti_case(f)
    k, n, c = _data.surfels(m)
    icp.set_surfels(k, n, c)
    for rep in range(2):
        icp.optimize(None, pts, Ti)
    st = icp.get_last_stats()
    out = (C.c_ulonglong * 16)()
    lib().lo_debug_counters(icp.ctx, out)
    t = [out[i] for i in range(16)]
    md = [t[i + 1] - t[i] for i in range(6)]
    cd = [t[9 + i] - t[8 + i] for i in range(7)]
    print(f"frame {f}: n={len(pts)} iters={st.num_iterations} em_iters={t[8 - 0] if False else out[8]} | main "
          + " ".join(f"{a}={b}" for a, b in zip(main_names, md)) + f" total={t[6] - t[0]} (chain 0's PKO) | chain0 "
          + " ".join(f"{a}={b}" for a, b in zip(chain_names, cd)) + f" total={t[15] - t[8]}", flush=True)
