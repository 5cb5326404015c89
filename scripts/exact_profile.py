#!/usr/bin/env python3
"""Diagnostic: time reference-exact mode (lo_set_exact) on a bench workload, scans enqueued back to back.

    python scripts/exact_profile.py [--config kitti|mid360|patch1m] [--steps K] [--mode exact|default]

Run under `rocprofv3 --kernel-trace --stats -- python scripts/exact_profile.py ...` for the per-kernel split.
"""
import argparse
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="kitti")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--mode", default="exact", choices=["exact", "default"])
    a = ap.parse_args()
    import torch

    import bench
    from lidar_odometry_amd import lib
    from lidar_odometry_amd.icp import AdaptiveMEstimatorConfig, ICPConfig, IterativeClosestPointOptimizer, MapGeometry
    wl = bench.WORKLOADS[a.config](0)
    max_pts = max(len(s) for s in wl["scans"])
    icp = IterativeClosestPointOptimizer(ICPConfig(), AdaptiveMEstimatorConfig(), MapGeometry(voxel_size=wl["voxel"]),
                                         device=0, max_points=max_pts)
    L = lib()
    assert L.lo_map_set_from_voxelmap(icp.ctx, wl["vm"].handle) == 0
    icp.set_exact(a.mode == "exact")
    dev = torch.device("cuda", 0)
    d_scans = [torch.from_numpy(s).to(dev) for s in wl["scans"]]
    inits = [bench.pose12(T) for T in wl["inits"]]
    fptr = lambda x: x.ctypes.data_as(C.POINTER(C.c_float))   # noqa: E731
    iters = []
    for i in range(len(d_scans)):
        icp.optimize(None, wl["scans"][i], inits[i])
        iters.append(icp.get_last_stats().num_iterations)

    def step(k):
        i = k % len(d_scans)
        rc = L.lo_icp_optimize_async(icp.ctx, C.c_void_p(d_scans[i].data_ptr()), d_scans[i].shape[0], fptr(inits[i]))
        assert rc == 0, rc
    for k in range(10):
        step(k)
    L.lo_sync(icp.ctx)
    em = (C.c_ulonglong * 3)()
    L.lo_set_stage_timing(icp.ctx, 1)                          # (also clocks the lead PKO workgroup's EM)
    L.lo_pko_em_stats(icp.ctx, em, 1)                          # zero the lead workgroup's EM clock sums
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(k)
    L.lo_sync(icp.ctx)
    el = time.perf_counter() - t0
    L.lo_pko_em_stats(icp.ctx, em, 0)
    print(f"{a.config} {a.mode}: {a.steps / el:.1f} scans/s, {el / a.steps * 1e6:.1f} us/scan, "
          f"{np.mean(iters):.2f} GN iters/scan, {np.mean([len(s) for s in wl['scans']]):.0f} pts/scan | EM of the lead "
          f"PKO workgroup: {em[0] / max(em[1], 1):.0f} cycles per EM iteration, {em[1] / max(em[2], 1):.1f} "
          f"iterations per fit, {em[2]} fits", flush=True)
    icp.close()


if __name__ == "__main__":
    main()
