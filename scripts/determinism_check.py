#!/usr/bin/env python3
"""Diagnostic: the same KITTI-like scans through lo_icp_optimize (host buffers) and lo_icp_optimize_async (device
buffers + lo_icp_export_pose), repeated, must give bit-identical poses and iteration counts.

    python scripts/determinism_check.py [rank ...]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from lidar_odometry_amd import lib
    from lidar_odometry_amd.icp import IterativeClosestPointOptimizer
    ranks = [int(a) for a in sys.argv[1:]] or [0, 1]
    dev = torch.device("cuda", 0)
    L = lib()
    fptr = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))   # noqa: E731
    bad = 0
    for r in ranks:
        wl = bench.build_kitti(r)
        icp = IterativeClosestPointOptimizer(device=0, max_points=max(len(s) for s in wl["scans"]))
        assert L.lo_map_set_from_voxelmap(icp.ctx, wl["vm"].handle) == 0
        inits = [bench.pose12(T) for T in wl["inits"]]
        d_scans = [torch.from_numpy(s).to(dev) for s in wl["scans"]]
        torch.cuda.synchronize()
        ref = []
        for i in range(len(d_scans)):
            ok, To = icp.optimize(None, wl["scans"][i], inits[i])
            ref.append((np.asarray(To, np.float32).reshape(12).copy(), icp.get_last_stats().num_iterations))
        rec = torch.zeros(16, dtype=torch.float32, device=dev)
        for rep in range(3):
            for i in range(len(d_scans)):
                assert L.lo_icp_optimize_async(icp.ctx, C.c_void_p(d_scans[i].data_ptr()), d_scans[i].shape[0],
                                               fptr(inits[i])) == 0
                L.lo_icp_export_pose(icp.ctx, C.c_void_p(rec.data_ptr()))
                L.lo_sync(icp.ctx)
                g = rec.cpu().numpy()
                T0, it0 = ref[i]
                if int(g[13]) != it0 or not np.array_equal(g[:12], T0):
                    bad += 1
                    print(f"rank {r} rep {rep} scan {i}: iters {int(g[13])} vs {it0}, "
                          f"max|dT| {np.abs(g[:12] - T0).max():.3e}", flush=True)
                ok, To = icp.optimize(None, wl["scans"][i], inits[i])
                it1 = icp.get_last_stats().num_iterations
                if it1 != it0 or not np.array_equal(np.asarray(To, np.float32).reshape(12), T0):
                    bad += 1
                    print(f"rank {r} rep {rep} scan {i}: host path repeat differs: iters {it1} vs {it0}", flush=True)
        print(f"rank {r}: iterations {[x[1] for x in ref]}", flush=True)
        icp.close()
    print("mismatches:", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
