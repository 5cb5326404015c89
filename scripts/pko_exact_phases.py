#!/usr/bin/env python3
"""Diagnostic: in the running GN loop of the bench's KITTI scans (reference-exact and default mode), the lead PKO
workgroup's phase clock (prefix .. JS, s_memtime) against candidate 0's workgroup (its 43 sums + solve), from the
-DLO_PKO_STAMPS library (make -C lidar_odometry_amd/csrc diag).  Stamps are of each scan's last PKO launch."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LO_ICP_LIB"] = os.environ.get("LO_DIAG_LIB", os.path.join(ROOT, "lidar_odometry_amd", "liblo_icp_diag.so"))
sys.path.insert(0, ROOT)


def main():
    import bench
    from lidar_odometry_amd import lib
    from lidar_odometry_amd.icp import AdaptiveMEstimatorConfig, ICPConfig, IterativeClosestPointOptimizer, MapGeometry
    wl = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "kitti"](0)
    icp = IterativeClosestPointOptimizer(ICPConfig(), AdaptiveMEstimatorConfig(), MapGeometry(voxel_size=wl["voxel"]),
                                         device=0, max_points=max(len(s) for s in wl["scans"]))
    L = lib()
    assert L.lo_map_set_from_voxelmap(icp.ctx, wl["vm"].handle) == 0
    L.lo_set_pipeline(icp.ctx, 0, 2)
    for mode in ("default", "exact"):
        icp.set_exact(mode == "exact")
        lead, cand, sums = [], [], []
        acc = np.zeros(24)
        prev = None
        for i in range(len(wl["scans"])):
            icp.optimize(None, wl["scans"][i], bench.pose12(wl["inits"][i]))
            d = (C.c_ulonglong * 16)()
            assert L.lo_debug_counters(icp.ctx, d) == 0
            lead.append(d[6] - d[0])
            cand.append(d[7])
            sums.append(d[15])
            d2 = (C.c_ulonglong * 24)()
            assert L.lo_debug_counters_ex(icp.ctx, d2, 24) == 0
            cur = np.array(list(d2), dtype=np.float64)
            if prev is not None and mode == "exact":
                acc += cur - prev
            prev = cur
        print(f"{mode}: lead PKO workgroup prefix..JS {np.mean(lead):.0f} cycles, candidate 0 {np.mean(cand):.0f} "
              f"cycles, slowest candidate's sums done at {np.mean(sums):.0f} (exact mode; mean over {len(lead)} scans' last launch)",
              flush=True)
        if mode == "exact" and acc[16] > 0:
            k = acc[16]
            print(f"  exact_sums_wg per call ({k:.0f} calls): consumer adds {acc[17] / k:.0f} + barrier {acc[18] / k:.0f} "
                  f"cycles; producer wave 1 terms {acc[19] / k:.0f} + barrier {acc[20] / k:.0f}", flush=True)
    icp.close()


if __name__ == "__main__":
    main()
