#!/usr/bin/env python3
"""Diagnostic (r06): which part bounds a reference-exact PKO launch -- the lead workgroup's GMM fit + JS, or the
exact candidates' 43 sums + fp32 solve.  From the -DLO_PKO_STAMPS library (make -C lidar_odometry_amd/csrc diag), all
on the chip-wide s_memrealtime clock (100 MHz) relative to the lead workgroup's start: dbg[22] lead JS end, dbg[15]
the last candidate's sums end, dbg[23] the last candidate's record end.  Stamps are of each scan's last working PKO
launch; the scan pipeline is off so every launch is on one stream."""
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
    icp.set_exact(True)
    rows = []
    for rep in range(2):
        for i in range(len(wl["scans"])):
            icp.optimize(None, wl["scans"][i], bench.pose12(wl["inits"][i]))
            d = (C.c_ulonglong * 24)()
            assert L.lo_debug_counters_ex(icp.ctx, d, 24) == 0
            t0 = d[21]
            if rep == 1 and t0:
                rows.append(((d[22] - t0) / 100.0, (d[15] - t0) / 100.0, (d[23] - t0) / 100.0, d[7], d[8], d[9]))
    a = np.array(rows)
    print(f"exact PKO launch (last working launch of {len(a)} scans), us from the lead workgroup's start:")
    print(f"  lead fit + JS end     mean {a[:, 0].mean():.1f}  median {np.median(a[:, 0]):.1f}  max {a[:, 0].max():.1f}")
    print(f"  candidates' sums end  mean {a[:, 1].mean():.1f}  median {np.median(a[:, 1]):.1f}  max {a[:, 1].max():.1f}")
    print(f"  candidates' records   mean {a[:, 2].mean():.1f}  median {np.median(a[:, 2]):.1f}  max {a[:, 2].max():.1f}")
    print(f"  candidate 0 cycles    mean {a[:, 3].mean():.0f}")
    print(f"  candidate 0's solve   mean {a[:, 4].mean():.0f} cycles = {a[:, 5].mean() / 100.0:.1f} us "
          f"(shader clock {a[:, 4].sum() / a[:, 5].sum() / 10.0:.2f} GHz)")
    print(f"  every candidate's solve: mean {d[17] / max(d[18], 1):.0f} cycles over {d[18]} solves, largest {d[16]} cycles")
    print(f"  the same solve again (code cached): mean {d[20] / max(d[18], 1):.0f} cycles, largest {d[19]} cycles")
    print(f"  launches bound by the candidates: {int((a[:, 2] > a[:, 0]).sum())} of {len(a)}")
    for r in rows:
        print("   " + " ".join(f"{v:8.1f}" for v in r[:3]))
    icp.close()


if __name__ == "__main__":
    main()
