#!/usr/bin/env python3
"""Diagnostic: phase clocks of the reference-exact iteration-0 scale kernel (liblo_icp_diagx.so, -DLO_EXACT_STAMPS).

    LO_ICP_LIB=lidar_odometry_amd/liblo_icp_diagx.so python scripts/exact_stamps.py [--config kitti]

Prints s_memtime deltas: load + count | sort | mean sum | variance sum, per scan of the bench workload.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="kitti")
    a = ap.parse_args()
    import bench
    from lidar_odometry_amd import lib
    from lidar_odometry_amd.icp import AdaptiveMEstimatorConfig, ICPConfig, IterativeClosestPointOptimizer, MapGeometry
    wl = bench.WORKLOADS[a.config](0)
    icp = IterativeClosestPointOptimizer(ICPConfig(), AdaptiveMEstimatorConfig(), MapGeometry(voxel_size=wl["voxel"]),
                                         device=0, max_points=max(len(s) for s in wl["scans"]))
    L = lib()
    assert L.lo_map_set_from_voxelmap(icp.ctx, wl["vm"].handle) == 0
    icp.set_exact(True)
    rows, stats, mrows = [], [], []
    for i in range(len(wl["scans"])):
        icp.optimize(None, wl["scans"][i], bench.pose12(wl["inits"][i]))
        d = (C.c_ulonglong * 24)()
        assert L.lo_debug_counters_ex(icp.ctx, d, 24) == 0
        if len(wl["scans"][i]) > 16384:                      # large scan: k_exact_sum43 walk statistics (cumulative)
            it = icp.get_last_stats().num_iterations
            print("scan %d: %d pts, %d iterations | sum43 cumulative: %d heads, %d segments term by term, %d chained "
                  "chunks | scale sums: %d / %d heads, %d / %d segments (%d / %d terms) term by term | mean walk %d cycles, "
                  "%d in its unrolled 64-head chains" % (i, len(wl["scans"][i]), it, d[15], d[13], d[12], d[5], d[8], d[6],
                                                         d[9], d[7], d[10], d[11], d[14]), flush=True)
            if d[21]:
                print("  sum43 walk cycles (cumulative, %d column walks): mean %.0f, slowest column %d | chained chunks "
                      "%.0f, failed segments %.0f, head-by-head rest %.0f per column walk" %
                      (d[21], d[16] / d[21], d[17], d[18] / d[21], d[19] / d[21], d[20] / d[21]), flush=True)
            continue
        if len(wl["scans"][i]) <= 8192:                       # one-launch path (k_exact_scale_c): 0 start, 12 sorted,
            mrows.append([d[12] - d[0], d[1] - d[12], d[4] - d[1], d[5] - d[4], d[6] - d[5], d[2] - d[6],   # 1 terms,
                          d[8] - d[2], d[9] - d[8], d[10] - d[9], d[3] - d[10],                            # 2 / 3 sums
                          d[13] - d[0], d[14] - d[13], d[15] - d[14], d[12] - d[15]])   # the sort's parts
            continue
        rows.append([d[1] - d[0], d[2] - d[1], d[3] - d[2], d[4] - d[3], d[6] - d[5], d[7] - d[6]])
        stats.append([d[14], d[8], d[9], d[10], d[11], d[12], d[13]])
    if mrows:
        m = np.array(mrows, dtype=np.float64)
        print("one-launch exact scale, cycles per phase, mean over %d scans: counting sort %.0f  terms %.0f | mean sum: "
              "heads + xor scan %.0f  increments scan %.0f  records %.0f  walk %.0f | variance sum: heads + xor scan "
              "%.0f  increments scan %.0f  records %.0f  walk %.0f | sort: loads + key stats %.0f  histogram + scan + "
              "scatter %.0f  rank in bin %.0f  write back %.0f" % (len(mrows), *m.mean(0)), flush=True)
    if not rows:
        for k, t in enumerate(stats):
            print("scan %d: %d accepted | mean sum: %d heads, %d segments / %d terms term by term | variance: %d heads, "
                  "%d / %d" % (k, *t), flush=True)
        icp.close()
        return
    r = np.array(rows, dtype=np.float64)
    print("cycles (s_memtime) per phase, mean over", len(rows), "scans: scale load/count %.0f  store %.0f  mean-sum "
          "%.0f  var-sum %.0f | rank-sort WG 0: staging %.0f  compares %.0f" % tuple(r.mean(0)), flush=True)
    for k, t in enumerate(stats):
        print("scan %d: %d accepted | mean sum: %d heads, %d segments / %d terms term by term | variance: %d heads, "
              "%d / %d" % (k, *t), flush=True)
    icp.close()


if __name__ == "__main__":
    main()
