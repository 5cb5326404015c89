"""Diagnostic: the KDTree correspondence stage on KITTI-like scans -- how many queries the grid search leaves to
the brute-force pass (lo_debug_counters slot 15, written by k_plane) and the isolated stage time
(lo_bench_kernel kernel 0 = k_knn + k_knn_brute + k_plane)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer, lib  # noqa: E402
from tests import _data  # noqa: E402

icp = IterativeClosestPointOptimizer(config=ICPConfig(use_surfel_correspondence=False), max_points=1 << 16)
for f in (11, 13, 17, 21, 25, 31):
    m, pts, Ti, _ = _data.kitti_case(f)
    icp.set_map_points(m.l0_cloud())
    icp.optimize(None, pts, Ti)
    it0 = icp.get_last_stats().iterations[0]
    d = torch.from_numpy(pts).cuda()
    ms = C.c_float(0.0)
    rc = lib().lo_bench_kernel(icp.ctx, C.c_void_p(d.data_ptr()), len(pts), Ti.ctypes.data_as(C.POINTER(C.c_float)),
                               C.c_double(it0["scale"]), C.c_double(it0["alpha"]), 0, 50, C.byref(ms))
    assert rc == 0, rc
    out = (C.c_ulonglong * 16)()
    lib().lo_debug_counters(icp.ctx, out)
    print(f"frame {f}: n={len(pts)} map={m.l0_count()} unresolved={out[15]} stage={ms.value * 1e3:.1f} us", flush=True)
icp.close()
