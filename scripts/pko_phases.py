"""Diagnostic: phase timing of k_pko on real ICP iterations (KITTI-like scans), from the -DLO_PKO_STAMPS
library (make -C lidar_odometry_amd/csrc diag).  For each scan: one optimize() for its iteration-0 scale/alpha,
then lo_bench_kernel(k_pko) launches at the initial pose; prints s_memtime deltas (cycles) per phase of the
lead workgroup, EM / k-means iteration counts and the isolated launch time."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LO_ICP_LIB"] = os.environ.get("LO_DIAG_LIB", os.path.join(ROOT, "lidar_odometry_amd", "liblo_icp_diag.so"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from lidar_odometry_amd import IterativeClosestPointOptimizer, lib  # noqa: E402
from tests import _data  # noqa: E402

icp = IterativeClosestPointOptimizer(max_points=1 << 17)
names = ["prefix", "sample", "kmeans", "initvar", "EM", "JS"]
tot = np.zeros(6)
for f in (11, 13, 17, 21, 25, 31):
    m, pts, Ti, _ = _data.kitti_case(f)
    k, n, c = _data.surfels(m)
    icp.set_surfels(k, n, c)
    icp.optimize(None, pts, Ti)
    it0 = icp.get_last_stats().iterations[0]
    d = torch.from_numpy(pts).cuda()
    ms = C.c_float(0.0)
    rc = lib().lo_bench_kernel(icp.ctx, C.c_void_p(d.data_ptr()), len(pts), Ti.ctypes.data_as(C.POINTER(C.c_float)),
                               C.c_double(it0["scale"]), C.c_double(it0["alpha"]), 2, 20, C.byref(ms))
    assert rc == 0, rc
    out = (C.c_ulonglong * 16)()
    lib().lo_debug_counters(icp.ctx, out)
    t = [out[i] for i in range(7)]
    dt = np.array([t[i + 1] - t[i] for i in range(6)], dtype=np.float64)
    tot += dt
    print(f"frame {f}: n={len(pts)} em_iters={out[8]} km_iters={out[9]} launch={ms.value * 1e3:.1f} us "
          + " ".join(f"{nm}={int(v)}" for nm, v in zip(names, dt)) + f" total={t[6] - t[0]} cyc"
          + f" | per EM iter {dt[4] / max(out[8], 1):.0f} cyc"
          + f" | JS: post-EM barrier {out[12] - t[5]} gpdf {out[10] - out[12]} terms {out[11] - out[10]}"
          + f" sum {t[6] - out[11]}"
          + f" | sample: events {out[13] - t[1]} residual {out[14] - out[13]} barrier {t[2] - out[14]}"
          + f" | candidate wg: first {out[7]} slowest {out[15]} cyc", flush=True)
    lib().lo_debug_reset(icp.ctx) if hasattr(lib(), "lo_debug_reset") else None
print("mean share: " + " ".join(f"{nm}={v / tot.sum():.2f}" for nm, v in zip(names, tot)))
