"""Diagnostic: phase timing of the batched PKO (k_pko_tb) from the -DLO_PKO_STAMPS library: B contexts on the
KITTI-like frames, one lo_batch optimize, then job 0's lead-workgroup stamps (s_memtime) of each launch's
last PKO.  Usage: python scripts/pko_phases_batch.py [B ...]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LO_ICP_LIB"] = os.environ.get("LO_DIAG_LIB", os.path.join(ROOT, "lidar_odometry_amd", "liblo_icp_diag.so"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from lidar_odometry_amd import BatchOptimizer, IterativeClosestPointOptimizer, lib  # noqa: E402
from lidar_odometry_amd._lib import LoBatchRec  # noqa: E402
from tests import _data  # noqa: E402

torch.zeros(1, device="cuda")
names = ["prefix", "sample", "kmeans", "initvar", "EM", "JS"]
frames = (11, 13, 17, 21, 25, 31)
cases = [_data.kitti_case(f) for f in frames]
for B in [int(a) for a in sys.argv[1:]] or [64, 1024]:
    ctxs = []
    for j in range(B):
        m, pts, Ti, _ = cases[j % len(cases)]
        o = IterativeClosestPointOptimizer(max_points=1 << 13)
        k, n, c = _data.surfels(m)
        o.set_surfels(k, n, c)
        ctxs.append(o)
    bo = BatchOptimizer(ctxs)
    scans = [torch.from_numpy(cases[j % len(cases)][1]).cuda() for j in range(B)]
    ptrs = (C.c_void_p * B)(*[t.data_ptr() for t in scans])
    cnts = (C.c_size_t * B)(*[t.shape[0] for t in scans])
    T = np.ascontiguousarray(np.stack([cases[j % len(cases)][2] for j in range(B)]), np.float32)
    recs = (LoBatchRec * B)()
    ms = C.c_double(0.0)
    L = lib()
    for _ in range(3):
        assert L.lo_batch_optimize_async(bo._b, ptrs, cnts, T.ctypes.data_as(C.POINTER(C.c_float))) == 0
        assert L.lo_batch_result(bo._b, recs, C.byref(ms)) == 0
    out = (C.c_ulonglong * 16)()
    L.lo_debug_counters(ctxs[0].ctx, out)
    t = [out[i] for i in range(7)]
    dt = np.array([t[i + 1] - t[i] for i in range(6)], dtype=np.float64)
    print(f"B={B}: batch {ms.value:.3f} ms, job 0 last PKO: em_iters={out[8]} km_iters={out[9]} "
          + " ".join(f"{nm}={int(v)}" for nm, v in zip(names, dt)) + f" total={t[6] - t[0]} cyc", flush=True)
    tot, em = [], []
    for o in ctxs:
        L.lo_debug_counters(o.ctx, out)
        tot.append(out[6] - out[0])
        em.append(out[8])
    tot, em = np.array(tot, dtype=np.float64), np.array(em)
    print(f"  all jobs: total cyc mean {tot.mean():.0f} max {tot.max():.0f}; em_iters per case "
          + " ".join(str(int(e)) for e in em[:len(cases)]) + f"; em max {em.max()}", flush=True)
    bo.close()
    for o in ctxs:
        o.close()
