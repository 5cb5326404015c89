#!/usr/bin/env python3
"""Same-box sweep of the PKO launch's EM workgroup count (lo_set_pko_groups): single-stream and 8-sequence
aggregate scans/s on the bench's KITTI workload, in both arithmetic modes; results checked identical for every G.

    python scripts/pko_groups_sweep.py [--groups 0,50,25,10,4] [--sequences 8] [--steps 600]
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
    ap.add_argument("--groups", default="0,50,25,10,4")
    ap.add_argument("--sequences", type=int, default=8)
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--modes", default="default,exact")
    ap.add_argument("--pipe", type=int, default=1, help="scan pipeline on (1) / off (0) in every context")
    a = ap.parse_args()
    import torch

    import bench
    from lidar_odometry_amd import lib
    from lidar_odometry_amd.icp import IterativeClosestPointOptimizer
    wl = bench.WORKLOADS["kitti"](0)
    L = lib()
    mp = max(len(s) for s in wl["scans"])
    ctxs = [IterativeClosestPointOptimizer(device=0, max_points=mp) for _ in range(a.sequences)]
    for o in ctxs:
        assert L.lo_map_set_from_voxelmap(o.ctx, wl["vm"].handle) == 0
    dev = torch.device("cuda", 0)
    d_scans = [torch.from_numpy(s).to(dev) for s in wl["scans"]]
    inits = [bench.pose12(T) for T in wl["inits"]]
    fptr = lambda x: x.ctypes.data_as(C.POINTER(C.c_float))   # noqa: E731

    def enq(o, k):
        i = k % len(d_scans)
        assert L.lo_icp_optimize_async(o.ctx, C.c_void_p(d_scans[i].data_ptr()), d_scans[i].shape[0], fptr(inits[i])) == 0

    ref = {}
    for mode in a.modes.split(","):
        for G in [int(g) for g in a.groups.split(",")]:
            for o in ctxs:
                o.set_exact(mode == "exact")
                o.set_pipeline(bool(a.pipe))
                assert L.lo_set_pko_groups(o.ctx, G) == 0
            res = []
            for i in range(len(d_scans)):
                ok, To = ctxs[0].optimize(None, wl["scans"][i], inits[i])
                res.append(np.asarray(To, np.float32).tobytes())
            same = ref.setdefault(mode, res) == res
            o = ctxs[0]
            for k in range(20):
                enq(o, k)
            L.lo_sync(o.ctx)
            t0 = time.perf_counter()
            for k in range(a.steps):
                enq(o, k)
            L.lo_sync(o.ctx)
            single = a.steps / (time.perf_counter() - t0)
            K = max(50, a.steps // 2)
            for k in range(10):
                for b, o in enumerate(ctxs):
                    enq(o, k + 7 * b)
            for o in ctxs:
                L.lo_sync(o.ctx)
            t1 = time.perf_counter()
            for k in range(K):
                for b, o in enumerate(ctxs):
                    enq(o, k + 7 * b)
            for o in ctxs:
                L.lo_sync(o.ctx)
            multi = a.sequences * K / (time.perf_counter() - t1)
            print(f"hwq={os.environ.get('GPU_MAX_HW_QUEUES', 'default')} pipe={a.pipe} {mode:8s} G={G:3d}: single {single:8.1f} scans/s, {a.sequences} sequences {multi:9.1f} scans/s "
                  f"({multi / single:.2f}x), results identical to G={a.groups.split(',')[0]}: {same}", flush=True)
    for o in ctxs:
        o.close()


if __name__ == "__main__":
    main()
