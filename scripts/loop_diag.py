"""Per-pair breakdown of the loop-closure ICP (bench.py --config kitti_loop pairs): cloud sizes, GN iterations,
wall vs device time per solve and the last iteration's unresolved-query count (queries k_knn could not certify
and k_knn_brute answered).  Diagnostic only; writes gpurun_out/loop_diag.json."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from lidar_odometry_amd import _lib, synth  # noqa: E402
from lidar_odometry_amd.icp import IterativeClosestPointOptimizer  # noqa: E402


def pose12(T):
    return np.asarray(T, np.float32)[:3, :4].reshape(12)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "exact"
    seq = synth.KittiLikeSequence(seed=7, n_frames=42)
    rng = np.random.default_rng(900)
    pairs = []
    for fa in range(0, 36, 3):
        fb = fa + 3 + (fa // 3) % 2
        cur = oracle.voxel_filter(seq.scan(fb), 0.5, 8)
        mat = oracle.voxel_filter(seq.scan(fa), 0.5, 8)
        pairs.append((cur, pose12(synth.perturb(seq.poses[fb], rng, 0.3, 0.03)), mat, pose12(seq.poses[fa])))
    icp = IterativeClosestPointOptimizer(device=0, max_points=max(len(p[0]) for p in pairs))
    icp.set_exact(mode == "exact")
    out = []
    try:
        for pr in pairs * 2:
            icp.optimize_loop(*pr)
        for pr in pairs:
            reps = 20
            t0 = time.perf_counter()
            for _ in range(reps):
                icp.optimize_loop(*pr)
            wall = (time.perf_counter() - t0) / reps * 1e3
            st = icp.get_last_stats()
            dbg = (C.c_ulonglong * 16)()
            _lib.lib().lo_debug_counters(icp._ctx, dbg)
            out.append({"n_curr": len(pr[0]), "n_matched": len(pr[2]), "iters": st.num_iterations,
                        "wall_ms": wall, "gpu_ms": st.optimization_time_ms, "unresolved_last": int(dbg[15]),
                        "n_corr": [it["n_corr"] for it in st.iterations]})
    finally:
        icp.close()
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/loop_diag_{mode}.json", "w") as f:
        json.dump(out, f, indent=1)
    for r in out:
        print(r["n_curr"], r["n_matched"], r["iters"], f"{r['wall_ms']:.3f} {r['gpu_ms']:.3f}", r["unresolved_last"])


if __name__ == "__main__":
    main()
