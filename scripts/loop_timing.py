"""Wall time vs device-timeline time of the loop-closure ICP (lo_icp_optimize_loop) on the bench's keyframe pairs:
the difference is host work (matched-cloud grid + kd visit order, uploads, per-chunk syncs)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import torch  # noqa: E402,F401

from tests import _data  # noqa: E402
from lidar_odometry_amd import IterativeClosestPointOptimizer  # noqa: E402

torch.zeros(1, device="cuda")
icp = IterativeClosestPointOptimizer(max_points=1 << 17)
pairs = [_data.loop_case(fa, fa + 3 + (fa % 2), seed=fa) for fa in range(2, 26, 2)]
for rep in range(2):
    wall, dev, iters = [], [], []
    for cur, Tc, mat, Tm, _ in pairs:
        t0 = time.perf_counter()
        icp.optimize_loop(cur, Tc, mat, Tm)
        wall.append(time.perf_counter() - t0)
        st = icp.get_last_stats()
        dev.append(st.optimization_time_ms * 1e-3)
        iters.append(st.num_iterations)
    print(f"rep {rep}: wall {1e3 * np.mean(wall):.3f} ms, device timeline {1e3 * np.mean(dev):.3f} ms, "
          f"GN iterations {np.mean(iters):.2f}")
icp.close()
