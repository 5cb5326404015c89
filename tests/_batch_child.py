"""Child process of tests/test_gpu_batch.py::test_batch_only_exact_in_fresh_process (test infrastructure).

A fresh process whose FIRST exact work is a lockstep batch (no single-context exact optimize before it, so nothing
else has set the exact-scale kernels' dynamic-LDS attribute): reference-exact jobs of 4096 < n <= 8192 points run
k_exact_scale_cb with its largest sort width.  Prints one JSON line: whether every batch record equals the same
context's own lo_icp_optimize afterwards, bit for bit, and the job sizes."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.zeros(1, device="cuda")
    from lidar_odometry_amd import BatchOptimizer
    from tests import _data
    from tests.test_gpu_batch import _ctx, _singles
    jobs = []
    for f in (11, 13, 17):
        m, pts, Ti, _ = _data.kitti_case(f)
        big = np.concatenate([pts, pts[: 6000 - len(pts)] + np.float32(0.013)]) if len(pts) < 6000 else pts
        jobs.append((m, 0.5, big.astype(np.float32), Ti))
    ctxs = [_ctx(m, v, exact=True) for (m, v, _, _) in jobs]
    try:
        b = BatchOptimizer(ctxs)
        try:
            res = b.optimize(None, [j[2] for j in jobs], [j[3] for j in jobs])
        finally:
            b.close()
        singles = _singles(ctxs, jobs)
        equal = []
        for r, s in zip(res, singles):
            ok, To, it, nc, _ = s
            same = r.success == ok and np.array_equal(np.asarray(r.pose, np.float32).reshape(12).view(np.uint32),
                                                      np.asarray(To, np.float32).view(np.uint32))
            equal.append(bool(same and (not ok or (r.iterations == it and r.n_corr == nc))))
    finally:
        for o in ctxs:
            o.close()
    print(json.dumps({"equal": equal, "n": [len(j[2]) for j in jobs]}))


if __name__ == "__main__":
    main()
