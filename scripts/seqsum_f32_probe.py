#!/usr/bin/env python3
"""Diagnostic: lo_seq_sum_f32 (the large-scan exact path's column sums) on one synthetic 1M-term column, repeated;
run under `rocprofv3 --kernel-trace --stats` for the split between chunk sums, drift, classification and walk."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from lidar_odometry_amd import IterativeClosestPointOptimizer, lib
    rng = np.random.default_rng(5)
    cases = {"products": (rng.normal(0, 1, 1_000_000) * rng.normal(0, 1, 1_000_000) * 0.01).astype(np.float32),
             "positive": (np.abs(rng.normal(0, 1, 1_000_000)) ** 2).astype(np.float32)}
    o = IterativeClosestPointOptimizer(max_points=1 << 14)
    for name, x in cases.items():
        for _ in range(5):
            out = C.c_float(0.0)
            st = (C.c_longlong * 4)()
            assert lib().lo_seq_sum_f32(o.ctx, x.ctypes.data_as(C.POINTER(C.c_float)), len(x), C.byref(out), st) == 0
        print(name, "heads / term-by-term segments / term-by-term chunks / us:", list(st), flush=True)
    o.close()


if __name__ == "__main__":
    main()
