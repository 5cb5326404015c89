"""Loop-closure ICP restatement (optimize_loop, IterativeClosestPointOptimizer.cpp:40-251) on
the CPU: it recovers a drifted keyframe pose against an earlier keyframe, the kd-tree and the index-ordered brute
force give identical results, and the failure paths return the reference's false.  No reference binary exists for
this path (Eigen is absent), so the restatement is checked by its behaviour here and by the GPU parity tests."""
import numpy as np

import oracle
from tests import _data


def _compose(T12a, T12b):
    A = np.eye(4); A[:3] = np.asarray(T12a, np.float64).reshape(3, 4)
    B = np.eye(4); B[:3] = np.asarray(T12b, np.float64).reshape(3, 4)
    return A @ B


def test_loop_recovers_drifted_pose():
    cur, Tc, mat, Tm, Tgt = _data.loop_case(2, 6)
    ok, conv, Tr, inl, iters, logs = oracle.icp_optimize_loop(cur, Tc, mat, Tm)
    assert ok and conv and 1 <= iters <= 100
    assert inl > 0.5
    est = _compose(Tc, Tr)
    gt = np.asarray(Tgt, np.float64).reshape(3, 4)
    assert np.linalg.norm(est[:3, 3] - gt[:, 3]) < 0.05          # 0.3 m / 0.03 rad drift removed to a few cm
    assert len(logs) == iters and all(L["n_corr"] >= 10 for L in logs)


def test_loop_tree_equals_brute_force():
    cur, Tc, mat, Tm, _ = _data.loop_case(4, 7, seed=3)
    a = oracle.icp_optimize_loop(cur, Tc, mat, Tm)
    oracle.set_kdtree_search(False)
    try:
        b = oracle.icp_optimize_loop(cur, Tc, mat, Tm)
    finally:
        oracle.set_kdtree_search(True)
    assert a[:2] == b[:2] and a[4] == b[4] and a[3] == b[3]
    np.testing.assert_array_equal(a[2], b[2])


def test_loop_failure_paths():
    cur, Tc, mat, Tm, _ = _data.loop_case(2, 6)
    # fewer than 5 matched points: no 5-NN anywhere -> insufficient correspondences at iteration 0
    ok, conv, Tr, inl, iters, _ = oracle.icp_optimize_loop(cur, Tc, mat[:4], Tm)
    assert not ok and not conv and Tr is None and inl is None and iters == 0
    ok, conv, *_ = oracle.icp_optimize_loop(cur[:0], Tc, mat, Tm)
    assert not ok and not conv
    # a far-away matched keyframe: correspondences exist (no distance gate) but the inlier test rejects it
    far = np.asarray(Tm, np.float32).copy()
    far[3] += 500.0
    ok, conv, Tr, inl, iters, _ = oracle.icp_optimize_loop(cur, Tc, mat, far)
    assert not ok
    assert (not conv) or inl < 0.5
