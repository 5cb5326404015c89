"""The lookahead launches (lo_lookahead.hip: two GN iterations per launch, every alpha candidate's next iteration --
its PKO included -- run speculatively) against the one-iteration-at-a-time path on the same context: identical
iteration count, status, and bit-identical per-iteration logs (pose, n_corr, scale, alpha, cost, H, g, delta).
The one-iteration path is itself held to the oracle by test_gpu_parity.py, so this pins the lookahead to it.
"""
import numpy as np
import pytest

from tests import _data

pytestmark = pytest.mark.gpu


def _run(o, pts, Ti, lookahead):
    o.set_lookahead(lookahead)
    ok, To = o.optimize(None, pts, Ti)
    st = o.get_last_stats()
    return ok, np.asarray(To, np.float32).reshape(12).copy(), st


def _same(a, b):
    ok_a, T_a, st_a = a
    ok_b, T_b, st_b = b
    assert ok_a == ok_b
    assert st_a.num_iterations == st_b.num_iterations
    assert st_a.num_correspondences == st_b.num_correspondences
    np.testing.assert_array_equal(T_a, T_b)
    for k, (la, lb) in enumerate(zip(st_a.iterations, st_b.iterations)):
        for key in ("pose", "n_corr", "scale", "alpha", "cost", "H", "g", "delta"):
            np.testing.assert_array_equal(np.asarray(la[key]), np.asarray(lb[key]), err_msg=f"iter {k} {key}")


def _ctx(max_iters=4, tol=0.005, voxel=0.5):
    from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer, MapGeometry
    cfg = ICPConfig(max_iterations=max_iters, translation_tolerance=tol, rotation_tolerance=tol)
    return IterativeClosestPointOptimizer(cfg, geometry=MapGeometry(voxel_size=voxel), max_points=1 << 16)


@pytest.mark.parametrize("frame", [11, 13, 17, 21, 25, 31])
def test_lookahead_kitti_bitwise(frame):
    m, pts, Ti, _ = _data.kitti_case(frame)
    o = _ctx()
    try:
        k, n, c = _data.surfels(m)
        o.set_surfels(k, n, c)
        _same(_run(o, pts, Ti, True), _run(o, pts, Ti, False))
    finally:
        o.close()


@pytest.mark.parametrize("max_iters", [1, 2, 3, 5, 6])
def test_lookahead_launch_counts_bitwise(max_iters):
    """Odd / even max_iterations and tolerance 1e-9 (every iteration runs): the last launch's chains stop after one
    iteration (odd) or run both; k_la_finish publishes the last record."""
    m, pts, Ti, _ = _data.kitti_case(13)
    o = _ctx(max_iters=max_iters, tol=1e-9)
    try:
        k, n, c = _data.surfels(m)
        o.set_surfels(k, n, c)
        a = _run(o, pts, Ti, True)
        assert a[2].num_iterations == max_iters
        _same(a, _run(o, pts, Ti, False))
    finally:
        o.close()


def test_lookahead_mid360_bitwise():
    m, pts, Ti, _ = _data.mid360_case()
    o = _ctx(voxel=0.4)
    try:
        k, n, c = _data.surfels(m)
        o.set_surfels(k, n, c)
        _same(_run(o, pts, Ti, True), _run(o, pts, Ti, False))
    finally:
        o.close()


def test_lookahead_large_perturbation_and_back_to_back():
    """A large initial error (4 iterations) and scans queued back to back on one context (the double-buffered
    records / correspondence sets of one scan must not leak into the next)."""
    cases = [_data.kitti_case(15, seed=5, sigma_t=0.3, sigma_r=0.03), _data.kitti_case(11), _data.kitti_case(21)]
    o = _ctx()
    try:
        k, n, c = _data.surfels(cases[0][0])
        o.set_surfels(k, n, c)
        la = [_run(o, pts, Ti, True) for (_, pts, Ti, _) in cases]
        one = [_run(o, pts, Ti, False) for (_, pts, Ti, _) in cases]
        for a, b in zip(la, one):
            _same(a, b)
    finally:
        o.close()


def test_lookahead_insufficient():
    m, pts, Ti, _ = _data.kitti_case(11)
    o = _ctx()
    try:
        k, n, c = _data.surfels(m)
        o.set_surfels(k, n, c)
        far = pts + np.float32(5000.0)
        a, b = _run(o, far, Ti, True), _run(o, far, Ti, False)
        assert not a[0] and not b[0]
        np.testing.assert_array_equal(a[1], Ti.reshape(12))
        _same(a, b)
        # a scan whose points leave the map after the first update: few correspondences in a later iteration
        sub = pts[:40]
        _same(_run(o, sub, Ti, True), _run(o, sub, Ti, False))
    finally:
        o.close()
