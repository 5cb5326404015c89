"""GPU parity of the loop-closure ICP (IterativeClosestPointOptimizer::optimize_loop, IterativeClosestPointOptimizer.cpp
:40-251 with find_correspondences_loop :465-585) against the oracle restatement.

Iteration 0 sees the same pose on both sides, so the exact 5-NN sets, collinearity gates and fp64 plane distances
are identical there: same correspondence count, scale and PKO alpha.  Later iterations start from poses that differ
by ~1e-7 (fp32 H/g sum order), so the bars are the north_star's 1e-4 m / 1e-4 rad per iteration and a handful of
correspondence flips.  The inlier ratio is a count of 1-NN threshold tests at the final pose: equal up to points
within ~1e-7 m of the 1 m threshold.  Only the loop-ICP's success/failure and T_rel are the reference's outputs.
"""
import numpy as np
import pytest

import oracle
from tests import _data

pytestmark = pytest.mark.gpu

TOL_T = 1e-4
TOL_R = 1e-4


@pytest.fixture(scope="module")
def icp():
    from lidar_odometry_amd import IterativeClosestPointOptimizer
    o = IterativeClosestPointOptimizer(max_points=1 << 17)
    yield o
    o.close()


def _pose_err(Ta, Tb):
    A = np.asarray(Ta, np.float64).reshape(3, 4)
    B = np.asarray(Tb, np.float64).reshape(3, 4)
    return float(np.linalg.norm(A[:, 3] - B[:, 3])), _data.rot_angle(A[:, :3], B[:, :3])


def _compare_loop(icp, cur, Tc, mat, Tm):
    ok_o, conv_o, Tr_o, inl_o, it_o, logs_o = oracle.icp_optimize_loop(cur, Tc, mat, Tm)
    ok_g, Tr_g, inl_g = icp.optimize_loop(cur, Tc, mat, Tm)
    st = icp.get_last_stats()
    assert ok_g == ok_o
    assert st.converged == conv_o
    assert st.num_iterations == it_o, f"iterations {st.num_iterations} vs oracle {it_o}"
    flips = 0
    for k, (lo, lg) in enumerate(zip(logs_o, st.iterations)):
        if k == 0:
            assert lg["n_corr"] == lo["n_corr"], f"iter 0: n_corr {lg['n_corr']} vs {lo['n_corr']}"
            assert lg["scale"] == pytest.approx(lo["scale"], rel=1e-12)
            assert lg["alpha"] == lo["alpha"]
        else:
            assert abs(lg["n_corr"] - lo["n_corr"]) <= max(2, 5e-4 * lo["n_corr"])
        et, er = _pose_err(lg["pose"], lo["pose"])
        if lg["alpha"] != lo["alpha"]:
            # PKO's alpha is a discrete argmin over the JS grid: a correspondence flipped by the ~1e-6 pose
            # difference entering this iteration can move it one grid step (measured: pair 20-23, iteration 2,
            # 2585 vs 2584 correspondences, alpha 0.138 vs 0.126, pose 1.4e-4 m apart, re-converged to 1.5e-5 m
            # one iteration later).  Once per solve, never at iteration 0, 1e-3 for that iteration only.
            flips += 1
            assert k > 0 and flips <= 1 and et <= 1e-3 and er <= 1e-3, f"iter {k}: dt {et:.2e} m, dr {er:.2e} rad"
            continue
        assert et <= TOL_T and er <= TOL_R, f"iter {k}: dt {et:.2e} m, dr {er:.2e} rad"
    if conv_o:
        et, er = _pose_err(Tr_g, Tr_o)
        assert et <= TOL_T and er <= TOL_R
        assert abs(inl_g - inl_o) <= 2.0 / len(cur)
    else:
        assert Tr_g is None and inl_g is None
    return ok_g, st


@pytest.mark.parametrize("fa,fb,seed", [(2, 6, 0), (4, 7, 3), (10, 14, 5), (20, 23, 9)])
def test_loop_icp_parity(icp, fa, fb, seed):
    cur, Tc, mat, Tm, Tgt = _data.loop_case(fa, fb, seed)
    ok, st = _compare_loop(icp, cur, Tc, mat, Tm)
    assert ok and st.converged


def test_loop_icp_failure_paths(icp):
    cur, Tc, mat, Tm, _ = _data.loop_case(2, 6)
    ok, Tr, inl = icp.optimize_loop(cur, Tc, mat[:4], Tm)        # no 5-NN anywhere
    assert not ok and Tr is None and inl is None
    ok, Tr, inl = icp.optimize_loop(cur[:0], Tc, mat, Tm)         # empty curr cloud
    assert not ok and Tr is None
    # a matched keyframe 500 m away: correspondences exist (no distance gate) but H is nearly singular, so the
    # reference's fp32 LDLT and the device's fp64 one diverge from the first step; only the outcome (false, no
    # T_rel) is the reference's, and both sides give it
    far = np.asarray(Tm, np.float32).copy()
    far[3] += 500.0
    ok_o, conv_o, *_ = oracle.icp_optimize_loop(cur, Tc, mat, far)
    ok, Tr, inl = icp.optimize_loop(cur, Tc, mat, far)
    assert not ok_o and not ok
    assert (Tr is None) or inl < 0.5


def test_loop_icp_leaves_the_map_alone(icp):
    """The loop ICP grids the matched keyframe separately: the context's surfel map and the next optimize are
    bit-identical before and after."""
    m, pts, Ti, _ = _data.kitti_case(11)
    k, n, c = _data.surfels(m)
    icp.set_surfels(k, n, c)
    _, A = icp.optimize(None, pts, Ti)
    cur, Tc, mat, Tm, _ = _data.loop_case(2, 6)
    icp.optimize_loop(cur, Tc, mat, Tm)
    _, B = icp.optimize(None, pts, Ti)
    np.testing.assert_array_equal(np.asarray(A), np.asarray(B))


def test_loop_icp_on_kdtree_context():
    from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer
    o = IterativeClosestPointOptimizer(ICPConfig(use_surfel_correspondence=False), max_points=1 << 17)
    try:
        m, pts, Ti, _ = _data.kitti_case(13)
        o.set_map_points(m.l0_cloud())
        _, A = o.optimize(None, pts, Ti)
        cur, Tc, mat, Tm, _ = _data.loop_case(4, 7, seed=3)
        _compare_loop(o, cur, Tc, mat, Tm)
        _, B = o.optimize(None, pts, Ti)
        np.testing.assert_array_equal(np.asarray(A), np.asarray(B))
    finally:
        o.close()


def _bits(a):
    return np.asarray(a, np.float32).reshape(-1).view(np.uint32)


@pytest.fixture(scope="module")
def exact_icp():
    from lidar_odometry_amd import IterativeClosestPointOptimizer
    o = IterativeClosestPointOptimizer(max_points=1 << 16)
    o.set_exact(True)
    yield o
    o.close()


@pytest.mark.parametrize("fa,fb,seed", [(2, 6, 0), (4, 7, 3), (10, 14, 5), (20, 23, 9)])
def test_loop_icp_exact_bitwise(exact_icp, fa, fb, seed):
    """Reference-exact mode (lo_set_exact): the loop ICP's every GN iteration bit-identical to the oracle (the same
    sequential fp32 normal equations, sorted-order scale, fp32 LDLT and SVD re-projection as the odometry ICP,
    tests/test_gpu_exact.py), hence the same iteration count, T_rel and inlier count -- no alpha-flip allowance.
    These keyframe clouds (~3.7k points) take the all-pairs LDS search (k_knn_all, k_pick_knn_all, k_inlier_all)."""
    cur, Tc, mat, Tm, _ = _data.loop_case(fa, fb, seed)
    _exact_loop_bitwise(exact_icp, cur, Tc, mat, Tm)


def test_loop_icp_exact_bitwise_grid_path(exact_icp):
    """A matched keyframe cloud beyond kKnnAllMax (8192) points: the cell grid (with the loop's adaptive cell edge),
    the shell search and the wave-per-query brute-force pass instead of the all-pairs search -- still bit-identical."""
    cur, Tc, _, Tm, _ = _data.loop_case(4, 7, 3)
    mat = oracle.voxel_filter(_data.kitti_scan(4, 40), 0.3, 1)          # 11.6k points
    assert len(mat) > 8192
    _exact_loop_bitwise(exact_icp, cur, Tc, mat, Tm)


def _exact_loop_bitwise(exact_icp, cur, Tc, mat, Tm):
    ok_o, conv_o, Tr_o, inl_o, it_o, logs_o = oracle.icp_optimize_loop(cur, Tc, mat, Tm)
    ok_g, Tr_g, inl_g = exact_icp.optimize_loop(cur, Tc, mat, Tm)
    st = exact_icp.get_last_stats()
    assert ok_g == ok_o and st.converged == conv_o and st.num_iterations == it_o
    for k, (lo, lg) in enumerate(zip(logs_o, st.iterations)):
        for key in ("pose", "H", "g", "delta"):
            np.testing.assert_array_equal(_bits(lg[key]), _bits(lo[key]), err_msg=f"iter {k} {key}")
        assert (lg["n_corr"], lg["scale"], lg["alpha"]) == (lo["n_corr"], lo["scale"], lo["alpha"]), k
        assert np.float32(lg["cost"]) == np.float32(lo["cost"]), k
    assert ok_g and conv_o
    np.testing.assert_array_equal(_bits(Tr_g), _bits(Tr_o))
    assert np.float32(inl_g) == np.float32(inl_o)


def test_loop_icp_exact_far_keyframe_same_outcome(exact_icp):
    """The near-singular case above (matched keyframe 500 m away): with the reference's fp32 LDLT the device now
    takes the same steps as the oracle, iteration by iteration."""
    cur, Tc, mat, Tm, _ = _data.loop_case(2, 6)
    far = np.asarray(Tm, np.float32).copy()
    far[3] += 500.0
    ok_o, conv_o, Tr_o, inl_o, it_o, logs_o = oracle.icp_optimize_loop(cur, Tc, mat, far)
    ok, Tr, inl = exact_icp.optimize_loop(cur, Tc, mat, far)
    st = exact_icp.get_last_stats()
    assert not ok_o and not ok
    assert st.num_iterations == it_o and st.converged == conv_o
    for k, (lo, lg) in enumerate(zip(logs_o, st.iterations)):
        np.testing.assert_array_equal(_bits(lg["pose"]), _bits(lo["pose"]), err_msg=f"iter {k}")


def test_loop_icp_lattice_ties_rerun_with_visit_order(exact_icp):
    """The matched keyframe's grid is built without the kd visit order; queries midway between lattice points
    meet exact distance ties, the solve is flagged and rerun with the order (nanoflann's tie-break), so every
    iteration still matches the oracle bit for bit."""
    g = np.arange(-8.0, 8.0, 0.5, dtype=np.float32)
    X, Y = np.meshgrid(g, g, indexing="ij")
    floor = np.stack([X.ravel(), Y.ravel(), np.zeros(X.size, np.float32)], 1)
    wall = np.stack([np.full(X.size, 8.0, np.float32), X.ravel(), Y.ravel() * 0.25 + 2.0], 1)
    wall2 = np.stack([X.ravel(), np.full(X.size, -8.0, np.float32), Y.ravel() * 0.25 + 2.0], 1)
    mat = np.concatenate([floor, wall, wall2]).astype(np.float32)
    cur = (mat + np.array([0.25, 0.0, 0.0], np.float32)).astype(np.float32)      # midway along x: ties
    I = np.eye(3, 4, dtype=np.float32).reshape(12)
    Tc = I.copy()
    Tc[3] = 0.02
    ok_o, conv_o, Tr_o, inl_o, it_o, logs_o = oracle.icp_optimize_loop(cur, Tc, mat, I)
    ok_g, Tr_g, inl_g = exact_icp.optimize_loop(cur, Tc, mat, I)
    st = exact_icp.get_last_stats()
    assert ok_g == ok_o and st.num_iterations == it_o and st.converged == conv_o
    for k, (lo, lg) in enumerate(zip(logs_o, st.iterations)):
        for key in ("pose", "H", "g", "delta"):
            np.testing.assert_array_equal(_bits(lg[key]), _bits(lo[key]), err_msg=f"iter {k} {key}")
        assert lg["n_corr"] == lo["n_corr"], k
    if conv_o:
        np.testing.assert_array_equal(_bits(Tr_g), _bits(Tr_o))
        assert np.float32(inl_g) == np.float32(inl_o)
