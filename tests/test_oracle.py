"""CPU tests: the oracle against the reference's own golden vectors and against known-answer properties."""
import json
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _golden():
    z = np.load(os.path.join(GOLD, "pko_inputs.npz"))
    with open(os.path.join(GOLD, "pko_golden.jsonl")) as f:
        for line in f:
            d = json.loads(line)
            yield d, z[f"case_{d['case']}"]


@pytest.mark.parametrize("case", list(range(26)))
def test_pko_matches_reference_golden_bitwise(case):
    d, r = [x for x in _golden()][case]
    assert len(r) == d["n"]
    a, g = oracle.pko_scale_factor(r)
    assert a == d["alpha"]
    for k in ("w", "mu", "var"):
        np.testing.assert_array_equal(g[k], np.array(d[k], dtype=np.float64))


def _kernel_golden():
    z = np.load(os.path.join(GOLD, "pko_inputs.npz"))
    with open(os.path.join(GOLD, "pko_golden_kernels.jsonl")) as f:
        for line in f:
            d = json.loads(line)
            yield d, z[f"case_{d['case']}"]


_KG = [(d["kernel"], d["name"]) for d, _ in _kernel_golden()]


@pytest.mark.parametrize("kernel,name", _KG)
def test_pko_other_kernels_match_reference_golden_bitwise(kernel, name):
    """pko_kernel_type tukey / welsch / gemanMcClure / pseudoHuber / cauchy and an unknown name (-> Cauchy),
    AdaptiveMEstimator.cpp:99-156, against the reference's own compiled AdaptiveMEstimator.cpp."""
    d, r = next((d, r) for d, r in _kernel_golden() if d["kernel"] == kernel and d["name"] == name)
    cfg = oracle.kitti_pko_cfg()
    cfg.kernel = oracle.pko_kernel_id(kernel)
    a, g = oracle.pko_scale_factor(r, cfg)
    assert a == d["alpha"]
    for k in ("w", "mu", "var"):
        np.testing.assert_array_equal(g[k], np.array(d[k], dtype=np.float64))
    al, z = oracle.pko_tables(cfg)
    np.testing.assert_array_equal(al, np.array(d["alphas"]))
    np.testing.assert_array_equal(z, np.array(d["Z"]))


def test_pko_tables_match_reference():
    d, _ = next(iter(_golden()))
    a, z = oracle.pko_tables()
    np.testing.assert_array_equal(a, np.array(d["alphas"]))
    np.testing.assert_array_equal(z, np.array(d["Z"]))


def test_shuffle_prefix_matches_reference():
    for d, r in _golden():
        np.testing.assert_array_equal(oracle.shuffle_prefix(len(r), 100), np.array(d["perm"], dtype=np.int32))
        if d["n"] > 0:
            np.testing.assert_array_equal(oracle.kmeans_seed_draws(min(100, d["n"])), np.array(d["kmeans_draws"], dtype=np.int32))


def test_jacobi_svd_reconstructs_and_sorts():
    rng = np.random.default_rng(0)
    for _ in range(200):
        A = rng.normal(size=(3, 3)).astype(np.float32)
        A = (A @ A.T).astype(np.float32)          # covariance-like (symmetric PSD)
        rc, U, S, V = oracle.jacobi_svd3(A)
        assert rc == 0
        assert S[0] >= S[1] >= S[2] >= 0
        np.testing.assert_allclose(U @ np.diag(S) @ V.T, A, atol=2e-5 * np.abs(A).max())
        np.testing.assert_allclose(U.T @ U, np.eye(3), atol=2e-6)


def test_jacobi_svd_degenerate():
    rc, U, S, V = oracle.jacobi_svd3(np.zeros((3, 3), np.float32))
    assert rc == 0 and np.all(S == 0)
    np.testing.assert_array_equal(U, np.eye(3, dtype=np.float32))
    rc, U, S, V = oracle.jacobi_svd3(np.diag([1.0, 4.0, 2.0]).astype(np.float32))
    np.testing.assert_array_equal(S, np.array([4, 2, 1], np.float32))


def test_so3_exp_matches_rodrigues():
    rng = np.random.default_rng(1)
    for _ in range(100):
        w = rng.normal(0, 0.3, 3).astype(np.float32)
        R = oracle.so3_exp(w)
        th = np.linalg.norm(w.astype(np.float64))
        k = w / th
        K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        Rr = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
        np.testing.assert_allclose(R, Rr, atol=1e-6)
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-6)
    assert np.array_equal(oracle.so3_normalize(np.eye(3)), np.eye(3, dtype=np.float32))


def test_ldlt_solve():
    rng = np.random.default_rng(2)
    for _ in range(50):
        J = rng.normal(size=(200, 6))
        H = (J.T @ J).astype(np.float32)
        b = rng.normal(size=6).astype(np.float32)
        x = oracle.ldlt6_solve(H, b)
        np.testing.assert_allclose(H.astype(np.float64) @ x, b, rtol=1e-3, atol=1e-3)
    # zero matrix -> zero solution (pivot handling of LDLT::compute / _solve_impl)
    np.testing.assert_array_equal(oracle.ldlt6_solve(np.zeros((6, 6), np.float32), np.ones(6, np.float32)), np.zeros(6))


def test_voxel_filter_first_occurrence_order():
    pts = np.array([[0.1, 0.1, 0.1], [5, 5, 5], [0.2, 0.2, 0.2], [np.nan, 0, 0], [5.1, 5.1, 5.1]], np.float32)
    out = oracle.voxel_filter(pts, 0.5, 1)
    assert out.shape == (2, 3)
    s = np.float32(0.1) + np.float32(0.2)
    np.testing.assert_array_equal(out[0], np.float32(s) * (np.float32(1.0) / np.float32(2.0)))
    out2 = oracle.voxel_filter(pts, 0.5, 2)     # stride picks 0, 2, 4
    assert out2.shape == (2, 3)


def test_voxelmap_surfels_and_lookup():
    rng = np.random.default_rng(3)
    # a dense horizontal plane z=0.2 over [0,6]^2 -> planar L1 voxels with normal +-z
    xy = rng.uniform(0, 6, (20000, 2))
    pts = np.concatenate([xy, np.full((20000, 1), 0.2)], axis=1).astype(np.float32)
    m = oracle.VoxelMap(0.5, 3, 0.1, True)
    m.update(pts, np.zeros(3), 100.0, True)
    k, n, c, pl = m.surfels()
    assert len(k) >= 9
    assert np.all(np.abs(np.abs(n[:, 2]) - 1) < 1e-5)
    ok, nn, cc = m.lookup(np.array([1.0, 1.0, 0.3], np.float32))
    assert ok and abs(cc[2] - 0.2) < 1e-5
    ok, _, _ = m.lookup(np.array([1.0, 1.0, 5.0], np.float32))
    assert not ok
    # radius pruning removes everything far from a distant sensor
    m.update(pts[:10], np.array([1000.0, 0, 0]), 10.0, True)
    assert m.l0_count() <= 10


def test_oracle_icp_converges_on_kitti_like():
    from tests import _data
    m, pts, Ti, Tgt = _data.kitti_case(11)
    ok, To, iters, logs = oracle.icp_optimize(m, pts, Ti)
    assert ok and 1 <= iters <= 4
    assert np.linalg.norm(To.reshape(3, 4)[:, 3] - Tgt.reshape(3, 4)[:, 3]) < 0.02
    assert logs[0]["n_corr"] > 1000


def test_oracle_icp_insufficient_on_empty_map():
    m = oracle.VoxelMap(0.5, 3, 0.1, True)
    pts = np.random.default_rng(0).normal(size=(100, 3)).astype(np.float32)
    Ti = np.eye(3, 4, dtype=np.float32).reshape(12)
    ok, To, iters, logs = oracle.icp_optimize(m, pts, Ti)
    assert not ok and iters == 0
    np.testing.assert_array_equal(To, Ti)


# ------------------------------------------------------------------ KDTree variant: kd-tree == brute force
def _kd_both(m, pts, T):
    oracle.set_kdtree_search(False)
    try:
        b = oracle.find_correspondences(m, pts, T, kdtree=True)
    finally:
        oracle.set_kdtree_search(True)
    t = oracle.find_correspondences(m, pts, T, kdtree=True)
    return b, t


def test_oracle_kdtree_matches_bruteforce_kitti():
    from tests import _data
    m, pts, Ti, _ = _data.kitti_case(11)
    (nb, vb, rb), (nt, vt, rt) = _kd_both(m, pts, Ti)
    assert nb == nt > 0
    np.testing.assert_array_equal(vb, vt)
    np.testing.assert_array_equal(rb.view(np.uint64), rt.view(np.uint64))


def test_oracle_kdtree_ties_and_nonfinite():
    """A lattice map makes many neighbour distances exactly equal: ties must resolve by index like the brute
    force; NaN / inf queries find nothing."""
    g = np.stack(np.meshgrid(np.arange(12), np.arange(12), np.arange(3), indexing="ij"), -1).reshape(-1, 3)
    lattice = (g * 0.5).astype(np.float32)
    m = oracle.VoxelMap(0.25, 3, 0.1, False)
    m.update(lattice, np.zeros(3), 1e3, True)
    rng = np.random.default_rng(5)
    q = (rng.integers(0, 22, size=(400, 3)) * 0.25).astype(np.float32)   # on-lattice / mid-cell: exact ties
    q[:5] = [[np.nan, 0, 0], [np.inf, 0, 0], [0, -np.inf, 0], [1, 1, np.nan], [1e30, 0, 0]]
    I = np.eye(3, 4, dtype=np.float32).reshape(12)
    (nb, vb, rb), (nt, vt, rt) = _kd_both(m, q, I)
    assert nb == nt
    np.testing.assert_array_equal(vb, vt)
    np.testing.assert_array_equal(rb.view(np.uint64), rt.view(np.uint64))
    assert not vb[:4].any()


def _knn_cases():
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "knn_golden.npz"))
    return g, sorted({k.rsplit("_", 1)[0] for k in g.files})


@pytest.mark.parametrize("use_tree", [True, False])
def test_knn_matches_nanoflann_golden(use_tree):
    """The oracle's restated nanoflann 1.7.1 tree (and its exhaustive scan ranked by nanoflann's visit order) returns
    exactly the reference's util::KdTree::nearestKSearch(q, 5) -- indices, order, tie-breaks and fp32 distances --
    on every fixture written by oracle/_ref/knn_golden (the reference's own nanoflann.hpp)."""
    g, names = _knn_cases()
    ties = 0
    for n in names:
        idx, dist, found = oracle.kdtree_knn5(g[n + "_cloud"], g[n + "_query"], use_tree=use_tree)
        np.testing.assert_array_equal(found, g[n + "_found"], err_msg=n)
        np.testing.assert_array_equal(idx, g[n + "_idx"], err_msg=n)
        np.testing.assert_array_equal(dist.view(np.uint32), g[n + "_dist"].view(np.uint32), err_msg=n)
        d = g[n + "_dist"]
        ties += int(np.sum((d[:, :4] == d[:, 1:]) & np.isfinite(d[:, 1:])))
    assert ties > 1000          # the lattice / duplicate cases exercise the visit-order tie-break
