"""GPU parity of the KDTree correspondence variant (use_surfel_correspondence = false).

The 5-NN is pinned to the reference's own nanoflann 1.7.1: tests/golden/knn_golden.npz was written by
oracle/_ref/knn_golden (the vendored nanoflann.hpp configured as util::KdTree) and the device search must return
its neighbour lists exactly -- indices, order, equal-distance tie-breaks (nanoflann's visit order) and fp32
distances.  The oracle (restated nanoflann tree, tests/test_oracle.py pins it to the same fixtures) adds the fp64
collinearity gate / 5-point plane fit; the device runs a grid search with a brute-force fallback.  Bars:
identical valid set and bit-identical fp64 plane distances at a given pose; optimize per GN iteration within
1e-4 m / 1e-4 rad (north_star).  The plane fit restates JacobiSVD<MatrixXd>(5x3) as a Jacobi eigen-solve of the
scatter matrix (Eigen is absent: parity unpinned at that boundary).
"""
import numpy as np
import pytest

import oracle
from tests import _data

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kd_icp():
    from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer
    o = IterativeClosestPointOptimizer(ICPConfig(use_surfel_correspondence=False), max_points=1 << 17)
    yield o
    o.close()


def _pose_err(Ta, Tb):
    A = np.asarray(Ta, np.float64).reshape(3, 4)
    B = np.asarray(Tb, np.float64).reshape(3, 4)
    return float(np.linalg.norm(A[:, 3] - B[:, 3])), _data.rot_angle(A[:, :3], B[:, :3])


@pytest.mark.parametrize("frame", [11, 21])
def test_kdtree_correspondences_bitwise(kd_icp, frame):
    m, pts, Ti, _ = _data.kitti_case(frame)
    kd_icp.set_map_points(m.l0_cloud())
    n_o, v_o, r_o = oracle.find_correspondences(m, pts, Ti, kdtree=True)
    n_g, v_g, r_g = kd_icp.find_correspondences(pts, Ti)
    assert n_o > 0.5 * len(pts)
    assert n_g == n_o
    np.testing.assert_array_equal(v_g, v_o)
    np.testing.assert_array_equal(r_g.view(np.uint64), r_o.view(np.uint64))


def _knn_golden():
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "knn_golden.npz"))
    return g, sorted({k.rsplit("_", 1)[0] for k in g.files})


@pytest.mark.parametrize("case", ["kitti", "lattice", "lattice_quarter", "duplicates", "patches", "tiny", "nonfinite"])
def test_knn_matches_nanoflann_golden(kd_icp, case):
    """Device 5-NN == the reference's nanoflann on its fixtures, ties included (the lattice / duplicate cases
    have thousands of exactly equal fp32 distances, ranked by nanoflann's visit order)."""
    g, names = _knn_golden()
    assert case in names
    cloud, q = g[case + "_cloud"], g[case + "_query"]
    kd_icp.set_map_points(cloud)
    idx, dist, found = kd_icp.nearest_k_search(q)
    want_found = g[case + "_found"]
    full = want_found == 5
    np.testing.assert_array_equal(found == 5, full)                 # < 5 neighbours: the ICP skips the query
    np.testing.assert_array_equal(idx[full], g[case + "_idx"][full])
    np.testing.assert_array_equal(dist[full].view(np.uint32), g[case + "_dist"][full].view(np.uint32))


def test_kdtree_fallback_and_edge_queries(kd_icp):
    """Far queries exceed the grid shells (brute-force pass); NaN/inf queries find nothing."""
    m, pts, Ti, _ = _data.kitti_case(13)
    kd_icp.set_map_points(m.l0_cloud())
    q = pts[:700].copy()
    q[:200] += np.float32(25.0)            # beyond the shell radius of the grid search
    q[200] = [np.nan, 0, 0]
    q[201] = [np.inf, 1, 1]
    n_o, v_o, r_o = oracle.find_correspondences(m, q, Ti, kdtree=True)
    n_g, v_g, r_g = kd_icp.find_correspondences(q, Ti)
    assert not v_g[200] and not v_g[201]
    assert n_g == n_o
    np.testing.assert_array_equal(v_g, v_o)
    np.testing.assert_array_equal(r_g.view(np.uint64), r_o.view(np.uint64))


def test_kdtree_tiny_maps():
    from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer
    o = IterativeClosestPointOptimizer(ICPConfig(use_surfel_correspondence=False), max_points=4096)
    try:
        rng = np.random.default_rng(3)
        pts = rng.normal(size=(300, 3)).astype(np.float32)
        I = np.eye(3, 4, dtype=np.float32)
        o.set_map_points(rng.normal(size=(4, 3)).astype(np.float32))      # fewer than K = 5 points
        n, v, _ = o.find_correspondences(pts, I)
        assert n == 0 and not v.any()
        five = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0.01], [0.5, 0.5, 0]], np.float32)
        o.set_map_points(five)                                             # every query sees the same plane
        n, v, r = o.find_correspondences(pts, I)
        assert n > 0
        ok = v.astype(bool)
        assert np.all(np.abs(r[ok]) <= 1.0)
        ok_opt, To = o.optimize(None, pts[:0], I)                         # empty scan -> failure
        assert not ok_opt
    finally:
        o.close()


@pytest.mark.parametrize("frame", [11, 17, 25])
def test_kdtree_optimize_per_iteration(kd_icp, frame):
    m, pts, Ti, _ = _data.kitti_case(frame)
    kd_icp.set_map_points(m.l0_cloud())
    ok_o, To_o, it_o, logs_o = oracle.icp_optimize(m, pts, Ti, kdtree=True)
    ok_g, To_g = kd_icp.optimize(None, pts, Ti)
    st = kd_icp.get_last_stats()
    assert ok_g == ok_o
    assert st.num_iterations == it_o
    for k, (lo, lg) in enumerate(zip(logs_o, st.iterations)):
        if k == 0:
            assert lg["n_corr"] == lo["n_corr"]
            assert lg["scale"] == pytest.approx(lo["scale"], rel=1e-12)
            assert lg["alpha"] == lo["alpha"]
        else:
            assert abs(lg["n_corr"] - lo["n_corr"]) <= max(2, 1e-4 * lo["n_corr"])
        et, er = _pose_err(lg["pose"], lo["pose"])
        assert et <= 1e-4 and er <= 1e-4, f"iter {k}: dt {et:.2e} m, dr {er:.2e} rad"


def test_kdtree_voxelmap_sync():
    """optimize(voxel_map, ...) uploads GetPointCloud from the product VoxelMap in KDTree mode."""
    from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer
    from lidar_odometry_amd import synth
    from lidar_odometry_amd.voxelmap import VoxelMap, voxel_filter
    seq = _data.kitti_seq()
    vm = VoxelMap(0.5, 3, 0.1, True)
    om = oracle.VoxelMap(0.5, 3, 0.1, True)
    for k in (0, 2, 4):
        p = voxel_filter(_data.kitti_scan(k), 0.5, 8)
        w = synth.transform(seq.poses[k], p)
        vm.update(w, seq.poses[k][:3, 3], 120.0, True)
        om.update(w, seq.poses[k][:3, 3], 120.0, True)
    np.testing.assert_array_equal(vm.l0_cloud(), om.l0_cloud())
    pts = voxel_filter(_data.kitti_scan(3), 0.5, 8)
    Ti = _data.pose12(seq.poses[3])
    o = IterativeClosestPointOptimizer(ICPConfig(use_surfel_correspondence=False), max_points=1 << 16)
    try:
        ok, T = o.optimize(vm, pts, Ti)
        ok_o, To, _, _ = oracle.icp_optimize(om, pts, Ti, kdtree=True)
        assert ok == ok_o
        et, er = _pose_err(T, To)
        assert et <= 1e-4 and er <= 1e-4
    finally:
        o.close()


def test_kdtree_exact_ties_lattice():
    """Lattice map: many exactly equal neighbour distances; the device must break ties by index like the
    oracle (grid shells and the brute-force pass both)."""
    from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer, MapGeometry
    g = np.stack(np.meshgrid(np.arange(12), np.arange(12), np.arange(3), indexing="ij"), -1).reshape(-1, 3)
    lattice = (g * 0.5).astype(np.float32)
    m = oracle.VoxelMap(0.25, 3, 0.1, False)
    m.update(lattice, np.zeros(3), 1e3, True)
    rng = np.random.default_rng(5)
    q = (rng.integers(0, 22, size=(600, 3)) * 0.25).astype(np.float32)
    q[500:] += np.float32(9.0)                       # some far queries -> brute-force pass
    I = np.eye(3, 4, dtype=np.float32).reshape(12)
    o = IterativeClosestPointOptimizer(ICPConfig(use_surfel_correspondence=False), geometry=MapGeometry(voxel_size=0.25),
                                       max_points=4096)
    try:
        o.set_map_points(m.l0_cloud())
        n_o, v_o, r_o = oracle.find_correspondences(m, q, I, kdtree=True)
        n_g, v_g, r_g = o.find_correspondences(q, I)
        assert n_g == n_o
        np.testing.assert_array_equal(v_g, v_o)
        np.testing.assert_array_equal(r_g.view(np.uint64), r_o.view(np.uint64))
    finally:
        o.close()


def test_kdtree_optimize_repeatable(kd_icp):
    """Atomics only build the unresolved-query list; results must be bitwise run-to-run."""
    m, pts, Ti, _ = _data.kitti_case(21)
    kd_icp.set_map_points(m.l0_cloud())
    outs = [kd_icp.optimize(None, pts, Ti)[1] for _ in range(3)]
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])


def test_device_grid_tie_reruns_with_kd_order():
    """A device-built grid (the device map's RebuildKdTree, lo_devmap_sync_points) carries no kd visit order: a scan
    whose 5-NN search meets a deciding distance tie is re-run by lo_icp_result with the order built on the host, and
    then equals, bit for bit, the same scan on the host-built grid of the same points (lo_map_set_points)."""
    import ctypes as C

    from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer, lib
    from lidar_odometry_amd.voxelmap import DeviceVoxelMap, VoxelMap
    # map points at L0 voxel centres on three orthogonal planes: the lattice makes equal distances everywhere
    g = np.arange(-12, 12) * 0.5 + 0.25
    A2, B2 = np.meshgrid(g, g)
    a, b = A2.ravel(), B2.ravel()
    c = np.full(a.size, 0.25)
    world = np.ascontiguousarray(np.concatenate([np.stack([a, b, c - 3.0], 1), np.stack([c + 3.0, a, b], 1),
                                                 np.stack([a, c + 3.0, b], 1)]), dtype=np.float32)
    # the scan: points halfway between lattice neighbours, slightly off the initial pose
    rng = np.random.default_rng(3)
    scan = world[rng.choice(len(world), 600, replace=False)] + np.float32(0.25) * np.array([1, 0, 0], np.float32)
    scan = np.ascontiguousarray(scan, dtype=np.float32)
    T0 = np.eye(3, 4, dtype=np.float32)
    T0[:, 3] = [0.02, -0.01, 0.01]
    dev = IterativeClosestPointOptimizer(ICPConfig(use_surfel_correspondence=False), max_points=4096)
    host = IterativeClosestPointOptimizer(ICPConfig(use_surfel_correspondence=False), max_points=4096)
    dm = DeviceVoxelMap(dev, 0.5, 3, 0.1, max_l0=1 << 14, max_points=1 << 14)
    try:
        dm.update(world, np.zeros(3), 1000.0, True)
        L = lib()
        assert L.lo_devmap_sync_points(dm._h) == 0
        hv = VoxelMap(0.5, 3, 0.1, False)                   # the host map without surfels: its GetPointCloud
        hv.update(world, np.zeros(3), 1000.0, True)
        host.set_map_points(hv.l0_cloud())
        ok_d, T_d = dev.optimize(None, scan, T0)
        ok_h, T_h = host.optimize(None, scan, T0)
        assert L.lo_kd_reruns(dev.ctx) >= 1                 # the lattice forced the tie path
        assert ok_d == ok_h
        np.testing.assert_array_equal(np.asarray(T_d, np.float32).view(np.uint32), np.asarray(T_h, np.float32).view(np.uint32))
        n_d, v_d, r_d = dev.find_correspondences(scan, T0)
        n_h, v_h, r_h = host.find_correspondences(scan, T0)
        assert n_d == n_h
        np.testing.assert_array_equal(v_d, v_h)
        np.testing.assert_array_equal(np.asarray(r_d).view(np.uint64), np.asarray(r_h).view(np.uint64))
    finally:
        dm.close()
        dev.close()
        host.close()
