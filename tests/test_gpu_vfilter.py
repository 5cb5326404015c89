"""Device FastVoxelFilter (Estimator::preprocess_frame, VoxelMap.h:73-104) against the
oracle restatement: identical output (order and bits), and raw-scan -> pose optimize against oracle
filter-then-optimize per GN iteration."""
import numpy as np
import pytest

import oracle
from tests import _data

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def icp():
    from lidar_odometry_amd import IterativeClosestPointOptimizer
    o = IterativeClosestPointOptimizer(max_points=1 << 18)
    yield o
    o.close()


@pytest.mark.parametrize("frame,stride,voxel", [(3, 8, 0.5), (11, 1, 0.5), (20, 4, 0.4), (7, 8, 1.0)])
def test_voxel_filter_bitwise(icp, frame, stride, voxel):
    raw = _data.kitti_scan(frame)
    ref = oracle.voxel_filter(raw, voxel, stride)
    got = icp.voxel_filter(raw, voxel, stride)
    assert len(ref) > 1000
    assert got.shape == ref.shape
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_voxel_filter_edge_cases(icp):
    rng = np.random.default_rng(9)
    raw = rng.normal(scale=20.0, size=(20000, 3)).astype(np.float32)
    raw[5] = [np.nan, 0, 0]
    raw[13] = [0, np.inf, 0]
    raw[21] = [1e30, 2.0, 3.0]          # floor(x / voxel) beyond int64: reference clamps cell to 0
    raw[29] = [-1e30, 2.0, 3.0]
    raw[37] = [6e5, -6e5, 1.0]          # beyond +-2^20 cells: clamped
    raw[45] = [-6e5, 6e5, 1.0]
    for stride in (1, 3, 8):
        ref = oracle.voxel_filter(raw, 0.5, stride)
        got = icp.voxel_filter(raw, 0.5, stride)
        np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    # all-invalid and empty inputs
    bad = np.full((100, 3), np.nan, np.float32)
    assert len(icp.voxel_filter(bad, 0.5, 1)) == 0
    assert len(icp.voxel_filter(raw[:0], 0.5, 1)) == 0
    # many points in one voxel: long in-order fp32 running sum
    one = (rng.uniform(0.0, 0.49, size=(50000, 3))).astype(np.float32)
    np.testing.assert_array_equal(icp.voxel_filter(one, 0.5, 1).view(np.uint32),
                                  oracle.voxel_filter(one, 0.5, 1).view(np.uint32))


def test_voxel_filter_density_mix_and_signed_zero(icp):
    """Voxels of 1..16, 17..64 and >64 samples interleaved in the input (the device's three summation paths), and a
    lone -0.0 point: the reference's sums start at +0.0f, so it comes out +0.0."""
    rng = np.random.default_rng(11)
    centers = rng.integers(-40, 40, size=(600, 3)).astype(np.float32) * 0.5 + 0.25
    counts = np.concatenate([rng.integers(1, 17, 300), rng.integers(17, 65, 200), rng.integers(65, 300, 100)])
    pts = np.concatenate([c + rng.uniform(-0.2, 0.2, size=(k, 3)).astype(np.float32) for c, k in zip(centers, counts)])
    pts = pts[rng.permutation(len(pts))]
    pts = np.concatenate([pts, np.array([[-0.0, 100.0, -0.0]], np.float32)])
    for stride in (1, 2):
        ref = oracle.voxel_filter(pts, 0.5, stride)
        got = icp.voxel_filter(pts, 0.5, stride)
        np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert oracle.voxel_filter(pts, 0.5, 1)[-1].view(np.uint32)[0] == 0      # +0.0, not -0.0


@pytest.mark.parametrize("frame", [11, 25])
def test_optimize_raw_per_iteration(icp, frame):
    m, pts, Ti, _ = _data.kitti_case(frame)
    k, n, c = _data.surfels(m)
    icp.set_surfels(k, n, c)
    raw = _data.kitti_scan(frame)
    np.testing.assert_array_equal(pts, oracle.voxel_filter(raw, 0.5, 8))
    ok_o, To_o, it_o, logs_o = oracle.icp_optimize(m, pts, Ti)
    ok_g, To_g = icp.optimize_raw(None, raw, Ti, stride=8, voxel_size=0.5)
    st = icp.get_last_stats()
    assert ok_g == ok_o and st.num_iterations == it_o
    assert st.iterations[0]["n_corr"] == logs_o[0]["n_corr"]
    assert st.iterations[0]["alpha"] == logs_o[0]["alpha"]
    for lg, lo in zip(st.iterations, logs_o):
        A = np.asarray(lg["pose"], np.float64).reshape(3, 4)
        B = np.asarray(lo["pose"], np.float64).reshape(3, 4)
        assert np.linalg.norm(A[:, 3] - B[:, 3]) <= 1e-4 and _data.rot_angle(A[:, :3], B[:, :3]) <= 1e-4
    np.testing.assert_array_equal(icp.filtered_points(), pts)   # feature cloud for the keyframe map update


def test_optimize_raw_matches_host_filtered(icp):
    """Device-count mode (grids sized for ceil(n/stride), count read on the device) gives the same pose as the
    host-count path on the same filtered points."""
    m, pts, Ti, _ = _data.kitti_case(17)
    k, n, c = _data.surfels(m)
    icp.set_surfels(k, n, c)
    ok_a, A = icp.optimize(None, pts, Ti)
    ok_b, B = icp.optimize_raw(None, _data.kitti_scan(17), Ti, stride=8, voxel_size=0.5)
    assert ok_a == ok_b
    np.testing.assert_array_equal(A, B)


def test_optimize_raw_pinned_input(icp):
    """A raw scan in pinned host memory (lo_host_alloc) is read by the device filter in place: same filtered cloud
    and pose as the staged pageable copy, bit for bit."""
    from lidar_odometry_amd import pinned_empty
    m, pts, Ti, _ = _data.kitti_case(19)
    k, n, c = _data.surfels(m)
    icp.set_surfels(k, n, c)
    raw = _data.kitti_scan(19)
    ok_a, A = icp.optimize_raw(None, raw, Ti, stride=8, voxel_size=0.5)
    fa = icp.filtered_points()
    pr = pinned_empty(raw.shape)
    pr[:] = raw
    ok_b, B = icp.optimize_raw(None, pr, Ti, stride=8, voxel_size=0.5)
    fb = icp.filtered_points()
    assert ok_a == ok_b
    np.testing.assert_array_equal(A, B)
    np.testing.assert_array_equal(fa.view(np.uint32), fb.view(np.uint32))
    del pr
