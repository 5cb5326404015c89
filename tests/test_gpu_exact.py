"""Reference-exact mode (lo_set_exact, lo_exact.hip) against the oracle restatement: every executed GN iteration's
log -- pose, n_corr, scale, alpha, cost, H, g, delta -- bit-identical, and the same iteration count.  The oracle
follows the reference source line by line (sequential fp32 normal equations in correspondence order, the sorted-order
iteration-0 scale, Eigen's fp32 LDLT, SO3 re-projection through JacobiSVD), so this pins the whole GN step, not
just its tolerance.  (sin / cos of the rotation update: the device rounds the fp64 value, glibc's sinf / cosf
differ from that in the last bit for 0.4 % / 0.01 % of the floats in [1e-7, 0.8]; none of these cases occurs here.)
"""
import numpy as np
import pytest

import oracle
from tests import _data

pytestmark = pytest.mark.gpu


def _bitwise(o, m, pts, Ti, ocfg=None, kdtree=False):
    ok_o, To_o, it_o, logs_o = oracle.icp_optimize(m, pts, Ti, ocfg, kdtree=kdtree)
    ok_g, To_g = o.optimize(None, pts, Ti)
    st = o.get_last_stats()
    assert ok_g == ok_o
    assert st.num_iterations == it_o
    for k, (lo, lg) in enumerate(zip(logs_o, st.iterations)):
        for key in ("pose", "H", "g", "delta"):
            np.testing.assert_array_equal(np.asarray(lg[key], np.float32).view(np.uint32),
                                          np.asarray(lo[key], np.float32).view(np.uint32), err_msg=f"iter {k} {key}")
        assert lg["n_corr"] == lo["n_corr"], k
        assert lg["scale"] == lo["scale"], (k, lg["scale"], lo["scale"])
        assert lg["alpha"] == lo["alpha"], k
        assert np.float32(lg["cost"]) == np.float32(lo["cost"]), k
    if ok_o:
        np.testing.assert_array_equal(np.asarray(To_g, np.float32).reshape(12).view(np.uint32),
                                      np.asarray(To_o, np.float32).reshape(12).view(np.uint32))
    return st


@pytest.fixture(scope="module")
def exact():
    from lidar_odometry_amd import IterativeClosestPointOptimizer
    o = IterativeClosestPointOptimizer(max_points=1 << 16)
    o.set_exact(True)
    yield o
    o.close()


@pytest.mark.parametrize("frame", [11, 13, 17, 21, 25, 31])
def test_exact_kitti_like_bitwise(exact, frame):
    m, pts, Ti, _ = _data.kitti_case(frame)
    k, n, c = _data.surfels(m)
    exact.set_surfels(k, n, c)
    _bitwise(exact, m, pts, Ti)


def test_exact_large_perturbation_bitwise(exact):
    m, pts, Ti, _ = _data.kitti_case(15, seed=5, sigma_t=0.3, sigma_r=0.03)
    k, n, c = _data.surfels(m)
    exact.set_surfels(k, n, c)
    st = _bitwise(exact, m, pts, Ti)
    assert st.num_iterations >= 3


@pytest.mark.parametrize("max_iters,pko", [(1, True), (6, True), (6, False)])
def test_exact_all_iterations_bitwise(max_iters, pko):
    from lidar_odometry_amd import AdaptiveMEstimatorConfig, ICPConfig, IterativeClosestPointOptimizer
    m, pts, Ti, _ = _data.kitti_case(13)
    o = IterativeClosestPointOptimizer(ICPConfig(max_iterations=max_iters, translation_tolerance=1e-9,
                                                 rotation_tolerance=1e-9),
                                       AdaptiveMEstimatorConfig(use_adaptive_m_estimator=pko), max_points=1 << 16)
    try:
        o.set_exact(True)
        k, n, c = _data.surfels(m)
        o.set_surfels(k, n, c)
        ocfg = oracle.kitti_icp_cfg(max_iters)
        ocfg.translation_tolerance = ocfg.rotation_tolerance = 1e-9
        ocfg.use_pko = int(pko)
        st = _bitwise(o, m, pts, Ti, ocfg)
        assert st.num_iterations == max_iters
    finally:
        o.close()


@pytest.mark.parametrize("frame", [281, 295, 313, 331])
def test_exact_city_map_bitwise(exact, frame):
    """The city-grid map (bench.py's KITTI workload, here after 300 frames: ~6k surfels, several streets in the
    120 m radius), scans between and beyond its keyframes, including the turns."""
    m, pts, Ti, _ = _data.city_case(frame, device="cuda")
    k, n, c = _data.surfels(m)
    exact.set_surfels(k, n, c)
    _bitwise(exact, m, pts, Ti)


def test_exact_mid360_bitwise():
    from lidar_odometry_amd import IterativeClosestPointOptimizer, MapGeometry
    m, pts, Ti, _ = _data.mid360_case()
    o = IterativeClosestPointOptimizer(geometry=MapGeometry(voxel_size=0.4), max_points=1 << 16)
    try:
        o.set_exact(True)
        k, n, c = _data.surfels(m)
        o.set_surfels(k, n, c)
        _bitwise(o, m, pts, Ti)
    finally:
        o.close()


def test_exact_kdtree_bitwise():
    from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer
    m, pts, Ti, _ = _data.kitti_case(17)
    o = IterativeClosestPointOptimizer(ICPConfig(use_surfel_correspondence=False), max_points=1 << 16)
    try:
        o.set_exact(True)
        o.set_map_points(m.l0_cloud())
        _bitwise(o, m, pts, Ti, kdtree=True)
    finally:
        o.close()


def test_exact_insufficient_and_capacity(exact):
    m, pts, Ti, _ = _data.kitti_case(11)
    k, n, c = _data.surfels(m)
    exact.set_surfels(k, n, c)
    ok, To = exact.optimize(None, pts + np.float32(5000.0), Ti)
    assert not ok
    # beyond the one-workgroup sort (16384 points) the scan takes the hipCUB-sort path instead of failing
    _bitwise(exact, m, np.zeros((20000, 3), np.float32), Ti)


@pytest.mark.parametrize("n_points", [40_000])
def test_exact_large_scan_bitwise(exact, n_points):
    """C5-style planar-patch scan beyond kExactMaxPoints: residuals sorted by hipCUB's radix sort, the sorted-order
    mean / variance and the 43 term sums staged through LDS -- still every iteration bit-identical to the oracle."""
    m, pts, Ti, _ = _data.patch_case(n_points=n_points)
    k, n, c = _data.surfels(m)
    exact.set_surfels(k, n, c)
    st = _bitwise(exact, m, pts, Ti)
    assert st.num_iterations >= 1


def _scale_width(o):
    """The sort width (points) the last one-workgroup exact scale ran with (DevState::dbg[23], product builds)."""
    import ctypes as C
    from lidar_odometry_amd._lib import lib
    d = (C.c_ulonglong * 24)()
    assert lib().lo_debug_counters_ex(o.ctx, d, 24) == 0
    return int(d[23])


def _bitwise_logs(st, ok_g, To_g, ref):
    ok_o, To_o, it_o, logs_o = ref
    assert ok_g == ok_o and st.num_iterations == it_o
    for k, (lo, lg) in enumerate(zip(logs_o, st.iterations)):
        for key in ("pose", "H", "g", "delta"):
            np.testing.assert_array_equal(np.asarray(lg[key], np.float32).view(np.uint32),
                                          np.asarray(lo[key], np.float32).view(np.uint32), err_msg=f"iter {k} {key}")
        assert lg["scale"] == lo["scale"] and lg["alpha"] == lo["alpha"] and lg["n_corr"] == lo["n_corr"], k
    np.testing.assert_array_equal(np.asarray(To_g, np.float32).reshape(12).view(np.uint32),
                                  np.asarray(To_o, np.float32).reshape(12).view(np.uint32))


@pytest.mark.parametrize("frame", [11, 25])
def test_exact_raw_scan_sorts_by_device_count(exact, frame):
    """A raw scan filtered on the device (lo_icp_optimize_raw) is sized on the host only by its bound ceil(n_raw /
    stride) (~14k points here), while ~4k points survive the filter.  The iteration-0 scale picks its sort width from
    the count on the device (k_exact_scale_cd): the one-workgroup path at <= 8192 points, not a 16k-wide sort.  Every
    iteration bit-identical to the oracle run on the host-filtered scan (Estimator.cpp:561-589 -> optimize)."""
    m, pts, Ti, _ = _data.kitti_case(frame)
    k, n, c = _data.surfels(m)
    exact.set_surfels(k, n, c)
    raw = _data.kitti_scan(frame)
    assert (len(raw) + 7) // 8 > 8192 >= len(pts)
    ok_g, To_g = exact.optimize_raw(None, raw, Ti, stride=8, voxel_size=0.5)
    _bitwise_logs(exact.get_last_stats(), ok_g, To_g, oracle.icp_optimize(m, pts, Ti))
    w = _scale_width(exact)
    assert len(pts) <= w <= 8192, w


def test_exact_raw_scan_beyond_8192_filtered_points(exact):
    """The device count above 8192 (a fine filter over a 14k-point raw scan): the widest one-workgroup sort (16384,
    out of line in k_exact_scale_cd), still bitwise."""
    m, pts, Ti, _ = _data.patch_case(n_points=14_000, seed=1003)
    k, n, c = _data.surfels(m)
    exact.set_surfels(k, n, c)
    filt = oracle.voxel_filter(pts, 0.001, 1)
    assert 8192 < len(filt) <= 16384
    ok_g, To_g = exact.optimize_raw(None, pts, Ti, stride=1, voxel_size=0.001)
    np.testing.assert_array_equal(exact.filtered_points().view(np.uint32), filt.view(np.uint32))
    _bitwise_logs(exact.get_last_stats(), ok_g, To_g, oracle.icp_optimize(m, filt, Ti))
    assert _scale_width(exact) == 16384


@pytest.mark.parametrize("extra,width", [(-800, 3072), (1000, 5120), (2200, 6144)])
def test_exact_scale_widths_between_powers_of_two(exact, extra, width):
    """The one-workgroup scale sorts ceil(n / 1024) keys per thread (r06: widths 3, 5 and 6 beside 1, 2, 4, 8, 16):
    scans of ~2.9k, ~4.7k and ~5.9k points run the 3072-, 5120- and 6144-wide sorts, every iteration bit-identical."""
    m, pts, Ti, _ = _data.kitti_case(11)
    k, n, c = _data.surfels(m)
    exact.set_surfels(k, n, c)
    if extra < 0:
        p = pts[: len(pts) + extra]
    else:
        p = np.concatenate([pts, pts[:extra] + np.float32(0.013)]).astype(np.float32)
    assert width - 1024 < len(p) <= width
    _bitwise(exact, m, p, Ti)
    assert _scale_width(exact) == width


@pytest.mark.parametrize("n_points", [12_000])
def test_exact_mid_size_scan_both_sort_paths(exact, monkeypatch, n_points):
    """8192 < n <= 16384 host-counted: the one-workgroup counting sort at width 16384 (default) and the chip-wide rank
    sort (LO_EXACT_RANKSORT, the round-5 path) give the oracle's bits."""
    m, pts, Ti, _ = _data.patch_case(n_points=n_points, seed=1001)
    k, n, c = _data.surfels(m)
    exact.set_surfels(k, n, c)
    _bitwise(exact, m, pts, Ti)
    assert _scale_width(exact) == 16384
    monkeypatch.setenv("LO_EXACT_RANKSORT", "1")
    _bitwise(exact, m, pts, Ti)
