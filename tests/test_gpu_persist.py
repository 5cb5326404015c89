"""The persistent GN launch (lo_persist.hip: k_gn, the whole optimize() of a small PKO scan in one launch, stages handed
between workgroups in place) against the launch-per-stage path on the same context (lo_set_persistent(ctx, 0)):
identical iteration count, status, and bit-identical per-iteration logs (pose, n_corr, scale, alpha, cost, H, g,
delta).  The launch-per-stage path is itself held to the oracle by test_gpu_parity.py / test_gpu_exact.py.
Reference: IterativeClosestPointOptimizer.cpp:281-449.
"""
import ctypes as C

import numpy as np
import pytest

from tests import _data

pytestmark = pytest.mark.gpu


def _run(o, pts, Ti, persistent):
    o.set_persistent(persistent)
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


def _ctx(max_iters=4, tol=0.005, voxel=0.5, max_points=1 << 16):
    from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer, MapGeometry
    cfg = ICPConfig(max_iterations=max_iters, translation_tolerance=tol, rotation_tolerance=tol)
    return IterativeClosestPointOptimizer(cfg, geometry=MapGeometry(voxel_size=voxel), max_points=max_points)


@pytest.mark.parametrize("frame", [11, 13, 17, 21, 25, 31])
def test_persistent_kitti_bitwise(frame):
    m, pts, Ti, _ = _data.kitti_case(frame)
    o = _ctx()
    try:
        o.set_surfels(*_data.surfels(m))
        _same(_run(o, pts, Ti, True), _run(o, pts, Ti, False))
    finally:
        o.close()


@pytest.mark.parametrize("max_iters", [1, 2, 3, 5, 6])
def test_persistent_iteration_counts_bitwise(max_iters):
    """Tolerance 1e-9: every iteration runs, both parities of the double-buffered JS grid / candidate sets are reused."""
    m, pts, Ti, _ = _data.kitti_case(13)
    o = _ctx(max_iters=max_iters, tol=1e-9)
    try:
        o.set_surfels(*_data.surfels(m))
        a = _run(o, pts, Ti, True)
        assert a[2].num_iterations == max_iters
        _same(a, _run(o, pts, Ti, False))
    finally:
        o.close()


def test_persistent_mid360_bitwise():
    m, pts, Ti, _ = _data.mid360_case()
    o = _ctx(voxel=0.4)
    try:
        o.set_surfels(*_data.surfels(m))
        _same(_run(o, pts, Ti, True), _run(o, pts, Ti, False))
    finally:
        o.close()


@pytest.mark.parametrize("copies", [2, 3, 5, 8])
def test_persistent_larger_scans_bitwise(copies):
    """4k .. 32k points: 2, 3 or 4 candidate workgroups per alpha (W) and more correspondence blocks than the grid has
    PKO workgroups (nb > 64 falls back to the launch-per-stage path -- bit-identical by construction)."""
    m, pts, Ti, _ = _data.kitti_case(17)
    rng = np.random.default_rng(copies)
    big = np.concatenate([pts + rng.normal(0.0, 0.02, pts.shape).astype(np.float32) for _ in range(copies)])
    o = _ctx()
    try:
        o.set_surfels(*_data.surfels(m))
        _same(_run(o, big, Ti, True), _run(o, big, Ti, False))
    finally:
        o.close()


def test_persistent_insufficient():
    m, pts, Ti, _ = _data.kitti_case(11)
    o = _ctx()
    try:
        o.set_surfels(*_data.surfels(m))
        far = pts + np.float32(5000.0)
        a, b = _run(o, far, Ti, True), _run(o, far, Ti, False)
        assert not a[0] and not b[0]
        np.testing.assert_array_equal(a[1], Ti.reshape(12))
        _same(a, b)
        sub = pts[:40]                      # few points: correspondences may drop below 10 in a later iteration
        _same(_run(o, sub, Ti, True), _run(o, sub, Ti, False))
        one = pts[:1]
        _same(_run(o, one, Ti, True), _run(o, one, Ti, False))
    finally:
        o.close()


def test_persistent_stage_timing_bitwise():
    """With in-step stage timing the first correspondence search runs as its own (timed) launch before k_gn."""
    from lidar_odometry_amd import lib
    m, pts, Ti, _ = _data.kitti_case(21)
    o = _ctx()
    try:
        o.set_surfels(*_data.surfels(m))
        ref = _run(o, pts, Ti, False)
        L = lib()
        assert L.lo_set_stage_timing(o.ctx, 1) == 0
        a = _run(o, pts, Ti, True)
        us, cnt = C.c_double(0.0), C.c_int(0)
        assert L.lo_stage_time(o.ctx, C.byref(us), C.byref(cnt)) == 0
        assert cnt.value == 1 and us.value > 0.0
        assert L.lo_set_stage_timing(o.ctx, 0) == 0
        _same(a, ref)
    finally:
        o.close()


def test_persistent_back_to_back_queue():
    """Scans queued on the stream with no host sync in between (lo_icp_optimize_async + lo_icp_export_pose per scan):
    every launch starts from counters the previous launch's last workgroup re-zeroed."""
    import torch
    from lidar_odometry_amd import lib
    cases = [_data.kitti_case(f) for f in (11, 13, 15, 17, 19, 21, 23, 25)]
    o = _ctx()
    try:
        o.set_surfels(*_data.surfels(cases[0][0]))
        want = []
        for (_, pts, Ti, _) in cases:
            ok, To, st = _run(o, pts, Ti, False)
            want.append((ok, To, st.num_iterations))
        o.set_persistent(True)
        L = lib()
        dev = [torch.from_numpy(np.ascontiguousarray(p, np.float32)).cuda() for (_, p, _, _) in cases]
        out = torch.zeros((3 * len(cases), 16), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        fp = C.POINTER(C.c_float)
        for rep in range(3):
            for i, (_, pts, Ti, _) in enumerate(cases):
                Tc = np.ascontiguousarray(Ti, np.float32)
                rc = L.lo_icp_optimize_async(o.ctx, C.c_void_p(dev[i].data_ptr()), pts.shape[0], Tc.ctypes.data_as(fp))
                assert rc == 0
                assert L.lo_icp_export_pose(o.ctx, C.c_void_p(out[rep * len(cases) + i].data_ptr())) == 0
        assert L.lo_sync(o.ctx) == 0
        got = out.cpu().numpy()
        for rep in range(3):
            for i, (ok, To, iters) in enumerate(want):
                rec = got[rep * len(cases) + i]
                assert int(rec[12]) == 0 and ok
                assert int(rec[13]) == iters
                np.testing.assert_array_equal(rec[:12], To)
    finally:
        o.close()


def test_persistent_city_map_bitwise():
    """The bench's workload class: the city-grid map (300 frames) and its scans."""
    dev = "cuda"
    for frame in (301, 311, 321):
        m, pts, Ti, _ = _data.city_case(frame, device=dev)
        o = _ctx()
        try:
            o.set_surfels(*_data.surfels(m))
            _same(_run(o, pts, Ti, True), _run(o, pts, Ti, False))
        finally:
            o.close()
