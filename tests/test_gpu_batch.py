"""GPU tests of the scan-parallel batch (lo_batch_*): B independent contexts advanced in lockstep.

Bar: every job's result is bit-identical to the same context running lo_icp_optimize alone on the same input
(same kernels, same per-job fixed-order reductions), and within the north-star tolerance of the CPU oracle.
Covers heterogeneous jobs (different maps, voxel sizes, scan sizes), insufficient / empty jobs, the cached
parameter path (repeat call), a re-pointed scan, and the argument checks.
"""
import numpy as np
import pytest

import oracle
from tests import _data

pytestmark = pytest.mark.gpu

TOL_T = 1e-4
TOL_R = 1e-4


def _ctx(m, voxel=0.5, max_points=1 << 16, exact=False):
    """A context for a batch job; the fast mode unless exact (the lockstep kernels' own tests -- the library default is
    reference-exact, whose batch form test_batch_exact_* covers)."""
    from lidar_odometry_amd import IterativeClosestPointOptimizer, MapGeometry
    o = IterativeClosestPointOptimizer(geometry=MapGeometry(voxel_size=voxel), max_points=max_points)
    o.set_exact(exact)
    if m is not None:
        k, n, c = _data.surfels(m)
        o.set_surfels(k, n, c)
    return o


def _jobs():
    """(map, voxel, points, T_init) for a heterogeneous batch."""
    jobs = []
    for f in (11, 13, 17, 21, 25, 31):
        m, pts, Ti, _ = _data.kitti_case(f)
        jobs.append((m, 0.5, pts, Ti))
    m, pts, Ti, _ = _data.mid360_case()
    jobs.append((m, 0.4, pts, Ti))
    m, pts, Ti, _ = _data.kitti_case(19, seed=5, sigma_t=0.3, sigma_r=0.03)     # large perturbation
    jobs.append((m, 0.5, pts, Ti))
    m, pts, Ti, _ = _data.kitti_case(11)
    jobs.append((m, 0.5, pts + np.float32(5000.0), Ti))                         # insufficient correspondences
    jobs.append((m, 0.5, pts[:0], Ti))                                          # empty cloud
    return jobs


def _singles(ctxs, jobs):
    out = []
    for o, (_, _, pts, Ti) in zip(ctxs, jobs):
        ok, To = o.optimize(None, pts, Ti)
        st = o.get_last_stats()
        out.append((ok, To.reshape(12).copy(), st.num_iterations, st.num_correspondences,
                    st.iterations[-1]["alpha"] if st.iterations else None))
    return out


def _check_equal(res, singles):
    for j, (r, s) in enumerate(zip(res, singles)):
        ok, To, it, nc, alpha = s
        assert r.success == ok, f"job {j}: success {r.success} vs single {ok}"
        np.testing.assert_array_equal(r.pose.reshape(12), To, err_msg=f"job {j}")
        if ok:
            assert r.iterations == it, f"job {j}: iterations {r.iterations} vs {it}"
            assert r.n_corr == nc, f"job {j}: n_corr {r.n_corr} vs {nc}"
            assert r.alpha == alpha, f"job {j}: alpha {r.alpha} vs {alpha}"


@pytest.fixture(params=["split", "one_wave", "split_solve"])
def pko_mode(request, monkeypatch):
    """The batch's launch shapes, forced: the two PKO forms (k_pko_tb<4, false> by default, <1, true> with
    LO_BATCH_ONE_WAVE=1) with the fused accumulate + solve, and the four-wave PKO with the separate k_solve_b1 (the
    default from 1024 jobs, LO_BATCH_FUSED_SOLVE=0)."""
    monkeypatch.setenv("LO_BATCH_ONE_WAVE", "1" if request.param == "one_wave" else "0")
    monkeypatch.setenv("LO_BATCH_FUSED_SOLVE", "0" if request.param == "split_solve" else "1")
    return request.param


def test_batch_heterogeneous_bitwise_vs_single(pko_mode):
    from lidar_odometry_amd import BatchOptimizer
    jobs = _jobs()
    ctxs = [_ctx(m, v) for (m, v, _, _) in jobs]
    try:
        singles = _singles(ctxs, jobs)
        b = BatchOptimizer(ctxs)
        try:
            res = b.optimize(None, [j[2] for j in jobs], [j[3] for j in jobs])
            _check_equal(res, singles)
            assert [r.success for r in res[-2:]] == [False, False]
            np.testing.assert_array_equal(res[-1].pose.reshape(12), jobs[-1][3])   # T_out = T_init on failure
            # same inputs again: the cached KParams path gives the same bits
            res2 = b.optimize(None, [j[2] for j in jobs], [j[3] for j in jobs])
            for r, r2 in zip(res, res2):
                np.testing.assert_array_equal(r.pose, r2.pose)
            # the oracle agrees with every successful job within the north-star tolerance
            for j, (m, _, pts, Ti) in enumerate(jobs):
                if not res[j].success:
                    continue
                ok_o, To_o, it_o, _ = oracle.icp_optimize(m, pts, Ti)
                assert ok_o and it_o == res[j].iterations
                A = res[j].pose.astype(np.float64)
                B = np.asarray(To_o, np.float64).reshape(3, 4)
                assert np.linalg.norm(A[:, 3] - B[:, 3]) <= TOL_T
                assert _data.rot_angle(A[:, :3], B[:, :3]) <= TOL_R
        finally:
            b.close()
    finally:
        for o in ctxs:
            o.close()


def test_batch_exact_jobs_bitwise_vs_single(pko_mode):
    """Reference-exact contexts in a batch (every other job): each exact job equals its context's own exact
    lo_icp_optimize bit for bit (and so the oracle, tests/test_gpu_exact.py), each fast-mode job its fast single run,
    also when the batch runs twice.  The exact jobs of at most kExactMergeMax (8192) points run in lockstep
    (k_exact_scale_cb + k_exact_acc_b); the appended 11k-point exact job runs its context's own exact GN loop."""
    from lidar_odometry_amd import BatchOptimizer
    jobs = _jobs()
    m, pts, Ti, _ = _data.kitti_case(11)
    big = np.concatenate([pts, pts + np.float32(0.01), pts - np.float32(0.01)])
    assert len(big) > 8192
    jobs.append((m, 0.5, big, Ti))
    ctxs = [_ctx(m, v) for (m, v, _, _) in jobs]
    try:
        for k, o in enumerate(ctxs):
            o.set_exact(k % 2 == 0)
        singles = _singles(ctxs, jobs)
        b = BatchOptimizer(ctxs)
        try:
            for _ in range(2):
                res = b.optimize(None, [j[2] for j in jobs], [j[3] for j in jobs])
                _check_equal(res, singles)
        finally:
            b.close()
    finally:
        for o in ctxs:
            o.close()


def test_batch_only_exact_in_fresh_process():
    """A process whose first exact work is a batch: exact jobs of 4096 < n <= 8192 points launch
    k_exact_scale_cb with 80 KB of dynamic LDS, whose attribute batch_alloc now sets itself (before, only a single
    exact optimize did, and in one pytest process an earlier test always had).  Every job equals its context's own
    exact lo_icp_optimize bit for bit (tests/_batch_child.py, a child process so no earlier test has run)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    child = os.path.join(root, "tests", "_batch_child.py")
    r = subprocess.run(["timeout", "-k", "10", "110", sys.executable, child], cwd=root, capture_output=True, text=True)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert all(4096 < n <= 8192 for n in out["n"]), out
    assert all(out["equal"]), out


def test_batch_follows_update_config():
    """lo_update_config on a context that belongs to a batch (IterativeClosestPointOptimizer::update_config): the next
    batch uses the new parameters -- a new alpha grid (the PKO tables and candidate buffers are re-made) and a new
    correspondence gate -- and stays bit-identical to the contexts' single optimize; a changed max_iterations (fixed at
    lo_batch_create) is refused."""
    from lidar_odometry_amd import BatchOptimizer
    from lidar_odometry_amd.icp import AdaptiveMEstimatorConfig, ICPConfig
    jobs = _jobs()[:4]
    ctxs = [_ctx(m, v) for (m, v, _, _) in jobs]
    try:
        b = BatchOptimizer(ctxs)
        try:
            pts, Ts = [j[2] for j in jobs], [j[3] for j in jobs]
            _check_equal(b.optimize(None, pts, Ts), _singles(ctxs, jobs))
            ctxs[1].update_config(ICPConfig(max_correspondence_distance=0.5), AdaptiveMEstimatorConfig(num_alpha_segments=60))
            ctxs[2].update_config(ICPConfig(max_correspondence_distance=0.7))
            _check_equal(b.optimize(None, pts, Ts), _singles(ctxs, jobs))
            ctxs[3].update_config(ICPConfig(max_iterations=6))
            with pytest.raises(RuntimeError):
                b.optimize(None, pts, Ts)
        finally:
            b.close()
    finally:
        for o in ctxs:
            o.close()


@pytest.mark.parametrize("exact", [False, True], ids=["fast", "exact"])
def test_batch_many_jobs_and_repointed_scans(pko_mode, exact):
    """64 jobs (fewer PKO workgroups per job than a single scan gets), then every job re-pointed at another scan; in
    both modes (all-exact: the lockstep exact scale + sums of 64 jobs)."""
    from lidar_odometry_amd import BatchOptimizer
    frames = [11, 13, 15, 17, 19, 21, 23, 25]
    cases = [_data.kitti_case(f) for f in frames]
    m = cases[0][0]
    ctxs = [_ctx(m, exact=exact) for _ in range(64)]
    try:
        b = BatchOptimizer(ctxs)
        try:
            for shift in (0, 3):
                sel = [cases[(j + shift) % len(cases)] for j in range(64)]
                res = b.optimize(None, [c[1] for c in sel], [c[2] for c in sel])
                ref = {}
                for j, c in enumerate(sel[:len(cases)]):
                    ok, To = ctxs[j].optimize(None, c[1], c[2])
                    ref[j % len(cases)] = (ok, To.reshape(12).copy())
                for j, r in enumerate(res):
                    ok, To = ref[j % len(cases)]
                    assert r.success == ok
                    np.testing.assert_array_equal(r.pose.reshape(12), To, err_msg=f"job {j} shift {shift}")
        finally:
            b.close()
    finally:
        for o in ctxs:
            o.close()


def test_batch_argument_checks():
    from lidar_odometry_amd import BatchOptimizer, ICPConfig, IterativeClosestPointOptimizer
    a = _ctx(None, max_points=1024)
    kd = IterativeClosestPointOptimizer(config=ICPConfig(use_surfel_correspondence=False), max_points=1024)
    try:
        with pytest.raises(RuntimeError):
            BatchOptimizer([a, a])             # a context twice
        with pytest.raises(RuntimeError):
            BatchOptimizer([a, kd])            # KDTree-mode context
        b = BatchOptimizer([a])
        try:
            with pytest.raises(RuntimeError):
                b.result()                     # nothing in flight
            big = np.zeros((2048, 3), np.float32)
            with pytest.raises(RuntimeError):
                b.optimize(None, [big], [np.eye(3, 4, dtype=np.float32)])   # exceeds max_points
            res = b.optimize(None, [np.zeros((100, 3), np.float32)], [np.eye(3, 4, dtype=np.float32)])
            assert not res[0].success          # empty map: no correspondences
            a.set_exact(True)                  # an exact-mode job runs its own exact GN loop inside the batch
            res = b.optimize(None, [np.zeros((100, 3), np.float32)], [np.eye(3, 4, dtype=np.float32)])
            assert not res[0].success
            a.set_exact(False)
        finally:
            b.close()
    finally:
        a.close()
        kd.close()
