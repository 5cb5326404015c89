"""GPU tests of the scan pipeline (lo_set_pipeline): a scan's GN iterations from `main_iterations` on run on the
context's tail stream (behind a device-side wait for the main part, k_wait_seq), and the context stream waits on the
device (k_wait_final, submitted after the tail) only until the scan's result is final, so a converged scan's early-exit launches drain beside
the next scan (they test the context's "last final scan" word, not the DevState the next scan already owns).

Bar: bit-identical to the pipeline switched off -- pose, every iteration's log, status, iteration count, n_corr --
for scans that converge in 1-4 iterations, scans that run out of iterations, too few correspondences and empty
clouds; for scans queued back to back (lo_icp_optimize_async, records exported per scan); for every split of the
iterations over the two streams; and for map changes between pipelined scans (the change must see the final
result of the scan before it and be seen by the scan after it).
Reference loop: IterativeClosestPointOptimizer.cpp:281-449 (optimize runs until convergence / max_iterations).
"""
import ctypes as C

import numpy as np
import pytest

from tests import _data

pytestmark = pytest.mark.gpu


def _cases():
    cs = []
    for f in (11, 13, 17, 21, 25):
        m, pts, Ti, _ = _data.kitti_case(f)
        cs.append((m, pts, Ti))
    m, pts, Ti, _ = _data.kitti_case(19, seed=5, sigma_t=0.3, sigma_r=0.03)        # large perturbation: more iterations
    cs.append((m, pts, Ti))
    m, pts, Ti, _ = _data.kitti_case(11)
    cs.append((m, pts + np.float32(5000.0), Ti))                                   # too few correspondences
    cs.append((m, pts[:0], Ti))                                                    # empty cloud
    return cs


def _ctx(m, max_iterations=None):
    from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer
    cfg = ICPConfig()
    if max_iterations is not None:
        cfg.max_iterations = max_iterations
    o = IterativeClosestPointOptimizer(config=cfg, max_points=1 << 16)
    k, n, c = _data.surfels(m)
    o.set_surfels(k, n, c)
    return o


def _run(o, pts, Ti):
    ok, To = o.optimize(None, pts, Ti)
    st = o.get_last_stats()
    logs = [(np.asarray(L["pose"], np.float32).tobytes(), float(L["alpha"]), float(L["cost"]), int(L["n_corr"]))
            for L in st.iterations]
    return ok, np.asarray(To, np.float32).reshape(12).tobytes(), st.num_iterations, st.num_correspondences, logs


@pytest.mark.parametrize("main", [1, 2, 3])
def test_pipeline_sync_bitwise(main):
    cs = _cases()
    o = _ctx(cs[0][0])
    try:
        ref = []
        o.set_pipeline(False)
        for _, pts, Ti in cs:
            ref.append(_run(o, pts, Ti))
        o.set_pipeline(True, main)
        for rep in range(2):                                   # every case after every other
            for j, (_, pts, Ti) in enumerate(cs):
                got = _run(o, pts, Ti)
                assert got == ref[j], f"case {j} (main {main}, rep {rep})"
        iters = sorted({r[2] for r in ref})
        assert max(iters) >= 3, iters                          # some scan really ran iterations on the tail stream
    finally:
        o.close()


def test_pipeline_more_iterations():
    """max_iterations 6 (forced non-convergence would need a looser map; the large perturbation runs > 2)."""
    cs = _cases()
    o = _ctx(cs[0][0], max_iterations=6)
    try:
        o.set_pipeline(False)
        ref = [_run(o, pts, Ti) for _, pts, Ti in cs]
        o.set_pipeline(True, 2)
        got = [_run(o, pts, Ti) for _, pts, Ti in cs]
        assert got == ref
    finally:
        o.close()


def _queued(o, d_scans, inits, order):
    """Every scan of `order` enqueued back to back; each one's 16-float record exported on the context stream."""
    import torch
    L = o._L
    recs = torch.zeros(len(order), 16, dtype=torch.float32, device="cuda:0")
    for k, i in enumerate(order):
        T = np.ascontiguousarray(inits[i], np.float32)
        rc = L.lo_icp_optimize_async(o.ctx, C.c_void_p(d_scans[i].data_ptr()), d_scans[i].shape[0],
                                     T.ctypes.data_as(C.POINTER(C.c_float)))
        assert rc == 0, rc
        assert L.lo_icp_export_pose(o.ctx, C.c_void_p(recs[k].data_ptr())) == 0
    assert L.lo_sync(o.ctx) == 0
    return recs.cpu().numpy()


def test_pipeline_async_queue_bitwise():
    import torch
    cs = _cases()
    o = _ctx(cs[0][0])
    try:
        d_scans = [torch.from_numpy(np.ascontiguousarray(p, np.float32).reshape(-1, 3)).to("cuda:0") if len(p)
                   else torch.zeros(1, 3, dtype=torch.float32, device="cuda:0") for _, p, _ in cs]
        inits = [Ti for _, _, Ti in cs]
        rng = np.random.default_rng(3)
        order = [int(x) for x in rng.integers(0, len(cs) - 1, size=40)]   # no empty cloud here (n = 0 -> k_init)
        o.set_pipeline(False)
        ref = _queued(o, d_scans, inits, order)
        o.set_pipeline(True, 2)
        got = _queued(o, d_scans, inits, order)
        np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
        # the records equal the synchronous results
        o.set_pipeline(False)
        for k in (0, 7, 19, 39):
            i = order[k]
            ok, To = o.optimize(None, cs[i][1], cs[i][2])
            if ok:
                np.testing.assert_array_equal(got[k, :12], np.asarray(To, np.float32).reshape(12))
            assert int(got[k, 13]) == o.get_last_stats().num_iterations
    finally:
        o.close()


def test_pipeline_map_change_between_scans():
    """A surfel upload between two pipelined scans: the upload waits for the first scan's final result and the second
    scan sees the new map -- both equal to the unpipelined sequence."""
    cs = _cases()
    m2, pts2, Ti2, _ = _data.kitti_case(27, last_kf=30)
    o = _ctx(cs[0][0])
    try:
        def seq():
            k, n, c = _data.surfels(cs[0][0])
            o.set_surfels(k, n, c)
            a = _run(o, cs[5][1], cs[5][2])                    # the many-iteration scan first
            k2, n2, c2 = _data.surfels(m2)
            o.set_surfels(k2, n2, c2)
            b = _run(o, pts2, Ti2)
            o.set_surfels(k, n, c)
            d = _run(o, cs[1][1], cs[1][2])
            return a, b, d
        o.set_pipeline(False)
        ref = seq()
        o.set_pipeline(True, 1)
        assert seq() == ref
        o.set_pipeline(True, 2)
        assert seq() == ref
    finally:
        o.close()


def test_pipeline_args():
    cs = _cases()
    o = _ctx(cs[0][0])
    try:
        assert o._L.lo_set_pipeline(o.ctx, 1, -1) != 0
        assert o._L.lo_set_pipeline(None, 1, 2) != 0
        o.set_pipeline(True, 0)                                # keeps the split
    finally:
        o.close()


def test_pipeline_tail_insufficient_queued():
    """A scan that drops below min_correspondence_points at an iteration on the tail stream (main = 1): the tail
    launch's lead workgroup publishes the scan final while its siblings may still be in the PKO prefix, and the next
    scan starts on the same buffers.  Queued back to back among other scans, every record equals the pipeline-off run
    (the tail workgroups re-test the scan's state after the prefix, lo_pko_body.h)."""
    import torch
    from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer
    cs = _cases()[:6]
    m0 = cs[0][0]
    o = _ctx(m0)
    try:
        o.set_pipeline(False)
        # a scan whose correspondence count at some iteration k >= 1 falls below every earlier count: with
        # min_corr = min(earlier counts) it passes iterations < k and fails at k (on the tail stream for main = 1)
        pool = []
        for f in range(11, 33):
            for sig in (0.05, 0.3, 0.6):
                _, pts, Ti, _ = _data.kitti_case(f, seed=7, sigma_t=sig, sigma_r=sig / 10)
                o.optimize(None, pts, Ti)
                n = [int(L["n_corr"]) for L in o.get_last_stats().iterations]
                ks = [k for k in range(1, len(n)) if n[k] < min(n[:k])]
                if ks:
                    pool.append((pts, Ti, min(n[:ks[0]]), ks[0]))
    finally:
        o.close()
    if not pool:
        pytest.skip("no scan in the pool loses correspondences at a later iteration")
    pts0, Ti0, min_corr, k_fail = pool[0]
    cs = [(None, pts0, Ti0)] + cs
    j0 = 0
    cfg = ICPConfig(min_correspondence_points=min_corr)
    o = IterativeClosestPointOptimizer(config=cfg, max_points=1 << 16)
    try:
        k, n, c = _data.surfels(m0)
        o.set_surfels(k, n, c)
        d_scans = [torch.from_numpy(np.ascontiguousarray(p, np.float32).reshape(-1, 3)).to("cuda:0") for _, p, _ in cs]
        inits = [Ti for _, _, Ti in cs]
        order = [j0 if k % 2 == 0 else k % len(cs) for k in range(40)]
        o.set_pipeline(False)
        ref = _queued(o, d_scans, inits, order)
        assert int(ref[0, 12]) == 1 and int(ref[0, 13]) == k_fail     # LO_INSUFFICIENT at iteration k_fail
        o.set_pipeline(True, max(1, k_fail))                  # the failing iteration runs on the tail stream
        for rep in range(3):
            got = _queued(o, d_scans, inits, order)
            np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32), err_msg=f"rep {rep}")
    finally:
        o.close()


def test_pipeline_forced_timeout_is_deterministic(monkeypatch):
    """The timeout path on demand (LO_PIPE_FAIL_AT=3: the third pipelined scan's tail wait gives up at once, the rest
    wait normally): a synchronous call re-runs that scan on one stream, bit-identical to the pipeline switched off,
    the pipeline stays off from then on, and lo_pipeline_status counts one timeout and one re-run; an async queue
    flags exactly the forced scan's record LO_ERR_PIPELINE and keeps every other record bit-identical."""
    cs = _cases()[:6]
    monkeypatch.setenv("LO_PIPE", "1")
    monkeypatch.setenv("LO_PIPE_FAIL_AT", "3")
    o = _ctx(cs[0][0])
    try:
        o.set_pipeline(False)
        ref = [_run(o, pts, Ti) for _, pts, Ti in cs]
        o.set_pipeline(True, 2)
        got = [_run(o, pts, Ti) for _, pts, Ti in cs]
        st = (C.c_int * 4)()
        o._L.lo_pipeline_status(o.ctx, st)
        assert got == ref
        assert st[0] == 0 and st[2] == 1 and st[3] == 1, list(st)   # off after the timeout, 1 timeout, 1 re-run
    finally:
        o.close()
    import torch
    o = _ctx(cs[0][0])
    try:
        d_scans = [torch.from_numpy(np.ascontiguousarray(p, np.float32).reshape(-1, 3)).to("cuda:0") for _, p, _ in cs]
        inits = [Ti for _, _, Ti in cs]
        order = list(range(len(cs)))
        o.set_pipeline(False)
        ref_q = _queued(o, d_scans, inits, order)
        o.set_pipeline(True, 2)
        got_q = _queued(o, d_scans, inits, order)
        flagged = [k for k in range(len(order)) if int(got_q[k, 12]) == -5]
        # the six scans are all pipelined: the third one's wait was forced to time out; the scans queued behind it
        # may find the pipeline broken (flagged) -- never a silently different record
        assert 2 in flagged and min(flagged) == 2, (flagged, got_q[:, 12])
        for k in range(len(order)):
            if k not in flagged:
                np.testing.assert_array_equal(got_q[k].view(np.uint32), ref_q[k].view(np.uint32), err_msg=f"scan {k}")
    finally:
        o.close()


def test_pipeline_timeout_under_counter_collection():
    """The failure the device-side waits had: under `rocprofv3 --pmc` dispatches are serialised across queues, and a
    wait can run before the work it waits for.  Forced on (LO_PIPE=1) with a 20 ms bound, a timed-out wait marks its
    scan LO_ERR_PIPELINE and breaks the pipeline for good: queued records are either bit-identical to the pipeline-off
    run or flagged (never silently wrong), synchronous calls re-run the scan on one stream (bit-identical), and
    lo_pipeline_status reports it.  Without LO_PIPE the context starts with the pipeline off under counter collection."""
    import json
    import os
    import shutil
    import subprocess
    import sys
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        pytest.skip("rocprofv3 not installed")
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_pipe_child.py")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    for force in ("1", ""):
        env = dict(os.environ, LO_PIPE_WAIT_MS="20", TMPDIR="/tmp")
        env.pop("LO_PIPE", None)
        if force:
            env["LO_PIPE"] = force
        outdir = os.path.join("/tmp", f"lo_pipe_pmc_{os.getpid()}_{force or 'auto'}")
        r = subprocess.run(["timeout", "-k", "10", "100", prof, "--pmc", "FETCH_SIZE", "-d", outdir, "-o", "run",
                            "--output-format", "csv", "--", sys.executable, child], cwd=root, env=env,
                           capture_output=True, text=True)
        shutil.rmtree(outdir, ignore_errors=True)
        assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        outs[force] = json.loads(line)
    forced, auto = outs["1"], outs[""]
    assert forced["sync_bitwise"] and forced["queued_bitwise_or_flagged"], forced
    assert forced["status_start"][0] == 1
    if forced["queued_flagged"] or forced["status_end"][2]:
        assert forced["status_end"][2] >= 1, forced                    # the timeout is reported
    assert auto["status_start"][0] == 0, auto                          # counter collection: pipeline off up front
    assert auto["sync_bitwise"] and auto["queued_bitwise_or_flagged"] and auto["queued_flagged"] == 0, auto
    print("forced:", forced, "auto:", auto)
