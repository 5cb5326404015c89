"""Parity on the bench's own headline workload: bench.py's KITTI-07-like city map after 660 frames (331 keyframes,
12.8k surfels, 120k L0 voxels) and its 20 measured scans with their perturbed initial poses -- the exact inputs the
`value` line times.  The GPU's per-iteration poses must stay within the north_star tolerance (1e-4 m / 1e-4 rad)
of the oracle restatement with equal iteration counts, status and alpha at every iteration; in reference-exact mode
every iteration's pose, alpha and correspondence count is bit-identical.  (The bench line repeats this comparison
in `cpu_baseline.parity` / `parity_exact` on every run; this makes it part of the GPU test tier.)"""
import numpy as np
import pytest

import bench
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def workload():
    wl = bench.build_kitti(0)
    m = oracle.VoxelMap(wl["voxel"], 3, 0.1, True)
    for w, s in wl["keyframes"]:
        m.update(w, s, wl["max_dist"], True)
    inits = [bench.pose12(T) for T in wl["inits"]]
    ref = []
    for pts, Ti in zip(wl["scans"], inits):
        ok, To, _, logs = oracle.icp_optimize(m, pts, Ti)
        ref.append({"ok": ok, "T": np.asarray(To if ok else Ti, np.float32), "logs": logs})
    return wl, inits, ref


def _gpu_results(wl, inits, exact: bool):
    from lidar_odometry_amd import AdaptiveMEstimatorConfig, ICPConfig, IterativeClosestPointOptimizer, MapGeometry
    from lidar_odometry_amd._lib import lib
    o = IterativeClosestPointOptimizer(ICPConfig(use_surfel_correspondence=True), AdaptiveMEstimatorConfig(),
                                       MapGeometry(voxel_size=wl["voxel"]),
                                       max_points=max(len(s) for s in wl["scans"]))   # as bench.py builds it
    try:
        assert lib().lo_map_set_from_voxelmap(o.ctx, wl["vm"].handle) == 0
        o.set_exact(exact)
        out = []
        for pts, Ti in zip(wl["scans"], inits):
            ok, To = o.optimize(None, pts, Ti)
            st = o.get_last_stats()
            out.append({"ok": bool(ok), "T": np.asarray(To, np.float32).reshape(12).copy(), "logs": st.iterations})
        return out
    finally:
        o.close()


def test_bench_workload_size(workload):
    wl, _, _ = workload
    assert len(wl["scans"]) == 20
    assert wl["vm"].surfel_count() > 10_000                     # 10^4-10^5 surfels


def test_bench_workload_default_parity(workload):
    wl, inits, ref = workload
    p = bench.parity_vs_oracle(_gpu_results(wl, inits, exact=False), ref)
    assert p["within_1e-4"], p
    assert p["status_equal"] == p["iteration_count_equal"] == p["alpha_every_iteration_equal"] == 20, p


def test_bench_workload_exact_bitwise(workload):
    wl, inits, ref = workload
    for g, c in zip(_gpu_results(wl, inits, exact=True), ref):
        assert g["ok"] == c["ok"]
        assert len(g["logs"]) == len(c["logs"])
        for a, b in zip(g["logs"], c["logs"]):
            np.testing.assert_array_equal(np.asarray(a["pose"], np.float32).view(np.uint32),
                                          np.asarray(b["pose"], np.float32).view(np.uint32))
            assert a["alpha"] == b["alpha"] and a["n_corr"] == b["n_corr"]
        np.testing.assert_array_equal(np.asarray(g["T"], np.float32).view(np.uint32),
                                      np.asarray(c["T"], np.float32).view(np.uint32))
