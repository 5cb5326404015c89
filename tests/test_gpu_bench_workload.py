"""Parity on the bench's own workloads -- the exact inputs the `value` lines time: KITTI-07-like city map after 660
frames (331 keyframes, 12.8k surfels, 120k L0 voxels) with its 20 measured scans (C2), the MID360-like rosette
sequence (C3, 20 scans) and the synthetic 1M-point patch scans (C5, 4 scans), each with its perturbed initial poses.
In reference-exact mode every iteration's pose, alpha and correspondence count is bit-identical to the oracle's on
all three; in the default (fp64 tree-sum) mode the KITTI workload stays within the north_star tolerance (1e-4 m /
1e-4 rad per iteration) with equal iteration counts, status and alpha at every iteration.  The default mode is not
required to pass on C3 / C5: an alpha near-tie there flips with the summation order (DESIGN.md "parity per config"),
which is why bench.py's auto mode reports exact mode as the value on those configs.  (The bench line repeats these
comparisons in `cpu_baseline.parity` / `parity_other` on every run; this makes them part of the GPU test tier.)"""
import numpy as np
import pytest

import bench
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["kitti", "mid360", "patch1m"])
def workload(request):
    wl = bench.WORKLOADS[request.param](0)
    wl["key"] = request.param
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
    if wl["key"] == "kitti":
        assert len(wl["scans"]) == 20
        assert wl["vm"].surfel_count() > 10_000                 # 10^4-10^5 surfels
    elif wl["key"] == "patch1m":
        assert len(wl["scans"]) == 4 and min(len(s) for s in wl["scans"]) == 1_000_000
    else:
        assert len(wl["scans"]) == 20


def test_bench_workload_default_parity(workload):
    wl, inits, ref = workload
    if wl["key"] != "kitti":
        pytest.skip("default mode is only required on C2; C3 / C5 report exact mode (see module docstring)")
    p = bench.parity_vs_oracle(_gpu_results(wl, inits, exact=False), ref)
    assert p["within_1e-4"], p
    assert p["status_equal"] == p["iteration_count_equal"] == p["alpha_every_iteration_equal"] == len(ref), p


def test_bench_workload_exact_bitwise(workload):
    wl, inits, ref = workload
    gpu = _gpu_results(wl, inits, exact=True)
    assert bench.parity_vs_oracle(gpu, ref)["within_1e-4"]
    for g, c in zip(gpu, ref):
        assert g["ok"] == c["ok"]
        assert len(g["logs"]) == len(c["logs"])
        for a, b in zip(g["logs"], c["logs"]):
            np.testing.assert_array_equal(np.asarray(a["pose"], np.float32).view(np.uint32),
                                          np.asarray(b["pose"], np.float32).view(np.uint32))
            assert a["alpha"] == b["alpha"] and a["n_corr"] == b["n_corr"]
        np.testing.assert_array_equal(np.asarray(g["T"], np.float32).view(np.uint32),
                                      np.asarray(c["T"], np.float32).view(np.uint32))
