"""Frame loop (lo_odometry.cpp; Estimator::process_frame without loop closure / PGO) on the device path
against the same loop on the oracle primitives (oracle.odometry), on raw synthetic KITTI-like scans:
per-frame pose within 1e-4 m / 1e-4 rad, identical keyframe decisions; trajectory accuracy vs ground truth;
KITTI trajectory file round trip."""
import numpy as np
import pytest

import oracle
from tests import _data

pytestmark = pytest.mark.gpu

N_FRAMES = 24


@pytest.fixture(scope="module")
def runs():
    from lidar_odometry_amd import synth
    from lidar_odometry_amd.odometry import LidarOdometry
    # the vehicle starts from rest (the reference's identity velocity prior at frame 1 is then reasonable), so
    # every frame's 4 GN iterations converge and the two loops can be compared frame by frame
    seq = synth.KittiLikeSequence(seed=7, n_frames=N_FRAMES, ramp_s=2.0)
    raws = [seq.scan(k) for k in range(N_FRAMES)]
    T0 = seq.poses[0]
    od = LidarOdometry(initial_pose=T0)
    try:
        got, infos = [], []
        for r in raws:
            T, info = od.process(r)
            got.append(T.reshape(12).copy())
            infos.append(info)
        kf_count = od.keyframes
    finally:
        od.close()
    ref, kfs = oracle.odometry(raws, initial=T0)
    return np.stack(got), infos, kf_count, ref, kfs, seq


def test_odometry_matches_oracle_loop(runs):
    got, infos, kf_count, ref, kfs, _ = runs
    assert [i.keyframe for i in infos] == list(kfs)
    assert kf_count == sum(kfs) >= 3
    # Closed loop in the default (fp64-tree) mode: every keyframe map is built from the loop's own poses, so the
    # ~1e-6 per-frame ICP differences (sum order of H, g; see test_gpu_parity) feed back through the map and
    # compound across keyframes.  The north_star 1e-4 bar holds per GN iteration on identical inputs
    # (test_gpu_parity); here frame k's inputs already differ by the accumulated drift, so the bound is
    # 5e-4 m / 1e-4 rad over 24 frames (8 keyframes).  With the reference's own arithmetic order
    # (test_odometry_exact_mode_is_bitwise) the same loop is bit-identical to the oracle's.
    errs = []
    for k in range(N_FRAMES):
        A, B = got[k].reshape(3, 4).astype(np.float64), ref[k].reshape(3, 4).astype(np.float64)
        et = np.linalg.norm(A[:, 3] - B[:, 3])
        er = _data.rot_angle(A[:, :3], B[:, :3])
        errs.append(et)
        assert et <= 5e-4 and er <= 1e-4, f"frame {k}: dt {et:.2e} m dr {er:.2e} rad"
    assert max(errs[:4]) <= 1e-4                   # the first keyframes, before the drift compounds
    assert all(i.status == 0 for i in infos[1:])


def test_odometry_exact_mode_is_bitwise():
    """Reference-exact ICP (lo_odom_set_exact) in the frame loop: every frame's pose bit-identical to the oracle
    loop, so the keyframe maps built from them are identical too and nothing compounds (contrast the 5e-4 m drift
    bound above for the default fp64-reduction ICP)."""
    from lidar_odometry_amd import synth
    from lidar_odometry_amd.odometry import LidarOdometry
    seq = synth.KittiLikeSequence(seed=7, n_frames=N_FRAMES, ramp_s=2.0)
    raws = [seq.scan(k) for k in range(N_FRAMES)]
    T0 = seq.poses[0]
    od = LidarOdometry(initial_pose=T0, exact=True)
    try:
        out = [od.process(r) for r in raws]
    finally:
        od.close()
    ref, kfs = oracle.odometry(raws, initial=T0)
    assert [i.keyframe for _, i in out] == list(kfs)
    for k, (T, info) in enumerate(out):
        np.testing.assert_array_equal(np.asarray(T, np.float32).reshape(12).view(np.uint32),
                                      np.asarray(ref[k], np.float32).view(np.uint32), err_msg=f"frame {k}")


def test_odometry_tracks_ground_truth(runs):
    got, infos, _, _, _, seq = runs
    err = [np.linalg.norm(got[k].reshape(3, 4)[:, 3] - seq.poses[k][:3, 3]) for k in range(N_FRAMES)]
    assert max(err) < 0.05
    assert all(i.n_filtered > 1000 for i in infos)


def test_trajectory_file_roundtrip(runs, tmp_path):
    from lidar_odometry_amd import io
    got = runs[0]
    f = tmp_path / "traj.txt"
    io.save_trajectory_kitti(f, [g.reshape(3, 4) for g in got])
    back = io.load_trajectory_kitti(f)
    np.testing.assert_allclose(back[:, :3, :4].reshape(-1, 12), got, atol=2e-9 + 1e-9 * np.abs(got).max())


def test_empty_first_frame_never_starts_a_map():
    """The reference's first frame with an empty feature cloud creates no keyframe (Estimator.cpp:247-251) and
    every later frame returns at "No keyframe available" (:140-144): the pose stays at the initial pose."""
    from lidar_odometry_amd import synth
    from lidar_odometry_amd.odometry import LidarOdometry
    seq = synth.KittiLikeSequence(seed=7, n_frames=4, ramp_s=2.0)
    raws = [np.zeros((0, 3), np.float32)] + [seq.scan(k) for k in range(1, 4)]
    T0 = seq.poses[0]
    od = LidarOdometry(initial_pose=T0)
    try:
        out = [od.process(r) for r in raws]
        assert od.keyframes == 0
    finally:
        od.close()
    ref, kfs = oracle.odometry(raws, initial=T0)
    assert not any(kfs)
    for k, (T, info) in enumerate(out):
        assert info.status == 0 and not info.keyframe
        np.testing.assert_array_equal(T.reshape(12), ref[k])
        np.testing.assert_array_equal(T.reshape(12), np.asarray(T0, np.float32)[:3, :4].reshape(12))


def test_map_overflow_reported_at_next_frame(monkeypatch):
    """A keyframe whose device-map update overflows (LO_DEVMAP_MAX_L0 = 64 L0 voxels) aborts the update; the frame loop
    copies the error bits back behind every keyframe's update without a sync and reports LO_ERR_CAPACITY at the very
    next frame (previously only every 8th keyframe was checked)."""
    from lidar_odometry_amd import synth
    from lidar_odometry_amd.odometry import LidarOdometry
    monkeypatch.setenv("LO_DEVMAP_MAX_L0", "64")
    seq = synth.KittiLikeSequence(seed=7, n_frames=3)
    od = LidarOdometry(initial_pose=seq.poses[0])
    try:
        _, info = od.process(seq.scan(0))                 # the first keyframe: its update overflows on the device
        assert info.keyframe
        from lidar_odometry_amd._lib import LO_ERR_CAPACITY
        with pytest.raises(RuntimeError, match=f"error {LO_ERR_CAPACITY}"):
            od.process(seq.scan(1))
    finally:
        od.close()


def test_map_overflow_at_last_keyframe_reported_by_flush(monkeypatch):
    """An overflow at the run's final keyframe has no next frame to report it: lo_odom_flush waits for the update and
    returns LO_ERR_CAPACITY."""
    from lidar_odometry_amd import synth
    from lidar_odometry_amd.odometry import LidarOdometry
    from lidar_odometry_amd._lib import LO_ERR_CAPACITY
    monkeypatch.setenv("LO_DEVMAP_MAX_L0", "64")
    seq = synth.KittiLikeSequence(seed=7, n_frames=2)
    od = LidarOdometry(initial_pose=seq.poses[0])
    try:
        _, info = od.process(seq.scan(0))
        assert info.keyframe
        with pytest.raises(RuntimeError, match=f"error {LO_ERR_CAPACITY}"):
            od.flush()
    finally:
        od.close()
    monkeypatch.delenv("LO_DEVMAP_MAX_L0")
    od = LidarOdometry(initial_pose=seq.poses[0])
    try:
        od.process(seq.scan(0))
        od.flush()                                        # a map within capacity: no error
    finally:
        od.close()


def test_kdtree_frame_loop_device_map_matches_host_map(monkeypatch):
    """KDTree correspondences (use_surfel_correspondence = false): the frame loop on the device map -- the map update
    without surfel decisions (SetComputeSurfels(false), so no planarity erases) and RebuildKdTree as a device grid
    from the L0 centroids (lo_devmap_sync_points) -- gives the same poses, bit for bit, and the same keyframes as
    the same loop on the host map (LO_HOST_MAP=1: host VoxelMap + lo_map_set_points, kd visit order built on the
    host)."""
    from lidar_odometry_amd import synth
    from lidar_odometry_amd.odometry import LidarOdometry
    n = 16
    seq = synth.KittiLikeSequence(seed=7, n_frames=n, ramp_s=2.0)
    raws = [seq.scan(k) for k in range(n)]

    def run():
        od = LidarOdometry(initial_pose=seq.poses[0], use_surfel_correspondence=False)
        try:
            return [od.process(r) for r in raws], od.keyframes
        finally:
            od.close()
    dev, kf_dev = run()
    monkeypatch.setenv("LO_HOST_MAP", "1")
    host, kf_host = run()
    assert kf_dev == kf_host >= 3
    for k, ((Td, idv), (Th, ih)) in enumerate(zip(dev, host)):
        assert idv.keyframe == ih.keyframe and idv.status == ih.status, f"frame {k}"
        np.testing.assert_array_equal(np.asarray(Td, np.float32).view(np.uint32), np.asarray(Th, np.float32).view(np.uint32),
                                      err_msg=f"frame {k}")
    err = max(float(np.linalg.norm(np.asarray(T)[:3, 3] - seq.poses[k][:3, 3])) for k, (T, _) in enumerate(dev))
    assert err < 0.05
