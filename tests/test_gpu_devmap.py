"""Device-resident voxel map (include/lo_map.h lo_devmap_*, csrc/lo_devmap.hip) against the host
map (lo_voxelmap_*, the UpdateVoxelMap restatement pinned to unordered_dense's orders by tests/test_map_side.py):
after every keyframe the L0 container (order, fp32 centroids) and the surfels (L1 order, keys, normals, centroids,
planarity) are bit-identical, the counts agree, and the context table the device map patches answers every lookup
exactly as a full upload of the host map -- across keyframes that insert, refit, lose, planarity-erase and prune,
and across ApplyTransformAndRehash.
"""
import numpy as np
import pytest

from lidar_odometry_amd import synth

pytestmark = pytest.mark.gpu


def _ctx(mp=1 << 16):
    from lidar_odometry_amd import IterativeClosestPointOptimizer
    return IterativeClosestPointOptimizer(max_points=mp)


def _same_maps(vm, dm):
    h0 = vm.l0_cloud()
    k0, c0, pc0 = dm.l0()
    assert len(h0) == len(c0) == vm.l0_count()
    np.testing.assert_array_equal(c0.view(np.uint32), h0.view(np.uint32))
    n0, n1, ns = dm.counts()
    assert (n0, n1, ns) == (vm.l0_count(), vm.l1_count(), vm.surfel_count())
    for x, y in zip(dm.surfels(), vm.surfels()):
        np.testing.assert_array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32))


def _same_lookups(a, b, pts, poses):
    for T in poses:
        na, va, ra = a.find_correspondences(pts, T)
        nb, vb, rb = b.find_correspondences(pts, T)
        assert na == nb
        np.testing.assert_array_equal(va, vb)
        np.testing.assert_array_equal(ra, rb)


@pytest.mark.parametrize("radius", [60.0, 120.0])
def test_devmap_matches_host_map(radius):
    from lidar_odometry_amd import lib
    from lidar_odometry_amd.voxelmap import DeviceVoxelMap, VoxelMap, voxel_filter
    seq = synth.KittiLikeSequence(seed=7, n_frames=44)
    vm = VoxelMap(0.5, 3, 0.1, True)
    A, B = _ctx(), _ctx()
    dm = DeviceVoxelMap(A, 0.5, 3, 0.1, max_l0=1 << 18, max_points=1 << 16)
    try:
        for k in range(0, 43, 2):
            T = seq.poses[k]
            w = synth.transform(T, voxel_filter(seq.scan(k), 0.5, 8))
            vm.update(w, T[:3, 3], radius, True)
            dm.update(w, T[:3, 3], radius, True)
            _same_maps(vm, dm)
            if k % 8 == 0:
                assert lib().lo_map_set_from_voxelmap(B.ctx, vm.handle) == 0
                f = k + 1
                scan = voxel_filter(seq.scan(f), 0.5, 8)
                rng = np.random.default_rng(k)
                poses = [seq.poses[f][:3].astype(np.float32).reshape(12)] + \
                        [synth.perturb(seq.poses[f], rng, 0.3, 0.03)[:3].astype(np.float32).reshape(12)]
                _same_lookups(A, B, scan, poses)
        # not a keyframe / empty cloud: nothing changes (UpdateVoxelMap returns before the prune)
        before = dm.counts()
        dm.update(w, seq.poses[0][:3, 3], 1.0, False)
        dm.update(w[:0], seq.poses[0][:3, 3], 1.0, True)
        assert dm.counts() == before
    finally:
        dm.close()
        A.close()
        B.close()


def test_devmap_planarity_erase_and_churn():
    """Noisy clutter (planarity failures erase voxels and their children) and a sensor jumping between two places
    with a small radius (whole regions pruned, L1 voxels emptied, tombstones renewing the indices)."""
    from lidar_odometry_amd.voxelmap import DeviceVoxelMap, VoxelMap
    sc = synth.patch_scene(n_patches=60, seed=3, extent=25.0)
    vm = VoxelMap(0.5, 3, 0.1, True)
    A = _ctx()
    dm = DeviceVoxelMap(A, 0.5, 3, 0.1, max_l0=1 << 17, max_points=1 << 16)
    try:
        rng = np.random.default_rng(4)
        for k in range(14):
            off = np.array([0.0 if k % 3 else 300.0, 40.0 * (k % 2), 0.0], np.float32)
            w = synth.sample_patches(sc, 20000, 50 + k, outlier_frac=0.3) + off
            w = w[rng.permutation(len(w))]
            vm.update(w, off.astype(np.float64), 35.0, True)
            dm.update(w, off.astype(np.float64), 35.0, True)
            _same_maps(vm, dm)
    finally:
        dm.close()
        A.close()


def test_devmap_apply_transform():
    """ApplyTransformAndRehash + RecomputeAllSurfels on the device, then updates continue: still the host map."""
    from lidar_odometry_amd import lib
    from lidar_odometry_amd.voxelmap import DeviceVoxelMap, VoxelMap, voxel_filter
    seq = synth.KittiLikeSequence(seed=7, n_frames=30)
    vm = VoxelMap(0.5, 3, 0.1, True)
    A, B = _ctx(), _ctx()
    dm = DeviceVoxelMap(A, 0.5, 3, 0.1, max_l0=1 << 18, max_points=1 << 16)
    try:
        for k in range(0, 21, 2):
            T = seq.poses[k]
            w = synth.transform(T, voxel_filter(seq.scan(k), 0.5, 8))
            vm.update(w, T[:3, 3], 120.0, True)
            dm.update(w, T[:3, 3], 120.0, True)
        C = synth.se3(synth.rot_z(0.05), [0.4, -0.3, 0.02])
        vm.apply_transform(C[:3].astype(np.float32))
        dm.apply_transform(C[:3].astype(np.float32))
        _same_maps(vm, dm)
        assert lib().lo_map_set_from_voxelmap(B.ctx, vm.handle) == 0
        f = 21
        scan = voxel_filter(seq.scan(f), 0.5, 8)
        Tf = (C @ seq.poses[f])[:3].astype(np.float32).reshape(12)
        _same_lookups(A, B, scan, [Tf])
        for k in (22, 24):
            T = C @ seq.poses[k]
            w = synth.transform(T, voxel_filter(seq.scan(k), 0.5, 8))
            vm.update(w, T[:3, 3], 120.0, True)
            dm.update(w, T[:3, 3], 120.0, True)
            _same_maps(vm, dm)
    finally:
        dm.close()
        A.close()
        B.close()


def test_devmap_device_points_and_table_reupload():
    """Points handed over as a device tensor; an unrelated upload into the context's table (lo_map_set_surfels)
    is noticed and the map refills the table from its L1 voxels at the next update."""
    import torch
    from lidar_odometry_amd import lib
    from lidar_odometry_amd.voxelmap import DeviceVoxelMap, VoxelMap, voxel_filter
    seq = synth.KittiLikeSequence(seed=9, n_frames=12)
    vm = VoxelMap(0.5, 3, 0.1, True)
    A, B = _ctx(), _ctx()
    dm = DeviceVoxelMap(A, 0.5, 3, 0.1, max_l0=1 << 17, max_points=1 << 16)
    try:
        for k in range(0, 11, 2):
            T = seq.poses[k]
            w = synth.transform(T, voxel_filter(seq.scan(k), 0.5, 8)).astype(np.float32)
            vm.update(w, T[:3, 3], 120.0, True)
            dm.update(torch.from_numpy(w).cuda(), T[:3, 3], 120.0, True)
            if k == 6:
                A.set_surfels(np.zeros((1, 3), np.int32), np.zeros((1, 3), np.float32), np.zeros((1, 3), np.float32))
        _same_maps(vm, dm)
        assert lib().lo_map_set_from_voxelmap(B.ctx, vm.handle) == 0
        scan = voxel_filter(seq.scan(11), 0.5, 8)
        _same_lookups(A, B, scan, [seq.poses[11][:3].astype(np.float32).reshape(12)])
    finally:
        dm.close()
        A.close()
        B.close()


def test_devmap_follows_context_stream_and_reports_overflow():
    """The map launches on its context's current stream: after lo_set_stream (which destroys the context's own
    stream) and back, updates still equal the host map.  An update beyond the map's capacity sets the error bits
    that lo_devmap_status reports as LO_ERR_CAPACITY, and so does lo_devmap_status_poll once the copy enqueued by
    lo_devmap_status_async has landed (the frame loop's per-keyframe check)."""
    import ctypes as C

    import torch

    from lidar_odometry_amd import lib
    from lidar_odometry_amd._lib import LO_ERR_CAPACITY
    from lidar_odometry_amd.voxelmap import DeviceVoxelMap, VoxelMap, voxel_filter
    seq = synth.KittiLikeSequence(seed=7, n_frames=12)
    vm = VoxelMap(0.5, 3, 0.1, True)
    A = _ctx()
    dm = DeviceVoxelMap(A, 0.5, 3, 0.1, max_l0=1 << 18, max_points=1 << 16)
    side = torch.cuda.Stream(device=0)
    try:
        for k in range(0, 11, 2):
            if k == 4:
                assert lib().lo_set_stream(A.ctx, C.c_void_p(side.cuda_stream)) == 0
            if k == 8:
                assert lib().lo_set_stream(A.ctx, None) == 0
            T = seq.poses[k]
            w = synth.transform(T, voxel_filter(seq.scan(k), 0.5, 8))
            vm.update(w, T[:3, 3], 120.0, True)
            dm.update(w, T[:3, 3], 120.0, True)
            _same_maps(vm, dm)
        assert dm.status() == 0
    finally:
        dm.close()
        A.close()
    B = _ctx()
    small = DeviceVoxelMap(B, 0.5, 3, 0.1, max_l0=64, max_points=1 << 16)
    try:
        w = synth.transform(seq.poses[0], voxel_filter(seq.scan(0), 0.5, 8))
        small.update(w, seq.poses[0][:3, 3], 120.0, True)
        L = lib()
        assert L.lo_devmap_status_poll(small._h) == 0           # nothing enqueued yet
        assert L.lo_devmap_status_async(small._h) == 0
        torch.cuda.synchronize()
        assert L.lo_sync(B.ctx) == 0
        assert L.lo_devmap_status_poll(small._h) == LO_ERR_CAPACITY
        assert L.lo_devmap_status_poll(small._h) == 0           # reported once per enqueued check
        assert small.status() == LO_ERR_CAPACITY
    finally:
        small.close()
        B.close()
